// probe_ring.hip -- round-trip latency of a resident "ring" kernel (NOT
// product code; scripts/r6_ring.sh).  A persistent workgroup polls a request
// record, reads the request's bytes from pinned host memory (system-scope
// sc0 sc1 buffer loads: no L1 / L2 hit on a line an earlier request left),
// writes a result and a per-workgroup completion word back to pinned host
// memory; the host posts requests one at a time and spins on the completion
// words.  Variants (argv[2]):
//   0: request record in fine-grained pinned host memory (the GPU polls over PCIe)
//   1: request record in fine-grained device memory written by the host
//      through the BAR (the GPU polls its own HBM)
// against a plain launch + hipStreamSynchronize of the same work.  Exit: a
// stop word or an s_memrealtime deadline (every wave reaches it).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

struct Req {  // one 64-B record; seq stored last by the host
  uint32_t seq, stop, n, pad0;
  uint64_t src;
  uint32_t pad[10];
};
struct Done {  // device -> host: per workgroup {seq, result}, each on its own 64 B
  uint32_t seq, result, exited, pad[13];
};

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// loads: 0 = sc0 sc1 buffer loads; otherwise plain loads
__device__ __forceinline__ uint32_t sum_bytes(const uint8_t* src, uint32_t n, int nb, int loads) {
  uint32_t acc = 0;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(src), (short)0, (int)n, 0x00020000);
  for (uint32_t o = (blockIdx.x * 256 + threadIdx.x) * 16; o < n; o += nb * 256 * 16) {
    u32x4 v;
    if (loads == 0) v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)o, 0, 17);  // sc0 sc1
    else v = *(const u32x4*)(src + o);
    acc += v[0] + v[1] + v[2] + v[3];
  }
  return acc;
}

__global__ __launch_bounds__(256) void ring_probe(Req* rq, Done* dn, uint64_t deadline_ticks, int nb, int loads) {
  __shared__ uint32_t s_seq, s_n, s_sum;
  __shared__ uint64_t s_src;
  uint32_t last = 0;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    if (threadIdx.x < 64) {
      // the whole record in one wave instruction (lanes 0-3: 16 B each), system scope
      uint32_t q = 0, stop = 0, n = 0;
      uint64_t src = 0;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(rq, (short)0, 64, 0x00020000);
      for (;;) {
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(16 * (threadIdx.x & 3)), 0, 17);
        q = __builtin_amdgcn_readlane(v[0], 0);
        stop = __builtin_amdgcn_readlane(v[1], 0);
        n = __builtin_amdgcn_readlane(v[2], 0);
        src = ((uint64_t)__builtin_amdgcn_readlane(v[1], 1) << 32) | __builtin_amdgcn_readlane(v[0], 1);
        if (stop || q != last) break;
        if (__builtin_amdgcn_s_memrealtime() - t0 > deadline_ticks) { stop = 1; break; }
        __builtin_amdgcn_s_sleep(1);
      }
      if (threadIdx.x == 0) {
        s_seq = stop ? 0xFFFFFFFFu : q;
        s_n = n;
        s_src = src;
        s_sum = 0;
      }
    }
    // (a hand-written cache invalidate here, loads 1 / 2 in an earlier
    // version, left the GPU faulted on the box: removed; loads 1-3 = plain)
    __syncthreads();
    const uint32_t q = s_seq;
    if (q == 0xFFFFFFFFu) break;
    atomicAdd(&s_sum, sum_bytes((const uint8_t*)s_src, s_n, nb, loads));
    __syncthreads();
    if (threadIdx.x == 0) {
      // result then seq in one 8-B write-through (sc0 sc1) store
      typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
      const __amdgpu_buffer_rsrc_t ds = __builtin_amdgcn_make_buffer_rsrc(dn + blockIdx.x, (short)0, 64, 0x00020000);
      const u32x2 w = {q, s_sum};
      __builtin_amdgcn_raw_buffer_store_b64(w, ds, 0, 0, 17);
    }
    last = q;
  }
  if (threadIdx.x == 0) __hip_atomic_fetch_add(&dn[blockIdx.x].exited, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void once_probe(const uint8_t* src, uint32_t n, uint32_t* out, int nb) {
  __shared__ uint32_t s_sum;
  if (threadIdx.x == 0) s_sum = 0;
  __syncthreads();
  atomicAdd(&s_sum, sum_bytes(src, n, nb, 3));
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(out, s_sum);
}

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const int nb = argc > 1 ? atoi(argv[1]) : 1;
  const int variant = argc > 2 ? atoi(argv[2]) : 0;
  const int loads = argc > 3 ? atoi(argv[3]) : 0;
  Req* rq;
  if (variant == 1) {
    CK(hipExtMallocWithFlags((void**)&rq, 4096, hipDeviceMallocFinegrained));
  } else {
    CK(hipHostMalloc((void**)&rq, 4096, hipHostMallocCoherent));
  }
  Done* dn;
  CK(hipHostMalloc((void**)&dn, 64 * sizeof(Done), hipHostMallocCoherent));
  memset(dn, 0, 64 * sizeof(Done));
  volatile Req* vrq = rq;
  vrq->seq = 0;
  vrq->stop = 0;
  uint8_t* buf;
  const size_t cap = 1 << 20;
  CK(hipHostMalloc((void**)&buf, cap, hipHostMallocCoherent));
  for (size_t i = 0; i < cap; ++i) buf[i] = (uint8_t)(i * 7 + 1);
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipLaunchKernelGGL(ring_probe, dim3(nb), dim3(256), 0, s, rq, dn, (uint64_t)300000000, nb, loads);  // 3 s deadline
  CK(hipGetLastError());
  const uint32_t sizes[] = {1536, 16384, 65536};
  uint32_t seq = 0;
  for (uint32_t n : sizes) {
    std::vector<double> ts;
    int bad = 0;
    for (int it = 0; it < 400; ++it) {
      const uint8_t salt = (uint8_t)(it * 13 + 5);
      for (uint32_t i = 0; i < n; i += 64) buf[i] = salt;
      uint32_t want = 0;
      for (uint32_t i = 0; i < n; i += 4)
        want += (uint32_t)buf[i] | ((uint32_t)buf[i + 1] << 8) | ((uint32_t)buf[i + 2] << 16) | ((uint32_t)buf[i + 3] << 24);
      vrq->n = n;
      vrq->src = (uint64_t)(uintptr_t)buf;
      const double t0 = now_us();
      __atomic_thread_fence(__ATOMIC_SEQ_CST);
      vrq->seq = ++seq;
      __atomic_thread_fence(__ATOMIC_SEQ_CST);
      uint32_t total = 0;
      for (int b = 0; b < nb; ++b) {
        volatile Done* d = dn + b;
        while (d->seq != seq) {
          if (now_us() - t0 > 1e6) { fprintf(stderr, "timeout seq %u\n", seq); vrq->stop = 1; hipStreamSynchronize(s); return 2; }
        }
        total += d->result;
      }
      ts.push_back(now_us() - t0);
      if (total != want) ++bad;
    }
    std::sort(ts.begin(), ts.end());
    printf("{\"probe\": \"ring\", \"variant\": %d, \"loads\": %d, \"blocks\": %d, \"bytes\": %u, \"median_us\": %.2f, \"p10_us\": %.2f, \"p90_us\": %.2f, \"bad_sums\": %d}\n",
           variant, loads, nb, n, ts[ts.size() / 2], ts[ts.size() / 10], ts[ts.size() * 9 / 10], bad);
  }
  vrq->stop = 1;
  CK(hipStreamSynchronize(s));
  uint32_t ex = 0;
  for (int b = 0; b < nb; ++b) ex += dn[b].exited;
  printf("{\"probe\": \"ring_exit\", \"variant\": %d, \"exited_blocks\": %u}\n", variant, ex);
  uint32_t* dres;
  CK(hipMalloc(&dres, 4));
  for (uint32_t n : sizes) {
    std::vector<double> ts;
    for (int it = 0; it < 200; ++it) {
      const double t0 = now_us();
      hipLaunchKernelGGL(once_probe, dim3(nb), dim3(256), 0, s, buf, n, dres, nb);
      CK(hipStreamSynchronize(s));
      ts.push_back(now_us() - t0);
    }
    std::sort(ts.begin(), ts.end());
    printf("{\"probe\": \"launch_sync\", \"blocks\": %d, \"bytes\": %u, \"median_us\": %.2f}\n", nb, n, ts[ts.size() / 2]);
  }
  return 0;
}
