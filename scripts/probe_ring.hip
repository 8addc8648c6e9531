// probe_ring.hip -- round-trip latency of a resident "ring" kernel (NOT
// product code; scripts/probe_ring.sh).  A persistent workgroup polls a
// request word in fine-grained (coherent) pinned host memory, reads the
// request's bytes from pinned host memory, writes a result back and bumps a
// completion word; the host posts requests one at a time and spins on the
// completion word.  Measures the per-request host-observed latency for a few
// request sizes, against a plain launch + hipStreamSynchronize of the same
// work.  Exit: a stop word or an s_memrealtime deadline (every wave reaches it).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

struct Ctl {
  uint32_t seq;    // host -> device: request number (0: none yet)
  uint32_t stop;   // host -> device
  uint32_t n;      // request bytes
  uint32_t pad0;
  uint64_t src;    // request bytes (pinned host)
  uint64_t pad1[5];
  uint32_t done;   // device -> host: blocks finished x request number
  uint32_t result;
  uint32_t exited;
  uint32_t pad2[13];
};

__device__ __forceinline__ uint32_t ld_sys(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(256) void ring_probe(Ctl* ctl, uint64_t deadline_ticks, int nb) {
  __shared__ uint32_t s_seq, s_n, s_sum;
  __shared__ uint64_t s_src;
  uint32_t last = 0;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    if (threadIdx.x == 0) {
      uint32_t q;
      for (;;) {
        q = ld_sys(&ctl->seq);
        if (q != last || ld_sys(&ctl->stop)) break;
        if (__builtin_amdgcn_s_memrealtime() - t0 > deadline_ticks) { q = 0xFFFFFFFFu; break; }
        __builtin_amdgcn_s_sleep(2);
      }
      s_seq = ld_sys(&ctl->stop) ? 0xFFFFFFFFu : q;
      s_n = ld_sys(&ctl->n);
      s_src = __hip_atomic_load(&ctl->src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      s_sum = 0;
    }
    __syncthreads();
    const uint32_t q = s_seq;
    if (q == 0xFFFFFFFFu) break;
    // the request: sum of its bytes, this block's share (16-B loads)
    const uint8_t* src = (const uint8_t*)s_src;
    const uint32_t n = s_n;
    uint32_t acc = 0;
    for (uint32_t o = (blockIdx.x * 256 + threadIdx.x) * 16; o < n; o += nb * 256 * 16) {
      uint4 v = *(const uint4*)(src + o);
      acc += v.x + v.y + v.z + v.w;
    }
    atomicAdd(&s_sum, acc);
    __syncthreads();
    if (threadIdx.x == 0) {
      __hip_atomic_fetch_add(&ctl->result, s_sum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_fetch_add(&ctl->done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    last = q;
    __syncthreads();
  }
  if (threadIdx.x == 0) __hip_atomic_fetch_add(&ctl->exited, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void once_probe(const uint8_t* src, uint32_t n, uint32_t* out, int nb) {
  __shared__ uint32_t s_sum;
  if (threadIdx.x == 0) s_sum = 0;
  __syncthreads();
  uint32_t acc = 0;
  for (uint32_t o = (blockIdx.x * 256 + threadIdx.x) * 16; o < n; o += nb * 256 * 16) {
    uint4 v = *(const uint4*)(src + o);
    acc += v.x + v.y + v.z + v.w;
  }
  atomicAdd(&s_sum, acc);
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
  const int nb = argc > 1 ? atoi(argv[1]) : 4;
  const unsigned flags = (argc > 2 && atoi(argv[2]) == 0) ? hipHostMallocDefault : hipHostMallocCoherent;
  Ctl* ctl;
  CK(hipHostMalloc((void**)&ctl, sizeof(Ctl), hipHostMallocCoherent));
  memset(ctl, 0, sizeof(Ctl));
  uint8_t* buf;
  const size_t cap = 1 << 20;
  CK(hipHostMalloc((void**)&buf, cap, flags));
  for (size_t i = 0; i < cap; ++i) buf[i] = (uint8_t)(i * 7 + 1);
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  // deadline: 2 s of s_memrealtime (100 MHz)
  hipLaunchKernelGGL(ring_probe, dim3(nb), dim3(256), 0, s, ctl, (uint64_t)200000000, nb);
  CK(hipGetLastError());
  const uint32_t sizes[] = {1500, 16384, 65536};
  uint32_t seq = 0;
  for (uint32_t n : sizes) {
    std::vector<double> ts;
    bool ok = true;
    for (int it = 0; it < 400; ++it) {
      // new content every request at the same address: a stale cached read shows as a wrong sum
      const uint8_t salt = (uint8_t)(it * 13 + 5);
      for (uint32_t i = 0; i < n; i += 64) buf[i] = salt;
      uint32_t want = 0;
      for (uint32_t i = 0; i < n; i += 4) want += (uint32_t)buf[i] | ((uint32_t)buf[i + 1] << 8) | ((uint32_t)buf[i + 2] << 16) | ((uint32_t)buf[i + 3] << 24);
      __atomic_store_n(&ctl->result, 0u, __ATOMIC_RELAXED);
      ctl->n = n;
      ctl->src = (uint64_t)(uintptr_t)buf;
      const uint32_t d0 = __atomic_load_n(&ctl->done, __ATOMIC_ACQUIRE);
      const double t0 = now_us();
      __atomic_store_n(&ctl->seq, ++seq, __ATOMIC_RELEASE);
      while (__atomic_load_n(&ctl->done, __ATOMIC_ACQUIRE) != d0 + (uint32_t)nb) {
        if (now_us() - t0 > 1e6) { fprintf(stderr, "timeout\n"); ctl->stop = 1; hipStreamSynchronize(s); return 2; }
      }
      ts.push_back(now_us() - t0);
      if (__atomic_load_n(&ctl->result, __ATOMIC_ACQUIRE) != want) ok = false;
    }
    std::sort(ts.begin(), ts.end());
    printf("{\"probe\": \"ring\", \"blocks\": %d, \"coherent\": %d, \"bytes\": %u, \"median_us\": %.2f, \"p10_us\": %.2f, \"p90_us\": %.2f, \"sums_ok\": %s}\n",
           nb, flags == hipHostMallocCoherent, n, ts[ts.size() / 2], ts[ts.size() / 10], ts[ts.size() * 9 / 10], ok ? "true" : "false");
  }
  __atomic_store_n(&ctl->stop, 1u, __ATOMIC_RELEASE);
  CK(hipStreamSynchronize(s));
  printf("{\"probe\": \"ring_exit\", \"exited_blocks\": %u}\n", ctl->exited);
  // the same work as a launch + hipStreamSynchronize per request
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
