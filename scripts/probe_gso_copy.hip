// probe_gso_copy.hip -- the access-pattern ceiling of cfg4 (NOT product code;
// VERDICT r5 item 1, scripts/probe_gso_copy.py).  Moves exactly the bytes
// gso_lds_kernel moves for BASELINE configs[3] -- per 65,545-B read (10-B
// virtio header + 65,535-B TCP/IPv4 packet, hdrLen 40, gsoSize 1460) its 45
// segments [header | payload slice] into slots `stride` apart at `offset` --
// with 16-byte loads and stores per lane and nothing else: no header decode,
// no checksums, no field rewrites.  One 16-lane row per segment (its payload
// from readBuf[40 + 1460 i] shifted to the slot's phase with v_alignbyte,
// then the 40 header bytes over the slot's first chunks), 16 rows per block,
// blocks (read, segment group).
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

constexpr int kHdr = 40, kGso = 1460, kU = 6;

__device__ __forceinline__ uint32_t row_next(uint32_t v) {  // lane r <- lane r + 1 (row_ror:15)
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x12F, 0xF, 0xF, false);
}

__device__ __forceinline__ uint4 ld16(const uint8_t* p) {  // 4-byte aligned, non-temporal
  typedef unsigned int u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
  const u32x4a4 t = __builtin_nontemporal_load(reinterpret_cast<const u32x4a4*>(p));
  return make_uint4(t.x, t.y, t.z, t.w);
}

// bytes [0, len) of src to the 16-byte aligned dst by one 16-lane row (lane r):
// chunk k = the dword-aligned window k plus the next lane's first dword.
// Stores of partial chunks go byte by byte (as the product's edges do).
__device__ __forceinline__ void row_copy(const uint8_t* src, int len, uint8_t* dst, int r) {
  const int sb = (int)((uintptr_t)src & 3u);
  const uint8_t* a = src - sb;
  const int nk = (len + 15) >> 4;
  uint4 A[kU];
#pragma unroll
  for (int u = 0; u < kU; ++u) {
    const int k = r + 16 * u;
    A[u] = 16 * k < len + sb ? ld16(a + 16 * k) : make_uint4(0, 0, 0, 0);
  }
  uint32_t E = 0;
  if (r == 15 && 16 * (16 * kU) < len + sb) E = *reinterpret_cast<const uint32_t*>(a + 16 * 16 * kU);
#pragma unroll
  for (int u = 0; u < kU; ++u) {
    const int k = r + 16 * u;
    const uint32_t nxt = u + 1 < kU ? row_next(A[u + 1 < kU ? u + 1 : u].x) : E;
    const uint32_t same = row_next(A[u].x);
    const uint32_t n4 = r == 15 ? nxt : same;
    if (k < nk) {
      const uint4 v = make_uint4(__builtin_amdgcn_alignbyte(A[u].y, A[u].x, sb),
                                 __builtin_amdgcn_alignbyte(A[u].z, A[u].y, sb),
                                 __builtin_amdgcn_alignbyte(A[u].w, A[u].z, sb), __builtin_amdgcn_alignbyte(n4, A[u].w, sb));
      if (16 * k + 16 <= len) {
        *reinterpret_cast<uint4*>(dst + 16 * k) = v;
      } else {
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
        for (int b = 0; b < len - 16 * k; ++b) dst[16 * k + b] = (uint8_t)(w[b >> 2] >> (8 * (b & 3)));
      }
    }
  }
}

__global__ __launch_bounds__(256) void gso_copy_probe(const uint8_t* __restrict__ arena, uint64_t jpitch,
                                                       uint32_t jlen, uint8_t* __restrict__ out, uint32_t stride,
                                                       uint32_t offset, uint32_t max_segs) {
  const int lane = threadIdx.x & 63, r = lane & 15;
  const int i = (int)blockIdx.y * 16 + (int)(threadIdx.x >> 4);  // this row's segment
  const uint8_t* rb = arena + (uint64_t)blockIdx.x * jpitch + 10;
  const int plen = (int)jlen - 10;
  const int nseg = (plen - kHdr + kGso - 1) / kGso;
  if (i >= nseg || i >= (int)max_segs) return;
  const int seg = kHdr + min(kGso, plen - kHdr - i * kGso);
  uint8_t* dst = out + ((uint64_t)blockIdx.x * max_segs + (uint64_t)i) * stride + offset;
  row_copy(rb + i * kGso + 32, seg - 32, dst + 32, r);  // payload (and 8 bytes the header pass rewrites)
  row_copy(rb, kHdr, dst, r);                             // the header over chunks 0-2 (same lanes: ordered)
}

}  // namespace

extern "C" int probe_gso_copy(const uint8_t* arena, uint64_t jpitch, uint32_t jlen, uint32_t n_jobs, uint8_t* out,
                              uint32_t stride, uint32_t offset, uint32_t max_segs, void* stream) {
  const int plen = (int)jlen - 10;
  const int nseg = (plen - kHdr + kGso - 1) / kGso;
  if (((uintptr_t)out + offset) % 16 || stride % 16 || nseg <= 0) return -1;
  hipLaunchKernelGGL(gso_copy_probe, dim3(n_jobs, (nseg + 15) / 16), dim3(256), 0, (hipStream_t)stream, arena, jpitch,
                     jlen, out, stride, offset, max_segs);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
