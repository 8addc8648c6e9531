// probe_strided.hip -- NOT product code.  The DRAM side of the outer-UDP
// batching kernels in isolation: one 16-lane row per 1452-B piece, 6 aligned
// 16-B loads (or stores) per lane, pieces `stride` bytes apart.  Read-only
// (XOR into a sink) or write-only (a constant pattern), so the time is the
// access pattern's alone.  1,024 x 128 pieces = 190 MB per launch, as
// udp_coalesce reads.
#include <hip/hip_runtime.h>
#include <stdint.h>

template <bool WRITE>
__global__ __launch_bounds__(256) void probe_strided(uint8_t* __restrict__ base, uint64_t stride, uint32_t npieces,
                                                     uint32_t piece, uint32_t* __restrict__ sink) {
  const int lane = threadIdx.x & 63, r = lane & 15;
  const uint32_t pc = blockIdx.x * 16 + (threadIdx.x >> 4);
  if (pc >= npieces) return;
  uint8_t* p = base + (uint64_t)pc * stride;
  const int nk = (int)(piece + 15) >> 4;
  if (WRITE) {
#pragma unroll
    for (int u = 0; u < 6; ++u) {
      const int k = r + 16 * u;
      if (k < nk) *reinterpret_cast<uint4*>(p + 16 * k) = make_uint4(pc, k, 0x5A5A5A5Au, u);
    }
    return;
  }
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  uint4 A[6];
#pragma unroll
  for (int u = 0; u < 6; ++u) {
    const int k = r + 16 * u;
    A[u] = make_uint4(0, 0, 0, 0);
    if (k < nk) {
      const u32x4 t = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p + 16 * k));
      A[u] = make_uint4(t.x, t.y, t.z, t.w);
    }
  }
  uint32_t acc = 0;
#pragma unroll
  for (int u = 0; u < 6; ++u) acc ^= A[u].x ^ A[u].y ^ A[u].z ^ A[u].w;
  if (acc == 0x12345678u) sink[0] = acc;
}

extern "C" int probe_strided_launch(void* base, uint64_t stride, uint32_t npieces, uint32_t piece, int write,
                                    void* sink, void* stream) {
  const dim3 grid((npieces + 15) / 16);
  if (write)
    hipLaunchKernelGGL((probe_strided<true>), grid, dim3(256), 0, (hipStream_t)stream, (uint8_t*)base, stride,
                       npieces, piece, (uint32_t*)sink);
  else
    hipLaunchKernelGGL((probe_strided<false>), grid, dim3(256), 0, (hipStream_t)stream, (uint8_t*)base, stride,
                       npieces, piece, (uint32_t*)sink);
  return (int)hipGetLastError();
}
