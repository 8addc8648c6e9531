// FETCH_SIZE calibration probes (NOT product code): known byte counts read
// with (a) a wide coalesced 16-B-per-lane stream and (b) gro_batch_kernel's
// pattern -- one 16-lane row per packet, 16-byte windows over the packet's
// 16-B-aligned span, packets 65,552 B apart at offset 16.
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ __launch_bounds__(256) void cal_wide(const uint4* __restrict__ src, size_t n16, uint32_t* __restrict__ out) {
  uint32_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = src[i];
    acc += v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ __launch_bounds__(256) void cal_rows(const uint8_t* __restrict__ arena, uint32_t npk, uint32_t stride,
                                                uint32_t off, uint32_t len, uint32_t* __restrict__ out) {
  const int r = threadIdx.x & 15;
  const uint32_t row = (blockIdx.x * blockDim.x + threadIdx.x) >> 4;
  const uint32_t nrows = (gridDim.x * blockDim.x) >> 4;
  uint32_t acc = 0;
  for (uint32_t p = row; p < npk; p += nrows) {
    const uint8_t* s = arena + (size_t)p * stride + off;
    const uintptr_t a0 = (uintptr_t)s & ~(uintptr_t)15, a1 = ((uintptr_t)s + len + 15) & ~(uintptr_t)15;
    for (uintptr_t a = a0 + 16 * r; a < a1; a += 256) {
      const uint4 v = *reinterpret_cast<const uint4*>(a);
      acc += v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

extern "C" int cal_wide_launch(const void* src, size_t bytes, void* out, void* stream) {
  hipLaunchKernelGGL(cal_wide, dim3(4096), dim3(256), 0, (hipStream_t)stream, (const uint4*)src, bytes / 16,
                     (uint32_t*)out);
  return (int)hipGetLastError();
}

extern "C" int cal_rows_launch(const void* arena, uint32_t npk, uint32_t stride, uint32_t off, uint32_t len, void* out,
                               void* stream) {
  hipLaunchKernelGGL(cal_rows, dim3(4096), dim3(256), 0, (hipStream_t)stream, (const uint8_t*)arena, npk, stride, off,
                     len, (uint32_t*)out);
  return (int)hipGetLastError();
}
