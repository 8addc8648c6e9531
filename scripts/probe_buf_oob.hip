// probe_buf_oob.hip -- NOT product code.  What a raw buffer dwordx4 / dword
// load returns when it straddles the descriptor's num_records (stride 0):
// lane l loads 16 bytes at byte offset 4*l from a buffer of n records whose
// bytes are 1..255; the host prints which dwords came back zero.
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void probe_buf_oob(const uint8_t* p, uint32_t n, uint4* out) {
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)n, 0x00020000);
  const int l = (int)threadIdx.x;
  auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, 4 * l, 0, 2);
  out[l] = make_uint4(v[0], v[1], v[2], v[3]);
}

extern "C" int probe_buf_oob_launch(const void* p, uint32_t n, void* out, void* stream) {
  hipLaunchKernelGGL(probe_buf_oob, dim3(1), dim3(16), 0, (hipStream_t)stream, (const uint8_t*)p, n, (uint4*)out);
  return (int)hipGetLastError();
}
