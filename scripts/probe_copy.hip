// probe_copy.hip -- NOT product code.  Copy-pattern probe for the GSO split:
// nseg segments of `seg` bytes, source segment s at src + s*seg (arbitrary
// byte alignment), destination slot s at dst + s*stride (16-B aligned).
// One 16-lane row per segment, U 16-B chunks per lane.
//  mode 0: unaligned 16-B source loads (hardware realignment)
//  mode 1: aligned loads + DPP neighbour + funnel shift (registers)
#include <hip/hip_runtime.h>
#include <stdint.h>

__device__ __forceinline__ uint32_t row_next(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x12F, 0xF, 0xF, false);
}
__device__ __forceinline__ uint4 funnel_v(const uint4& a, const uint4& b, int s) {
  const bool q1 = (s & 4) != 0, q2 = (s & 8) != 0;
  const uint32_t f0 = q1 ? a.y : a.x, f1 = q1 ? a.z : a.y, f2 = q1 ? a.w : a.z, f3 = q1 ? b.x : a.w;
  const uint32_t f4 = q1 ? b.y : b.x, f5 = q1 ? b.z : b.y, f6 = q1 ? b.w : b.z;
  const uint32_t e0 = q2 ? f2 : f0, e1 = q2 ? f3 : f1, e2 = q2 ? f4 : f2, e3 = q2 ? f5 : f3, e4 = q2 ? f6 : f4;
  const int r = s & 3;
  return make_uint4(__builtin_amdgcn_alignbyte(e1, e0, r), __builtin_amdgcn_alignbyte(e2, e1, r),
                    __builtin_amdgcn_alignbyte(e3, e2, r), __builtin_amdgcn_alignbyte(e4, e3, r));
}

template <int U, int MODE>
__global__ __launch_bounds__(256) void probe_copy(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                  uint32_t nseg, uint32_t seg, uint32_t stride, uint32_t* sink) {
  const int lane = threadIdx.x & 63, r = lane & 15;
  const uint32_t sg = blockIdx.x * 16 + (threadIdx.x >> 4);
  if (sg >= nseg) return;
  const uint8_t* s0 = src + (uint64_t)sg * seg;
  uint8_t* d0 = dst + (uint64_t)sg * stride;
  const int nk = (int)(seg + 15) >> 4;
  uint32_t acc = 0;
  if (MODE == 0) {
    for (int k0 = 0; k0 < nk; k0 += 16 * U) {
      uint4 A[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = k0 + r + 16 * u;
        A[u] = make_uint4(0, 0, 0, 0);
        if (k < nk) __builtin_memcpy(&A[u], s0 + 16 * k, 16);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = k0 + r + 16 * u;
        if (k < nk) {
          *reinterpret_cast<uint4*>(d0 + 16 * k) = A[u];
          acc += A[u].x ^ A[u].w;
        }
      }
    }
  } else if (MODE == 2) {
    // dword-aligned 16-B loads (source rounded down to 4 B), byte shift by
    // alignbyte with the next lane's first dword
    const int s = (int)((uintptr_t)s0 & 3);
    const uint8_t* ab = s0 - s;
    const uint8_t* hi = s0 + seg;
    for (int k0 = 0; k0 < nk; k0 += 16 * U) {
      uint4 A[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint8_t* ca = ab + 16 * (k0 + r + 16 * u);
        A[u] = ca < hi ? *reinterpret_cast<const uint4*>(ca) : make_uint4(0, 0, 0, 0);
      }
      uint32_t E = 0;
      if (r == 15) {
        const uint8_t* ce = ab + 16 * (k0 + 16 * U);
        if (ce < hi) E = *reinterpret_cast<const uint32_t*>(ce);
      }
      uint32_t Rc = row_next(A[0].x);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = k0 + r + 16 * u;
        const uint32_t Rx = u + 1 < U ? row_next(A[u + 1 < U ? u + 1 : u].x) : E;
        const uint32_t nx = r == 15 ? Rx : Rc;
        Rc = Rx;
        if (k < nk) {
          const uint4 v = make_uint4(__builtin_amdgcn_alignbyte(A[u].y, A[u].x, s),
                                     __builtin_amdgcn_alignbyte(A[u].z, A[u].y, s),
                                     __builtin_amdgcn_alignbyte(A[u].w, A[u].z, s),
                                     __builtin_amdgcn_alignbyte(nx, A[u].w, s));
          *reinterpret_cast<uint4*>(d0 + 16 * k) = v;
          acc += v.x ^ v.w;
        }
      }
    }
  } else if (MODE == 3) {
    // aligned 16-byte loads, staged through LDS, read back at the byte phase
    // (ds_read_b128 at any byte address: unaligned LDS access mode)
    __shared__ uint4 stage[16][16 * U + 1];  // per row: its 16U+1 aligned chunks
    const int row = threadIdx.x >> 4;
    const int s = (int)((uintptr_t)s0 & 15);
    const uint8_t* ab = s0 - s;
    const uint8_t* hi = s0 + seg;
    uint8_t* lrow = reinterpret_cast<uint8_t*>(&stage[row][0]);
    for (int k0 = 0; k0 < nk; k0 += 16 * U) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint8_t* ca = ab + 16 * (k0 + r + 16 * u);
        stage[row][r + 16 * u] = ca < hi ? *reinterpret_cast<const uint4*>(ca) : make_uint4(0, 0, 0, 0);
      }
      if (r == 0) {
        const uint8_t* ce = ab + 16 * (k0 + 16 * U);
        stage[row][16 * U] = ce < hi ? *reinterpret_cast<const uint4*>(ce) : make_uint4(0, 0, 0, 0);
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes done
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = k0 + r + 16 * u;
        if (k < nk) {
          uint4 v;
          __builtin_memcpy(&v, lrow + 16 * (r + 16 * u) + s, 16);
          *reinterpret_cast<uint4*>(d0 + 16 * k) = v;
          acc += v.x ^ v.w;
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
  } else {
    const int s = (int)((uintptr_t)s0 & 15);
    const uint8_t* ab = s0 - s;
    const uint8_t* hi = s0 + seg;
    for (int k0 = 0; k0 < nk; k0 += 16 * U) {
      uint4 A[U], Rn[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint8_t* ca = ab + 16 * (k0 + r + 16 * u);
        A[u] = ca < hi ? *reinterpret_cast<const uint4*>(ca) : make_uint4(0, 0, 0, 0);
      }
      uint4 E = make_uint4(0, 0, 0, 0);
      if (r == 15) {
        const uint8_t* ce = ab + 16 * (k0 + 16 * U);
        if (ce < hi) E = *reinterpret_cast<const uint4*>(ce);
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        Rn[u] = make_uint4(row_next(A[u].x), row_next(A[u].y), row_next(A[u].z), row_next(A[u].w));
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = k0 + r + 16 * u;
        const uint4 B = r == 15 ? (u + 1 < U ? Rn[u + 1 < U ? u + 1 : u] : E) : Rn[u];
        if (k < nk) {
          const uint4 v = funnel_v(A[u], B, s);
          *reinterpret_cast<uint4*>(d0 + 16 * k) = v;
          acc += v.x ^ v.w;
        }
      }
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

extern "C" int probe_copy_launch(const void* src, void* dst, uint32_t nseg, uint32_t seg, uint32_t stride, int mode,
                                 void* sink, void* stream) {
  const dim3 grid((nseg + 15) / 16);
  if (mode == 3)
    hipLaunchKernelGGL((probe_copy<6, 3>), grid, dim3(256), 0, (hipStream_t)stream, (const uint8_t*)src,
                       (uint8_t*)dst, nseg, seg, stride, (uint32_t*)sink);
  else if (mode == 2)
    hipLaunchKernelGGL((probe_copy<6, 2>), grid, dim3(256), 0, (hipStream_t)stream, (const uint8_t*)src,
                       (uint8_t*)dst, nseg, seg, stride, (uint32_t*)sink);
  else if (mode == 0)
    hipLaunchKernelGGL((probe_copy<6, 0>), grid, dim3(256), 0, (hipStream_t)stream, (const uint8_t*)src,
                       (uint8_t*)dst, nseg, seg, stride, (uint32_t*)sink);
  else
    hipLaunchKernelGGL((probe_copy<6, 1>), grid, dim3(256), 0, (hipStream_t)stream, (const uint8_t*)src,
                       (uint8_t*)dst, nseg, seg, stride, (uint32_t*)sink);
  return (int)hipGetLastError();
}
