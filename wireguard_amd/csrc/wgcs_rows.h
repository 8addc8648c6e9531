// wgcs_rows.h -- 16-lane DPP row helpers shared by the row-mapped gfx950
// kernels (GSO split, outer-UDP message split/coalesce): cross-lane neighbour
// fetches inside a row, per-lane funnel shifts, dword-aligned 16-byte loads.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "wgcs_common.h"

namespace wgcs {

// DPP row_ror:15 -- lane r of each 16-lane row receives lane (r + 1) & 15.
__device__ __forceinline__ uint32_t row_next(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x12F, 0xF, 0xF, false);
}
__device__ __forceinline__ uint4 row_next4(const uint4& v) {
  return make_uint4(row_next(v.x), row_next(v.y), row_next(v.z), row_next(v.w));
}

// Bytes [s, s + 16) of the 32-byte concatenation a|b, s per lane in [0, 16).
__device__ __forceinline__ uint4 funnel_v(const uint4& a, const uint4& b, int s) {
  // two select stages on plain values (no private arrays: a select between
  // array elements becomes a dynamically indexed alloca -> scratch/LDS)
  const bool q1 = (s & 4) != 0, q2 = (s & 8) != 0;
  const uint32_t f0 = q1 ? a.y : a.x, f1 = q1 ? a.z : a.y, f2 = q1 ? a.w : a.z, f3 = q1 ? b.x : a.w;
  const uint32_t f4 = q1 ? b.y : b.x, f5 = q1 ? b.z : b.y, f6 = q1 ? b.w : b.z;
  const uint32_t e0 = q2 ? f2 : f0, e1 = q2 ? f3 : f1, e2 = q2 ? f4 : f2, e3 = q2 ? f5 : f3, e4 = q2 ? f6 : f4;
  const int r = s & 3;
  return make_uint4(__builtin_amdgcn_alignbyte(e1, e0, r), __builtin_amdgcn_alignbyte(e2, e1, r),
                    __builtin_amdgcn_alignbyte(e3, e2, r), __builtin_amdgcn_alignbyte(e4, e3, r));
}

// DPP row_shr:1 -- lane r of each row receives lane r - 1 (lane 0: zero).
__device__ __forceinline__ uint4 row_prev4(const uint4& v) {
  return make_uint4((uint32_t)__builtin_amdgcn_update_dpp(0, (int)v.x, 0x111, 0xF, 0xF, false),
                    (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v.y, 0x111, 0xF, 0xF, false),
                    (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v.z, 0x111, 0xF, 0xF, false),
                    (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v.w, 0x111, 0xF, 0xF, false));
}

// 16 bytes at the 4-byte aligned address p (global_load_dwordx4 tolerates
// dword alignment), optionally non-temporal.
template <bool NT>
__device__ __forceinline__ uint4 ld16_a4(const uint8_t* p) {
  typedef unsigned int u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
  const u32x4a4* q = reinterpret_cast<const u32x4a4*>(__builtin_assume_aligned(p, 4));
  const u32x4a4 t = NT ? __builtin_nontemporal_load(q) : *q;
  return make_uint4(t.x, t.y, t.z, t.w);
}

// The dword-aligned 16-byte window at p, of which only bytes below `hi` are
// needed: one load when the window cannot cross into a page past the last
// needed byte, else per-dword loads (each dword holds a needed byte or is skipped).
template <bool NT>
__device__ __forceinline__ uint4 ld_window(const uint8_t* p, const uint8_t* hi) {
  const uintptr_t a = (uintptr_t)p, h = (uintptr_t)hi;
  if (a + 16 <= h || ((a + 15) >> 12) == ((h - 1) >> 12)) return ld16_a4<NT>(p);
  const uint32_t* d = reinterpret_cast<const uint32_t*>(__builtin_assume_aligned(p, 4));
  uint4 v = make_uint4(0, 0, 0, 0);
  v.x = d[0];  // p < hi: the first dword holds a needed byte
  if (a + 4 < h) v.y = d[1];
  if (a + 8 < h) v.z = d[2];
  if (a + 12 < h) v.w = d[3];
  return v;
}

// Workgroup barrier that orders LDS only: waits for this wave's LDS (and
// scalar) operations, not for its outstanding global loads.  __syncthreads()'s
// workgroup fence also drains vmcnt, which would expose the latency of loads
// issued speculatively before the barrier.  The "memory" clobber keeps the
// compiler from moving memory accesses across it.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

}  // namespace wgcs
