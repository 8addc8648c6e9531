// wgcs_copy.h -- device helpers for byte-stream copies between arbitrary
// source / destination alignments (GSO split and GRO coalesce kernels).
// Destination-aligned 16-byte chunks are assembled from aligned source loads
// with a cross-lane neighbour fetch and a uniform funnel shift, so every HBM
// load and every full-chunk store is a 16-byte global_load/store_dwordx4.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "wgcs_common.h"

namespace wgcs {

// All addresses stay pointers derived from kernel arguments (no integer round
// trips), so the compiler keeps them in the global address space and emits
// global_load/store (not flat_*, which forces full vmcnt+lgkmcnt waits).
//
// WGCS_RING_TU (ring_kernels.hip, the resident per-call ring): the request
// bytes change between requests at one address while the kernel stays
// resident, so every load of them is a system-scope one (relaxed atomic: sc0
// sc1, it misses the CU's L1 and the L2 -- no stale line of an earlier
// request; no ordering waits).  Elsewhere these are plain loads.
#ifdef WGCS_RING_TU
__device__ __forceinline__ uint4 ld16(const uint8_t* a) {
  const uint64_t* q = reinterpret_cast<const uint64_t*>(a);
  const uint64_t lo = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const uint64_t hi = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  return make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
}
__device__ __forceinline__ uint32_t ldg8(const uint8_t* a) {
  return __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
#define WGCS_LD_AUX(nt) 17  // buffer loads: sc0 sc1
#else
__device__ __forceinline__ uint4 ld16(const uint8_t* a) { return *reinterpret_cast<const uint4*>(a); }
__device__ __forceinline__ uint32_t ldg8(const uint8_t* a) { return *a; }
#define WGCS_LD_AUX(nt) ((nt) ? 2 : 0)
#endif
// Stores of results: plain everywhere.  (Round 6 measured system-scope
// write-through stores for the ring's results into host memory: 0.5 ms per
// 64-KiB read instead of 13 us; the ring releases its plain stores once at
// the end of a request instead.)
__device__ __forceinline__ void st128(uint8_t* d, const uint4& v) { *reinterpret_cast<uint4*>(d) = v; }
__device__ __forceinline__ void st64(uint8_t* d, uint32_t a, uint32_t b) {
  *reinterpret_cast<uint2*>(d) = make_uint2(a, b);
}
__device__ __forceinline__ void st32(uint8_t* d, uint32_t a) { *reinterpret_cast<uint32_t*>(d) = a; }
__device__ __forceinline__ void st16(uint8_t* d, uint16_t a) { *reinterpret_cast<uint16_t*>(d) = a; }
__device__ __forceinline__ void st8(uint8_t* d, uint8_t a) { *d = a; }

// Funnel: bytes [s, s+16) of the 32-byte concatenation a|b (s wave-uniform).
__device__ __forceinline__ uint4 funnel(const uint4& a, const uint4& b, int s) {
  const int r = s & 3;
  uint32_t d0 = a.x, d1 = a.y, d2 = a.z, d3 = a.w, d4 = b.x, d5 = b.y, d6 = b.z, d7 = b.w;
  uint32_t e0, e1, e2, e3, e4;
  switch (s >> 2) {
    case 0: e0 = d0; e1 = d1; e2 = d2; e3 = d3; e4 = d4; break;
    case 1: e0 = d1; e1 = d2; e2 = d3; e3 = d4; e4 = d5; break;
    case 2: e0 = d2; e1 = d3; e2 = d4; e3 = d5; e4 = d6; break;
    default: e0 = d3; e1 = d4; e2 = d5; e3 = d6; e4 = d7; break;
  }
  uint4 o;
  o.x = __builtin_amdgcn_alignbyte(e1, e0, r);
  o.y = __builtin_amdgcn_alignbyte(e2, e1, r);
  o.z = __builtin_amdgcn_alignbyte(e3, e2, r);
  o.w = __builtin_amdgcn_alignbyte(e4, e3, r);
  return o;
}

// Dynamic byte access goes through a 128-bit value (shifts and selects), never
// through an indexed private array: a runtime index into one becomes an alloca
// in scratch (or LDS) memory.
typedef unsigned __int128 u128;
__device__ __forceinline__ u128 to128(const uint4& v) {
  return ((u128)(((uint64_t)v.w << 32) | v.z) << 64) | (((uint64_t)v.y << 32) | v.x);
}
__device__ __forceinline__ uint4 from128(u128 t) {
  const uint64_t lo = (uint64_t)t, hi = (uint64_t)(t >> 64);
  return make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
}

__device__ __forceinline__ uint32_t chunk_byte(const uint4& v, int j) {
  return (uint32_t)(to128(v) >> (8 * j)) & 0xFFu;
}

__device__ __forceinline__ uint4 set_chunk_byte(const uint4& v, int j, uint32_t b) {
  const int sh = 8 * j;
  const u128 t = (to128(v) & ~((u128)0xFFu << sh)) | ((u128)(b & 0xFFu) << sh);
  return from128(t);
}

// Masked LE sum of the chunk's bytes at packet positions [lo, hi) (chunk at x0).
__device__ __forceinline__ uint64_t chunk_sum(const uint4& v, int x0, int lo, int hi) {
  if (x0 >= lo && x0 + 16 <= hi) return (uint64_t)v.x + v.y + v.z + v.w;
  const uint32_t m16 = byte_bits16(lo - x0, hi - x0);
  return (uint64_t)(v.x & expand_nibble(m16 & 0xF)) + (v.y & expand_nibble((m16 >> 4) & 0xF)) +
         (v.z & expand_nibble((m16 >> 8) & 0xF)) + (v.w & expand_nibble((m16 >> 12) & 0xF));
}

// Dword i (0..3) of a chunk: bit-field selects (v_bfi), no 128-bit shifts --
// and no ternaries on the components, which the compiler may turn into an
// indexed private array promoted to LDS.
__device__ __forceinline__ uint32_t dword_at(const uint4& v, int i) {
  const uint32_t m1 = 0u - ((uint32_t)i & 1u), m2 = 0u - (((uint32_t)i >> 1) & 1u);
  const uint32_t a = (v.y & m1) | (v.x & ~m1), b = (v.w & m1) | (v.z & ~m1);
  return (b & m2) | (a & ~m2);
}

// Store the part of a destination chunk that lies in [0, pkt_len): full
// chunks as one dwordx4; a partial chunk [lo, hi) as naturally aligned
// byte/short/dword/dwordx2 pieces (at most 7 stores instead of 16 bytes).
// Each piece's value is picked by dword selects: every piece lies inside one
// dword, or is the aligned dword pair (0,1) / (2,3).
//
// The two one-sided cases -- the chunk's first bytes [0, hi) (a packet's last
// chunk) and its last bytes [lo, 16) (the chunk a packet, or its payload,
// starts in) -- are by far the common partial chunks; each takes at most
// four stores whose values come from fixed dwords shifted as they are
// consumed (no per-piece dword selects).
__device__ __forceinline__ void store_lo(uint8_t* d, const uint4& v, int hi) {  // bytes [0, hi), 0 < hi < 16
  int p = 0;
  uint32_t a = v.x, b = v.y;  // the dwords at p and p + 4
  if (hi & 8) {
    st64(d, v.x, v.y);
    p = 8;
    a = v.z;
    b = v.w;
  }
  if (hi & 4) {
    st32(d + p, a);
    p += 4;
    a = b;
  }
  if (hi & 2) {
    st16(d + p, (uint16_t)a);
    p += 2;
    a >>= 16;
  }
  if (hi & 1) st8(d + p, (uint8_t)a);
}
__device__ __forceinline__ void store_hi(uint8_t* d, const uint4& v, int lo) {  // bytes [lo, 16), 0 < lo < 16
  const int n = 16 - lo;
  int e = 16;                 // end of the bytes still to store
  uint32_t a = v.w, b = v.z;  // the dwords ending at e and at e - 4
  if (n & 8) {
    st64(d + 8, v.z, v.w);
    e = 8;
    a = v.y;
    b = v.x;
  }
  if (n & 4) {
    st32(d + e - 4, a);
    e -= 4;
    a = b;
  }
  if (n & 2) {
    st16(d + e - 2, (uint16_t)(a >> 16));
    e -= 2;
    a <<= 16;
  }
  if (n & 1) st8(d + e - 1, (uint8_t)(a >> 24));
}

__device__ __forceinline__ void store_chunk(uint8_t* dchunk, const uint4& v, int x0, int pkt_len) {
  const int lo = -x0, hi = pkt_len - x0;  // the chunk's bytes [lo, hi) are stored
  if (lo <= 0 && hi >= 16) {
    st128(dchunk, v);
    return;
  }
  if (lo <= 0) {
    if (hi > 0) store_lo(dchunk, v, hi);
    return;
  }
  if (hi >= 16) {
    if (lo < 16) store_hi(dchunk, v, lo);
    return;
  }
  // both ends inside the chunk (a packet shorter than 16 bytes)
  int p = lo;
  if (p >= hi) return;
  auto b8 = [&](int q) { return (uint8_t)(dword_at(v, q >> 2) >> (8 * (q & 3))); };
  auto b16 = [&](int q) { return (uint16_t)(dword_at(v, q >> 2) >> (8 * (q & 2))); };  // q even
  if ((p & 1) && p < hi) { st8(dchunk + p, b8(p)); p += 1; }
  if ((p & 2) && p + 2 <= hi) { st16(dchunk + p, b16(p)); p += 2; }
  if ((p & 4) && p + 4 <= hi) { st32(dchunk + p, dword_at(v, p >> 2)); p += 4; }
  if (p + 8 <= hi) {  // p is 0 or 8 here
    if (p) st64(dchunk + p, v.z, v.w);
    else st64(dchunk + p, v.x, v.y);
    p += 8;
  }
  if (p + 4 <= hi) { st32(dchunk + p, dword_at(v, p >> 2)); p += 4; }
  if (p + 2 <= hi) { st16(dchunk + p, b16(p)); p += 2; }
  if (p < hi) st8(dchunk + p, b8(p));
}

template <bool SUM>
__device__ __forceinline__ void copy_tail(const uint4& a, const uint4& b, int s, int k, int k_end, int dalign,
                                          int pkt_len, int sum_lo, int pf, uint32_t pv, uint8_t* dbase,
                                          uint64_t& acc) {
  if (k < k_end) {
    uint4 v = funnel(a, b, s);
    const int x0 = 16 * k - dalign;
    if (pf >= 0) {
      const int j0 = pf - x0, j1 = pf + 1 - x0;
      if (j0 >= 0 && j0 < 16) v = set_chunk_byte(v, j0, pv >> 8);
      if (j1 >= 0 && j1 < 16) v = set_chunk_byte(v, j1, pv);
    }
    if (SUM) acc += chunk_sum(v, x0, sum_lo, pkt_len);
    store_chunk(dbase + 16 * k, v, x0, pkt_len);
  }
}

__device__ __forceinline__ void neighbour(const uint4& a, uint4& b, const uint8_t* ca, const uint8_t* src_lo,
                                          const uint8_t* src_hi, int lane) {
  b.x = __shfl_down(a.x, 1);
  b.y = __shfl_down(a.y, 1);
  b.z = __shfl_down(a.z, 1);
  b.w = __shfl_down(a.w, 1);
  if (lane == 63) {
    const uint8_t* cb = ca + 16;
    b = make_uint4(0, 0, 0, 0);
    if (cb < src_hi && cb + 16 > src_lo) b = ld16(cb);
  }
}

// Copy source positions -> destination chunks [k_begin, k_end) of a packet
// whose byte x lives at src0 + x (source bytes valid in [src_lo, src_hi)),
// destination chunk k covering packet positions [16k - dalign, +16).  Sums the
// bytes at positions [sum_lo, pkt_len) into acc; optionally overrides the two
// bytes at [pf, pf+2) with the big-endian value pv.  Two 64-chunk iterations
// are loaded before either is consumed (2 KiB in flight per wave).
template <bool SUM>
__device__ __forceinline__ void stream_copy(const uint8_t* src0, const uint8_t* src_lo, const uint8_t* src_hi,
                                            uint8_t* dbase, int dalign, int k_begin, int k_end, int pkt_len,
                                            int sum_lo, int pf, uint32_t pv, int lane, uint64_t& acc) {
  const uint8_t* w0 = src0 - dalign;  // source address of dest chunk 0's first byte
  const int s = (int)((uintptr_t)w0 & 15);
  const uint8_t* abase = w0 - s;
  for (int k0 = k_begin; k0 < k_end; k0 += 128) {
    const int ka = k0 + lane, kb = k0 + 64 + lane;
    const uint8_t* ca = abase + 16 * (long)ka;
    const uint8_t* cb = abase + 16 * (long)kb;
    uint4 a0 = make_uint4(0, 0, 0, 0), a1 = make_uint4(0, 0, 0, 0);
    if (ca < src_hi && ca + 16 > src_lo) a0 = ld16(ca);
    if (k0 + 64 < k_end && cb < src_hi && cb + 16 > src_lo) a1 = ld16(cb);
    uint4 b0, b1;
    neighbour(a0, b0, ca, src_lo, src_hi, lane);
    copy_tail<SUM>(a0, b0, s, ka, k_end, dalign, pkt_len, sum_lo, pf, pv, dbase, acc);
    if (k0 + 64 < k_end) {  // wave-uniform
      neighbour(a1, b1, cb, src_lo, src_hi, lane);
      copy_tail<SUM>(a1, b1, s, kb, k_end, dalign, pkt_len, sum_lo, pf, pv, dbase, acc);
    }
  }
}

// dst[0:n) = src[0:n), any alignments (no checksum).
__device__ __forceinline__ void copy_range(const uint8_t* src, int n, uint8_t* dst, int lane) {
  if (n <= 0) return;
  const int dalign = (int)((uintptr_t)dst & 15);
  const int nk = (n + dalign + 15) >> 4;
  uint64_t unused = 0;
  stream_copy<false>(src, src, src + n, dst - dalign, dalign, 0, nk, n, n, -1, 0, lane, unused);
}

}  // namespace wgcs
