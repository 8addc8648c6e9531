// wgcs_common.h -- device helpers shared by the gfx950 kernels.
//
// Arithmetic model (derived from /root/reference/tun/checksum.go:8-167 and
// verified in SURVEY.md §0 / tests/test_oracle.py): checksum(b, init) only
// depends on the plain integer S = sum(big-endian u16 words of b, odd tail
// zero-padded) + init, via  S == 0 ? 0 : 1 + (S - 1) mod 0xFFFF.  So any
// summation order, lane split or word width is bit-exact, provided
//  * all-zero input (S == 0 -> 0x0000) stays distinct from S ≡ 0 (-> 0xFFFF):
//    every fold below is an end-around-carry fold, which maps 0 -> 0 and
//    every positive value to [1, 0xFFFF];
//  * byte parity is handled: summing little-endian words at absolute
//    addresses gives S_le with S_be ≡ 256 * S_le (mod 0xFFFF) when the range
//    starts at an even absolute address and S_be ≡ S_le when it starts at an
//    odd one; 256 * x mod 0xFFFF for x in [0, 0xFFFF] is bswap16(x), and
//    256 * w mod (2^32 - 1) for a u32 w is rotl(w, 8).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace wgcs {

// 64-bit accumulator -> [0, 0xFFFF], end-around (0 iff x == 0).
__device__ __forceinline__ uint32_t fold64_16(uint64_t x) {
  uint64_t t = (x & 0xFFFFFFFFull) + (x >> 32);               // <= 2^33 - 2
  uint32_t t32 = (uint32_t)(t & 0xFFFFFFFFull) + (uint32_t)(t >> 32);  // no overflow
  uint32_t f = (t32 >> 16) + (t32 & 0xFFFFu);                // <= 0x1FFFE
  return (f >> 16) + (f & 0xFFFFu);                          // <= 0xFFFF
}

__device__ __forceinline__ uint32_t fold32_16(uint32_t x) {
  uint32_t f = (x >> 16) + (x & 0xFFFFu);
  f = (f >> 16) + (f & 0xFFFFu);
  return f;
}

__device__ __forceinline__ uint32_t bswap16(uint32_t x) {
  return ((x & 0xFFu) << 8) | ((x >> 8) & 0xFFu);
}

__device__ __forceinline__ uint32_t rotl8(uint32_t x) {
  return __builtin_amdgcn_alignbit(x, x, 24);  // (x << 8) | (x >> 24)
}

// Sum of a u32 over the 64 lanes of a wave (all lanes must be active).
// DPP quad_perm / half-row mirror / row mirror, then 4 readlanes.
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);   // quad [1,0,3,2]
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);   // quad [2,3,0,1]
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);  // row_half_mirror
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false);  // row_mirror
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 0) + (uint32_t)__builtin_amdgcn_readlane((int)v, 16) +
         (uint32_t)__builtin_amdgcn_readlane((int)v, 32) + (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
}

// Sum of a u32 over each 16-lane DPP row; every lane of the row gets its
// row's total (butterfly: quad xor 1, quad xor 2, half-row mirror, row mirror).
__device__ __forceinline__ uint32_t row16_sum_u32(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false);
  return v;
}

// Bit mask of bytes [lo, hi) inside a 16-byte chunk (lo/hi relative to the
// chunk, any int; clamped).
__device__ __forceinline__ uint32_t byte_bits16(int lo, int hi) {
  lo = lo < 0 ? 0 : (lo > 16 ? 16 : lo);
  hi = hi < 0 ? 0 : (hi > 16 ? 16 : hi);
  uint32_t h = (1u << hi) - 1u;
  uint32_t l = (1u << lo) - 1u;
  return h & ~l;
}

// acc + lo16(w) + hi16(w) in ONE instruction (v_dot2_u32_u16 with {1,1}):
// w ≡ lo16 + hi16 (mod 0xFFFF) and the sum is 0 iff w is 0, so a u32 of these
// is an exact, zero-preserving partial sum as long as it cannot overflow
// (< 2^15 dwords per accumulator).
__device__ __forceinline__ uint32_t add_halves(uint32_t acc, uint32_t w) {
  typedef unsigned short us2 __attribute__((ext_vector_type(2)));
  const us2 one = {1, 1};
  return __builtin_amdgcn_udot2(__builtin_bit_cast(us2, w), one, acc, false);
}

// Expand a 4-bit byte mask into a 32-bit byte mask (bit j -> byte j = 0xFF).
// t = one bit per byte; then v_perm_b32 with selector byte 0x0C (-> 0x00) or
// 0x0D (-> 0xFF), not t * 255, which the compiler emits as a quarter-rate
// 32-bit multiply (nib * 0x204081 fits the full-rate 24-bit one)
__device__ __forceinline__ uint32_t expand_nibble(uint32_t nib) {
  const uint32_t t = (nib * 0x00204081u) & 0x01010101u;
  return __builtin_amdgcn_perm(0u, 0u, t | 0x0C0C0C0Cu);
}

}  // namespace wgcs
