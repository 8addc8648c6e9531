// checksum_kernels.hip -- gfx950 (CDNA4) batch Internet-checksum kernels.
//
// Replaces, at batch granularity, the per-packet Go loops of
//   checksum()                     /root/reference/tun/checksum.go:152-167
//   checksumValid()                /root/reference/tun/gro.go:554-612
//   gsoSplit's L4 checksum step    /root/reference/tun/gro.go:1469-1488
//   gsoNoneChecksum()              /root/reference/tun/gro.go:1497-1517
//   IPv4 header checksum sites     /root/reference/tun/gro.go:1134-1138,1434-1436
//
// Design: the launched kernel is checksum_batch_kernel<MODE,
// G = 32, U = 4, NT>: one G-lane group (half a wave64) per packet, two packets
// per wave, an XCD-aware block order, one pass of the grid over batches of up
// to num_cu x 1,024 x 8 frames (grid-stride beyond that; round 5, wgcs_host.h).
// Each lane streams 16-byte chunks of its packet with non-temporal
// global_load_dwordx4 (U loads in flight per lane: 2 KiB per half-wave step,
// so one iteration covers a 1500-B frame), masks only the head / checksum
// field / tail chunks, and adds both u16 halves of every dword into a u32
// accumulator with one v_dot2 (re-folded each iteration).  Per-lane fold to 16
// bits, DPP row sums + one cross-row exchange, parity correction,
// pseudo-header / initial, final fold.  G = 16 (a DPP row) and G = 64 (a
// wave) are the tuning alternatives (WGCS_LANES_PER_PKT).  No LDS staging:
// each byte is read once and used once, and a 16-B register load per lane
// already moves 1 KiB per wave instruction -- measured, LDS-DMA staging ties
// register loads on this pattern (profiles/r1_probe_glds.jsonl) -- and no MFMA
// (a byte reduction, not a contraction).
#include <hip/hip_runtime.h>

#include "../../include/wgcsum.h"
#include "wgcs_common.h"
#include "wgcs_kernels.h"

namespace wgcs {

// Per-packet byte-set description, all positions relative to the packet start.
struct Ranges {
  int main_lo, main_hi;  // summed range (BE word pairing starts at main_lo)
  int addr_lo, addr_hi;  // pseudo-header address range (may be empty)
  int fld;               // 2 excluded bytes at [fld, fld+2) (or far away)
};

// Masked contribution of an edge chunk (head: addresses / gap / field; tail)
// at packet position `pos`.
// `addr`: wave-uniform, false when no packet of the wave has a separate
// address range (merged into the main range, below): the second mask is skipped.
__device__ __forceinline__ uint32_t edge_chunk(uint32_t acc, const uint4& v, int pos, const Ranges& r, bool rot_addr,
                                               bool addr) {
  const int f = r.fld - pos;
  uint32_t fb = 0;
  if (f >= -1 && f < 16) fb = ((3u << (f + 1)) >> 1) & 0xFFFFu;
  const uint32_t m16 = byte_bits16(r.main_lo - pos, r.main_hi - pos) & ~fb;
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) acc = add_halves(acc, w[k] & expand_nibble((m16 >> (4 * k)) & 0xFu));
  if (addr) {
    const uint32_t a16 = byte_bits16(r.addr_lo - pos, r.addr_hi - pos) & ~fb;  // the field is zeroed memory
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      uint32_t y = w[k] & expand_nibble((a16 >> (4 * k)) & 0xFu);
      if (rot_addr) y = rotl8(y);  // 256*y (mod 2^32-1): address pairing parity differs from the main range
      acc = add_halves(acc, y);
    }
  }
  return acc;
}

template <bool NT>
__device__ __forceinline__ uint4 ld_chunk(const uint4* p) {
  if (NT) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 t = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    return make_uint4(t.x, t.y, t.z, t.w);
  }
  return *p;
}

// Descriptor fields (include/wgcsum.h wgcs_pkt), unpacked from one dwordx4.
struct Desc {
  uint64_t off;
  int len, cs, co, proto, flags;
};
__device__ __forceinline__ Desc unpack(const uint4& d) {
  Desc r;
  r.off = (uint64_t)d.x | ((uint64_t)(d.y & 0xFFFFu) << 32);
  r.proto = (int)((d.y >> 16) & 0xFFu);
  r.flags = (int)(d.y >> 24);
  r.len = (int)d.z;
  r.cs = (int)(d.w & 0xFFFFu);
  r.co = (int)(d.w >> 16);
  return r;
}

// One packet per group of G lanes (G = 16: 4 packets per wave in flight; G = 64:
// one wavefront per packet).  The packet's 16-byte chunks are split into
// "edge" chunks (the first ones, up to the end of the address range / gap /
// checksum field, and a partial last one) that need byte masks, and interior
// chunks that are summed unmasked: lanes stream interior chunk
// c = c_lo + sub + G*(u + U*it), so one wave instruction reads 64/G
// contiguous 16*G-byte runs, and each lane owns at most a few edge chunks.
// The wave's first PPW consecutive descriptors through the scalar path (the
// address is wave-uniform, so these are s_load_dwordx4: no TA/TD round trip
// before the first frame load); each group picks its own.  Later descriptors
// are prefetched with vector loads, which the frame loads do not wait on.
template <int PPW>
__device__ __forceinline__ uint4 wave_desc(const uint4* __restrict__ pkts, uint32_t base, uint32_t n, int grp) {
  uint4 d[PPW];
#pragma unroll
  for (int k = 0; k < PPW; ++k) d[k] = (base + (uint32_t)k < n) ? pkts[base + k] : make_uint4(0, 0, 0, 0);
  uint4 r = d[0];
#pragma unroll
  for (int k = 1; k < PPW; ++k)
    if (grp == k) r = d[k];
  return r;
}

#ifndef WGCS_CS_ACC2
#define WGCS_CS_ACC2 1  // two accumulator chains per lane (0: one, round 5)
#endif
#ifndef WGCS_CS_MERGE
#define WGCS_CS_MERGE 1  // contiguous address + summed ranges as one (0: two masks per edge chunk, round 5)
#endif
#ifndef WGCS_CS_BLOCK
#define WGCS_CS_BLOCK 256  // threads per block (A/B builds: 512, 1024)
#endif
template <int MODE, int G, int U, bool NT>
__global__ __launch_bounds__(WGCS_CS_BLOCK) void checksum_batch_kernel(uint8_t* __restrict__ arena,
                                                             const uint4* __restrict__ pkts,
                                                             const uint64_t* __restrict__ initial,
                                                             uint32_t n, void* __restrict__ out,
                                                             int inplace, uint32_t amask, int xcd) {
  static_assert(G == 16 || G == 32 || G == 64, "group = DPP row, half wave or wave");
  constexpr int PPW = 64 / G;  // packets per wave per step
  const int lane = threadIdx.x & 63;
  const int grp = lane / G;
  const int sub = lane % G;
  // XCD-aware order (xcd != 0, grid a multiple of 8): blocks are dealt
  // round-robin over the 8 XCDs, so logical block (b % 8) * (grid / 8) + b / 8
  // gives each XCD one contiguous eighth of every grid-stride pass -- frames
  // that share a 128-B line at their boundary are fetched through one L2.
  uint32_t blk = blockIdx.x;
  if (xcd) blk = (blk & 7u) * (gridDim.x >> 3) + (blk >> 3);
  const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(blk * (blockDim.x >> 6) + (threadIdx.x >> 6)));
  const uint32_t step = gridDim.x * (blockDim.x >> 6) * PPW;
  uint4 dn = wave_desc<PPW>(pkts, wave * PPW, n, grp);
  for (uint32_t base = wave * PPW; base < n; base += step) {  // wave-uniform loop
    const uint32_t p = base + grp;
    const bool active = p < n;
    const Desc d = unpack(dn);
    if (p + step < n) dn = pkts[p + step];  // prefetch the next descriptor (vector: waited on by vmcnt only)
    uint8_t* pkt = arena + d.off;
    const int len = active ? d.len : 0;
    const int cs = d.cs;
    const bool v6 = (d.flags & WGCS_PKT_V6) != 0;
    const int fld16 = (cs + d.co) & 0xFFFF;  // u16 field position (gro.go:1391, :1503)
    Ranges r;
    r.main_lo = 0;
    r.main_hi = len;
    r.addr_lo = 0;
    r.addr_hi = 0;
    r.fld = -1000000;
    uint32_t pre = 0;
    uint64_t init = 0;
    if (MODE == WGCS_MODE_FOLD) {
      init = (initial && active) ? initial[p] : 0;
    } else if (MODE == WGCS_MODE_L4_FILL || MODE == WGCS_MODE_VALIDATE) {
      r.main_lo = min(cs, len);
      // the address slices are not bounded by len: a packet shorter than its
      // addresses has them read from the arena bytes after it, its Go slice's
      // spare capacity (gro.go:558-563, :1471-1477)
      r.addr_lo = v6 ? 8 : 12;
      r.addr_hi = v6 ? 40 : 20;
      if (MODE == WGCS_MODE_L4_FILL) r.fld = fld16;
      pre = (uint32_t)d.proto + ((uint32_t)(len - cs) & 0xFFFFu);  // {0, proto} + BE16(len - iphLen)
    } else if (MODE == WGCS_MODE_PARTIAL) {
      r.main_lo = min(cs, len);
      r.fld = fld16;
      if (r.fld + 1 < len) init = ((uint32_t)pkt[r.fld] << 8) | pkt[r.fld + 1];  // gro.go:1508
    } else {  // WGCS_MODE_IP4HDR
      r.main_hi = min(cs, len);
      r.fld = 10;
    }
#if WGCS_CS_MERGE
    // pseudo-header addresses that end where the summed range starts (iphLen
    // 20 / 40, the usual case) pair the same way: one range [addr_lo, len)
    // with one mask, and from there no gap to mask (round 6)
    if (r.addr_hi > r.addr_lo && r.addr_hi == r.main_lo && ((r.addr_lo ^ r.main_lo) & 1) == 0) {
      r.main_lo = r.addr_lo;
      r.addr_lo = r.addr_hi = 0;
    }
#endif
    const bool any_addr = __builtin_amdgcn_ballot_w64(r.addr_hi > r.addr_lo) != 0;  // wave-uniform
    const uintptr_t pbase = (uintptr_t)pkt;
    const bool rot_addr = (((pbase + r.addr_lo) ^ (pbase + r.main_lo)) & 1u) != 0;
    int lo_all = r.main_lo, hi_all = r.main_hi, hole_end = r.main_lo;
    if (r.addr_hi > r.addr_lo) {
      lo_all = min(lo_all, r.addr_lo);
      hi_all = max(hi_all, r.addr_hi);
      hole_end = max(hole_end, r.addr_hi);
    }
    if (r.fld + 2 > lo_all && r.fld < hi_all) hole_end = max(hole_end, r.fld + 2);
    // keep pointer provenance from the kernel argument (global address space):
    // an integer round trip would turn the loads into flat_load (full waits)
    // chunk grid origin: rounded down to `amask + 1` bytes (16, or a cache-line
    // multiple so each row's loads cover whole lines); chunks wholly before
    // lo_all are edge chunks with an empty mask and are not loaded
    const int rel0 = lo_all - (int)((pbase + (uintptr_t)lo_all) & amask);
    const int nch = hi_all > lo_all ? (hi_all - rel0 + 15) >> 4 : 0;
    int c_lo = min((hole_end - rel0 + 15) >> 4, nch);  // first unmasked chunk
    int c_hi = nch ? max((hi_all - rel0) >> 4, c_lo) : 0;  // end of unmasked chunks (none for an empty range:
                                                             // with a 128-B origin rel0 may lie 127 B below it)
    const int n_edge = c_lo + (nch - c_hi);
    const uint4* __restrict__ src = reinterpret_cast<const uint4*>(pkt + rel0);
    uint32_t acc = 0;
    // edge chunks: issued first, consumed after the first interior batch is in flight
    int ce = sub < c_lo ? sub : c_hi + (sub - c_lo);
    uint4 ve = (sub < n_edge && rel0 + 16 * ce + 16 > lo_all) ? ld_chunk<NT>(src + ce) : make_uint4(0, 0, 0, 0);
    bool edge_pending = true;
    // With a 128-byte chunk grid origin (amask 127) the interior iterations
    // start on a line boundary too (c_it: c_lo rounded down to 8 chunks; the
    // lanes below c_lo idle in the first one), so no 128-byte line is shared by
    // two iterations of a row -- with non-temporal loads such a line can be
    // evicted between them and read twice (round 5, profiles/r5_cfg5_traffic*)
    const int c_it = amask >= 127u ? (c_lo & ~7) : c_lo;
    for (int c0 = c_it + sub; c0 < c_hi || edge_pending; c0 += G * U) {
      uint4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int c = c0 + u * G;
        v[u] = (c < c_hi && c >= c_lo) ? ld_chunk<NT>(src + c) : make_uint4(0, 0, 0, 0);
      }
      if (edge_pending) {
        for (int e = sub;;) {  // rows with more than G edge chunks (long field offsets) loop
          if (e < n_edge) acc = edge_chunk(acc, ve, rel0 + 16 * ce, r, rot_addr, any_addr);
          e += G;
          if (e >= n_edge) break;
          ce = e < c_lo ? e : c_hi + (e - c_lo);
          ve = rel0 + 16 * ce + 16 > lo_all ? ld_chunk<NT>(src + ce) : make_uint4(0, 0, 0, 0);
        }
        edge_pending = false;
      }
      acc = (acc >> 16) + (acc & 0xFFFFu);  // keep the u32 partial sum far from overflow (huge packets)
#if WGCS_CS_ACC2
      // two independent v_dot2 chains (x,y / z,w), joined once per iteration:
      // half the serial dependency length of one chain of 4U (round 6)
      uint32_t acc2 = 0;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        acc = add_halves(acc, v[u].x);
        acc2 = add_halves(acc2, v[u].z);
        acc = add_halves(acc, v[u].y);
        acc2 = add_halves(acc2, v[u].w);
      }
      acc += acc2;  // < 2^17 + 16 U x 2^17: no overflow
#else
#pragma unroll
      for (int u = 0; u < U; ++u) {
        acc = add_halves(acc, v[u].x);
        acc = add_halves(acc, v[u].y);
        acc = add_halves(acc, v[u].z);
        acc = add_halves(acc, v[u].w);
      }
#endif
    }
    // all lanes converge here: per-lane fold, group sum, parity, pseudo/initial
    uint32_t s = fold32_16(acc);
    if (G == 16) {
      s = row16_sum_u32(s);
    } else if (G == 32) {  // two DPP rows of the half wave: row sums, then the partner row's (lane ^ 16)
      s = row16_sum_u32(s);
      s += (uint32_t)__shfl_xor((int)s, 16);
    } else {
      s = wave_sum_u32(s);
    }
    s = fold32_16(s);
    if (((pbase + (uintptr_t)r.main_lo) & 1u) == 0) s = bswap16(s);
    uint32_t t = fold32_16(s + pre + fold64_16(init));  // == the reference's checksum(...)
    // csum_start past the packet: the reference panics on pkt[iphLen:] (a
    // batch has no error channel: VALIDATE 0, L4_FILL 0 and no field write)
    const bool past = (MODE == WGCS_MODE_L4_FILL || MODE == WGCS_MODE_VALIDATE) && cs > len;
    if (sub == 0 && active) {
      if (MODE == WGCS_MODE_VALIDATE) {
        reinterpret_cast<uint8_t*>(out)[p] = (t == 0xFFFFu && !past) ? 1 : 0;  // ^checksum == 0
      } else if (MODE == WGCS_MODE_FOLD) {
        reinterpret_cast<uint16_t*>(out)[p] = (uint16_t)t;
      } else {
        const uint16_t c = past ? (uint16_t)0 : (uint16_t)~t;
        reinterpret_cast<uint16_t*>(out)[p] = c;
        if (inplace && !past && r.fld >= 0 && r.fld + 1 < len) {
          pkt[r.fld] = (uint8_t)(c >> 8);
          pkt[r.fld + 1] = (uint8_t)c;
        }
      }
    }
  }
}

template <int MODE>
static hipError_t launch_mode(uint8_t* arena, const wgcs_pkt* pkts, const uint64_t* init, uint32_t n, void* out,
                              int inplace, hipStream_t s, int num_cu, const LaunchTuning& t) {
  const int ppb = (64 / t.lanes_per_pkt) * (WGCS_CS_BLOCK / 64);  // packets per block per step
  long want = ((long)n + ppb - 1) / ppb;
  want = (want + 7) & ~7L;  // a multiple of 8 keeps the XCD-aware order (blocks past n exit at once)
  long cap = (long)num_cu * t.blocks_per_cu;
  cap = cap > 8 ? cap & ~7L : cap;
  const int grid = (int)(want < cap ? want : cap);
  const uint32_t amask = (uint32_t)(t.align >= 16 ? t.align : 16) - 1u;
  const int xcd = (t.xcd && grid % 8 == 0) ? 1 : 0;
  const uint4* d = reinterpret_cast<const uint4*>(pkts);
#define WGCS_LAUNCH(G, U)                                                                                    \
  do {                                                                                                      \
    if (t.nt)                                                                                               \
      hipLaunchKernelGGL((checksum_batch_kernel<MODE, G, U, true>), dim3(grid), dim3(WGCS_CS_BLOCK), 0, s, arena, d, \
                         init, n, out, inplace, amask, xcd);                                                \
    else                                                                                                    \
      hipLaunchKernelGGL((checksum_batch_kernel<MODE, G, U, false>), dim3(grid), dim3(WGCS_CS_BLOCK), 0, s, arena, d, \
                         init, n, out, inplace, amask, xcd);                                                \
  } while (0)
  if (t.lanes_per_pkt == 64) {
    if (t.unroll >= 4) WGCS_LAUNCH(64, 4);
    else WGCS_LAUNCH(64, 2);
  } else if (t.lanes_per_pkt == 32) {
    if (t.unroll >= 6) WGCS_LAUNCH(32, 6);
    else if (t.unroll >= 4) WGCS_LAUNCH(32, 4);
    else WGCS_LAUNCH(32, 3);
  } else {
    if (t.unroll >= 8) WGCS_LAUNCH(16, 8);
    else if (t.unroll >= 6) WGCS_LAUNCH(16, 6);
    else WGCS_LAUNCH(16, 4);
  }
#undef WGCS_LAUNCH
  return hipGetLastError();
}

hipError_t launch_checksum_batch(int mode, unsigned flags, uint8_t* arena, const wgcs_pkt* pkts,
                                 const uint64_t* init, uint32_t n, void* out, hipStream_t s, int num_cu,
                                 const LaunchTuning& tune) {
  if (n == 0) return hipSuccess;
  const int inplace = (flags & WGCS_F_INPLACE) ? 1 : 0;
  switch (mode) {
    case WGCS_MODE_FOLD:
      return launch_mode<WGCS_MODE_FOLD>(arena, pkts, init, n, out, inplace, s, num_cu, tune);
    case WGCS_MODE_L4_FILL:
      return launch_mode<WGCS_MODE_L4_FILL>(arena, pkts, init, n, out, inplace, s, num_cu, tune);
    case WGCS_MODE_VALIDATE:
      return launch_mode<WGCS_MODE_VALIDATE>(arena, pkts, init, n, out, inplace, s, num_cu, tune);
    case WGCS_MODE_PARTIAL:
      return launch_mode<WGCS_MODE_PARTIAL>(arena, pkts, init, n, out, inplace, s, num_cu, tune);
    case WGCS_MODE_IP4HDR:
      return launch_mode<WGCS_MODE_IP4HDR>(arena, pkts, init, n, out, inplace, s, num_cu, tune);
    default:
      return hipErrorInvalidValue;
  }
}

}  // namespace wgcs
