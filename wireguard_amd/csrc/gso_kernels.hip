// gso_kernels.hip -- gfx950 GSO split (TSO/USO super-packet -> MSS segments).
//
// Device-resident batch of the reference's Tun.Read path:
//   handleVirtioRead validation/dispatch   /root/reference/tun/tun.go:514-632
//   gsoSplit                               /root/reference/tun/gro.go:1373-1493
//   gsoNoneChecksum (GSO_NONE + NEEDS_CSUM) /root/reference/tun/gro.go:1497-1517
//
// Mapping (gso_rows_kernel): one 16-lane DPP row per OUTPUT segment (slot =
// job * max_segs + i), 64 segments per 1024-thread block, grid = (job,
// segment group).  Every row first issues its payload loads (dword-aligned
// 16-byte windows, U per lane in flight, which need only gsoSize) and its
// header-chunk loads (L2-resident, shared by the job); the decoder wave
// meanwhile validates the job and publishes its geometry through LDS
// (barrier 1), then computes the job-constant header sums (barrier 2) while
// every row
//   1. shifts each window to the destination's byte phase (alignbyte with the
//      next lane's first dword via DPP row_ror), sums the L4 bytes from the
//      same registers (v_dot2) and stores full global_store_dwordx4 chunks;
//   2. after barrier 2, computes the IPv4 and L4 checksums from the row sum
//      plus the job constants and the rewritten field values, rewrites the
//      header chunk and stores it last -- every output byte is written once.
// The barriers order LDS only (lds_barrier): loads stay in flight across them.
// Reference quirks reproduced bit-for-bit: IPv4 ID is
// id0 + 1 for every segment i >= 1; TCP seq uses a uint16 product
// gsoSize * uint16(i); FIN/PSH cleared on all but the last segment; no UDP
// 0 -> 0xFFFF substitution; ErrTooManySegments returns n = max_segs - 1.
#include <hip/hip_runtime.h>

#include "../../include/wgcsum.h"
#include "wgcs_common.h"
#include "wgcs_copy.h"
#include "wgcs_rows.h"
#include "wgcs_kernels.h"

namespace wgcs {

namespace {

constexpr int kMaxHdrLen = 240;  // header bytes held by the 16 lanes of a row (+ destination phase <= 15)

enum : int { GSO_NONE = 0, GSO_TCPV4 = 1, GSO_TCPV6 = 4, GSO_UDP_L4 = 5 };

__device__ __forceinline__ uint32_t u8at(const uint8_t* p) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)*p); }
__device__ __forceinline__ uint32_t be16at(const uint8_t* p) { return (u8at(p) << 8) | u8at(p + 1); }
__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }

// The first 256 bytes of a job ([virtio hdr | packet...]) held across the
// wave, one byte per lane per register: a single batch of byte loads instead
// of a chain of dependent scalar reads.  byte(k) for uniform k < 256.
struct HdrBytes {
  uint32_t r0, r1, r2, r3;
  int len;
  const uint8_t* base;
  __device__ __forceinline__ void load(const uint8_t* vb, int n, int lane) {
    base = vb;
    len = n;
    r0 = lane < n ? vb[lane] : 0u;
    r1 = lane + 64 < n ? vb[lane + 64] : 0u;
    r2 = lane + 128 < n ? vb[lane + 128] : 0u;
    r3 = lane + 192 < n ? vb[lane + 192] : 0u;
  }
  __device__ __forceinline__ uint32_t operator()(int k) const {  // k wave-uniform
    if (k >= 256) return u8at(base + k);
    const int l = k & 63;
    const uint32_t v = k < 64 ? r0 : (k < 128 ? r1 : (k < 192 ? r2 : r3));
    return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
  }
  // byte k (k per lane, 0 <= k < 256) fetched across lanes (ds_bpermute, no
  // memory access); all lanes must be active.
  __device__ __forceinline__ uint32_t lane_byte(int k) const {
    const int a = (k & 63) << 2;
    const uint32_t t0 = (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)r0);
    const uint32_t t1 = (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)r1);
    const uint32_t t2 = (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)r2);
    const uint32_t t3 = (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)r3);
    return k < 64 ? t0 : (k < 128 ? t1 : (k < 192 ? t2 : t3));
  }
  __device__ __forceinline__ uint32_t le16(int k) const { return (*this)(k) | ((*this)(k + 1) << 8); }
  __device__ __forceinline__ uint32_t be16(int k) const { return ((*this)(k) << 8) | (*this)(k + 1); }
  __device__ __forceinline__ uint32_t be32(int k) const { return (be16(k) << 16) | be16(k + 2); }
};

struct Job {
  int status;    // 0 or WGCS_ERR_*
  int nseg;      // segments to write (<= max_segs)
  int count;     // return value n
  int type, flags, ipv;
  int hdr_len, gso, cs, co, plen;
  int gen;       // 1: byte-granular general path (gso_general_row); 0: the row-streaming fast path
};

// Bytes of bufs[i][offset:] one gsoSplit segment writes (gro.go:1419-1488,
// oracle or_gso_split_need): the packet plus fixed-position header writes that
// may lie past it (IPv4 [2:12), IPv6 [4:6), seq / UDP length at csumStart+4,
// the flags byte on non-last segments, the checksum field; u16 positions).
__device__ __forceinline__ int split_need(const Job& j, int pkt_len, bool any_non_last) {
  const bool tcp = j.type != GSO_UDP_L4;
  int need = max(pkt_len, j.ipv == 4 ? 12 : 6);
  need = max(need, ((j.cs + 4) & 0xFFFF) + (tcp ? 4 : 2));
  if (tcp && any_non_last) need = max(need, ((j.cs + 13) & 0xFFFF) + 1);
  return max(need, ((j.cs + j.co) & 0xFFFF) + 2);
}

// Segment count / ErrTooManySegments (gro.go:1406-1410) + output room.
__device__ void count_segments(Job& j, uint32_t out_room, uint32_t max_segs) {
  const int plen = j.plen;
  long nseg = 0;
  if (j.hdr_len < plen) nseg = j.gso == 0 ? 0x7FFFFFFF : ((long)plen - j.hdr_len + j.gso - 1) / j.gso;
  if (nseg > 0) {  // segment 0 is the largest; Go panics on a bufs[0] slice shorter than what it writes
    const int first = j.hdr_len + min(j.gso, plen - j.hdr_len);
    const bool non_last = nseg > 1;
    if ((uint32_t)split_need(j, first, non_last) > out_room) { j.status = WGCS_ERR_OUT_OF_RANGE; return; }
  }
  if (nseg > (long)max_segs) {  // gro.go:1409-1410: all bufs written, n = i - 1
    j.nseg = (int)max_segs;
    j.count = (int)max_segs - 1;
    j.status = WGCS_ERR_TOO_MANY_SEGMENTS;
  } else {
    j.nseg = (int)nseg;
    j.count = (int)nseg;
  }
}

// gsoSplit's own bounds (gro.go:1387-1405 before the loop; :1419-1478 once it
// runs): an index the Go code would panic on is OUT_OF_RANGE.  Every position
// is the reference's uint16 sum.  Pseudo-header addresses past len(readBuf)
// (Go's spare capacity) are refused as well.  Then: does the
// job fit the row-streaming path (header <= 240 bytes, IP header at least the
// fixed IPv4 / IPv6 size, checksum field inside the header), or does it take
// the byte-granular general path?
__device__ bool split_bounds(Job& j) {
  const int plen = j.plen;
  const bool v4 = j.ipv == 4, tcp = j.type != GSO_UDP_L4;
  const int ca = (j.cs + j.co) & 0xFFFF;
  if (v4 && plen < 12) return false;                           // readBuf[10], [11]
  if (ca + 2 > plen) return false;                             // readBuf[checksumAt+1]
  if (tcp && ((j.cs + 4) & 0xFFFF) + 4 > plen) return false;   // Uint32(readBuf[csumStart+4:])
  if (j.hdr_len < plen) {                                      // the loop runs
    if (j.cs > j.hdr_len) return false;                        // pkt[csumStart:hdrLen]
    if (plen < (v4 ? 20 : 40)) return false;                   // address slices
  }
  j.gen = !(j.cs >= (v4 ? 20 : 40) && ca + 2 <= j.hdr_len && j.hdr_len <= kMaxHdrLen);
  return true;
}

// handleVirtioRead's checks (tun/tun.go:522-630), then gsoSplit's.
__device__ Job decode_job(const HdrBytes& hb, uint32_t len, uint32_t jflags, uint32_t out_room, uint32_t max_segs) {
  Job j = {};
  if (len < 10) { j.status = WGCS_ERR_SHORT_BUFFER; return j; }  // gro.go:84-86
  j.flags = (int)hb(0);
  j.type = (int)hb(1);
  j.hdr_len = (int)hb.le16(2);
  j.gso = (int)hb.le16(4);
  j.cs = (int)hb.le16(6);
  j.co = (int)hb.le16(8);
  const int plen = (int)len - 10;
  j.plen = plen;
  if (jflags & WGCS_GSO_JOB_RAW) {  // gsoSplit with the caller's header (gro.go:1373)
    j.ipv = (jflags & WGCS_GSO_JOB_V6) ? 6 : 4;
    if (j.type != GSO_TCPV4 && j.type != GSO_TCPV6) j.type = GSO_UDP_L4;  // protocol choice :1398-1405
    if (!split_bounds(j)) { j.status = WGCS_ERR_OUT_OF_RANGE; return j; }
    count_segments(j, out_room, max_segs);
    return j;
  }
  if (j.type == GSO_NONE) {  // tun/tun.go:532-556
    if (j.flags & 1) {
      const int at = (j.cs + j.co) & 0xFFFF;
      if (at + 2 > plen || j.cs > plen) { j.status = WGCS_ERR_OUT_OF_RANGE; return j; }
    }
    if ((uint32_t)plen > out_room) { j.status = WGCS_ERR_READ_OVERFLOW; return j; }
    j.nseg = 1;
    j.count = 1;
    return j;
  }
  if (j.type != GSO_TCPV4 && j.type != GSO_TCPV6 && j.type != GSO_UDP_L4) {
    j.status = WGCS_ERR_UNSUPPORTED_GSO;  // :564-568
    return j;
  }
  if (plen < 1) { j.status = WGCS_ERR_OUT_OF_RANGE; return j; }
  j.ipv = (int)(hb(10) >> 4);  // :570
  if (j.ipv == 4) {
    if (j.type != GSO_TCPV4 && j.type != GSO_UDP_L4) { j.status = WGCS_ERR_IP_GSO_MISMATCH; return j; }
  } else if (j.ipv == 6) {
    if (j.type != GSO_TCPV6 && j.type != GSO_UDP_L4) { j.status = WGCS_ERR_IP_GSO_MISMATCH; return j; }
  } else {
    j.status = WGCS_ERR_BAD_IP_VERSION;
    return j;
  }
  if (j.type == GSO_UDP_L4) {  // :597-614
    j.hdr_len = (j.cs + 8) & 0xFFFF;
  } else {
    const int at = (j.cs + 12) & 0xFFFF;
    if (plen <= at) { j.status = WGCS_ERR_PACKET_TOO_SHORT; return j; }
    const int th = (int)((hb(10 + at) >> 4) * 4);
    if (th < 20 || th > 60) { j.status = WGCS_ERR_TCP_HDR_LEN; return j; }
    j.hdr_len = (j.cs + th) & 0xFFFF;
  }
  if (plen < j.hdr_len) { j.status = WGCS_ERR_HDR_LEN; return j; }               // :615-621
  const int csum_at = (j.cs + j.co) & 0xFFFF;
  if (csum_at + 1 >= plen) { j.status = WGCS_ERR_CSUM_OFFSET; return j; }        // :622-630
  if (!split_bounds(j)) { j.status = WGCS_ERR_OUT_OF_RANGE; return j; }
  count_segments(j, out_room, max_segs);
  return j;
}

// ---------------------------------------------------------------------------
// General path: one 16-lane row per segment, byte-granular, for every header
// geometry the reference accepts that the row-streaming path does not take
// (IP headers shorter than 20 / 40 bytes, headers over 240 bytes, checksum
// fields outside the header or wrapped past 2^16).  Each output byte is the
// last value gsoSplit's write sequence leaves at its position
// (gro.go:1419-1488, in order: IP header copy, id / length / IPv4 checksum,
// L4 header copy, seq + flags or UDP length, payload, L4 checksum), computed
// from readBuf with its zeroed fields (:1388, :1393).  Three passes over the
// segment's chunks: IPv4 header sum, L4 sum, store.
struct GenSeg {
  const uint8_t* rb;
  int plen, cs, hdr_len, ca, s4, f13, i;
  int seg_start, pkt_len;
  bool v4, tcp, last;
  uint32_t id45;    // IPv4 bytes 4-5 after the id step (i > 0: BE16 + 1)
  uint32_t seq, ulen;
  uint32_t ipc;     // IPv4 header checksum (bytes 10-11)
};

// readBuf byte x after gsoSplit zeroed its IPv4 checksum and L4 checksum fields
__device__ __forceinline__ uint32_t rbz(const GenSeg& g, int x) {
  if ((g.v4 && (x == 10 || x == 11)) || x == g.ca || x == g.ca + 1) return 0u;
  return g.rb[x];
}

// byte x of the IP header after the id / length writes (x < csumStart = iphLen)
__device__ __forceinline__ uint32_t ip_stage(const GenSeg& g, int x) {
  if (g.v4) {
    if (x == 2) return ((uint32_t)g.pkt_len >> 8) & 0xFFu;
    if (x == 3) return (uint32_t)g.pkt_len & 0xFFu;
    if (x == 4) return g.id45 >> 8;
    if (x == 5) return g.id45 & 0xFFu;
  } else {
    const uint32_t pl = (uint32_t)(g.pkt_len - g.cs) & 0xFFFFu;  // :1439
    if (x == 4) return pl >> 8;
    if (x == 5) return pl & 0xFFu;
  }
  return rbz(g, x);
}

// byte x (< pkt_len) before the L4 checksum store
__device__ __forceinline__ uint32_t pre_csum(const GenSeg& g, int x) {
  if (x >= g.hdr_len) return rbz(g, g.seg_start + (x - g.hdr_len));  // payload (:1468)
  const int t = x - g.s4;
  if (g.tcp && t >= 0 && t < 4) return (g.seq >> (24 - 8 * t)) & 0xFFu;
  if (!g.tcp && t >= 0 && t < 2) return (g.ulen >> (8 - 8 * t)) & 0xFFu;
  uint32_t b;
  if (x >= g.cs) b = rbz(g, x);
  else if (g.v4 && x == 10) b = g.ipc >> 8;
  else if (g.v4 && x == 11) b = g.ipc & 0xFFu;
  else b = ip_stage(g, x);
  if (g.tcp && !g.last && x == g.f13) b &= ~0x09u;  // FIN|PSH (:1447-1459)
  return b;
}

// One segment on one 16-lane row (lane r): the three passes, then sizes[].
__device__ void gso_general_row(const uint8_t* rb, int plen, int type, int ipv, int hdr_len, int gso, int cs, int co,
                                int i, uint8_t* dst, int r, int32_t* size_out) {
  GenSeg g;
  g.rb = rb;
  g.plen = plen;
  g.cs = cs;
  g.hdr_len = hdr_len;
  g.v4 = ipv == 4;
  g.tcp = type != GSO_UDP_L4;
  g.ca = (cs + co) & 0xFFFF;
  g.s4 = (cs + 4) & 0xFFFF;
  g.f13 = (cs + 13) & 0xFFFF;
  g.i = i;
  g.seg_start = hdr_len + i * gso;
  const int seg_end = min(plen, g.seg_start + gso);
  const int seg_len = seg_end - g.seg_start;
  g.pkt_len = hdr_len + seg_len;
  g.last = seg_end == plen;
  g.seq = 0;
  if (g.tcp) {  // firstSeq from the zeroed readBuf (:1402), u16 product (:1445)
    const uint32_t s0 = (rbz(g, g.s4) << 24) | (rbz(g, g.s4 + 1) << 16) | (rbz(g, g.s4 + 2) << 8) | rbz(g, g.s4 + 3);
    g.seq = s0 + (uint32_t)(uint16_t)((uint16_t)gso * (uint16_t)i);
  }
  g.ulen = (uint32_t)(uint16_t)(seg_len + (hdr_len - cs));  // :1462-1465
  g.id45 = 0;
  if (g.v4) {  // pkt[4:6] after copy(pkt, readBuf[:iphLen]); bytes past iphLen are what bufs[i] held (:1427)
    const uint32_t b4 = 4 < cs ? rbz(g, 4) : (uint32_t)dst[4];
    const uint32_t b5 = 5 < cs ? rbz(g, 5) : (uint32_t)dst[5];
    g.id45 = (b4 << 8) | b5;
    if (i > 0) g.id45 = (g.id45 + 1) & 0xFFFFu;  // quirk: id0 + 1 (:1426-1431)
  }
  // pass 1: IPv4 header checksum over pkt[:iphLen] after the id / length writes (:1434)
  g.ipc = 0;
  const int dalign = (int)((uintptr_t)dst & 15u);
  uint8_t* dbase = dst - dalign;
  if (g.v4) {
    uint64_t acc = 0;
    for (int x = r; x < cs; x += 16) acc += (uint64_t)ip_stage(g, x) << ((x & 1) ? 0 : 8);
    const uint32_t t = fold32_16(row16_sum_u32(fold64_16(acc)));
    g.ipc = (~t) & 0xFFFFu;
  }
  // pass 2: L4 sum over pkt[csumStart:pktLen] + the pseudo header (:1469-1483)
  uint64_t acc = 0;
  for (int x = cs + r; x < g.pkt_len; x += 16) acc += (uint64_t)pre_csum(g, x) << (((x - cs) & 1) ? 0 : 8);
  {
    const int a_lo = g.v4 ? 12 : 8, a_n = g.v4 ? 4 : 16;  // address words (readBuf, zeroed fields)
    if (r < a_n) acc += (rbz(g, a_lo + 2 * r) << 8) | rbz(g, a_lo + 2 * r + 1);
  }
  const uint32_t tlen = (uint32_t)(uint16_t)(hdr_len - cs + seg_len);
  uint32_t t = fold32_16(row16_sum_u32(fold64_16(acc)));
  t = fold32_16(t + (g.tcp ? 6u : 17u) + tlen);
  const uint32_t l4c = (~t) & 0xFFFFu;
  // pass 3: every byte of the packet, the checksum last (:1485-1488)
  const int nk = (g.pkt_len + dalign + 15) >> 4;
  for (int k = r; k < nk; k += 16) {
    const int x0 = 16 * k - dalign;
    uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
    for (int b = 0; b < 16; ++b) {
      const int x = x0 + b;
      uint32_t v = 0;
      if (x >= 0 && x < g.pkt_len) {
        if (x == g.ca) v = l4c >> 8;
        else if (x == g.ca + 1) v = l4c & 0xFFu;
        else v = pre_csum(g, x);
      }
      w[b >> 2] |= v << (8 * (b & 3));
    }
    store_chunk(dbase + 16 * k, make_uint4(w[0], w[1], w[2], w[3]), x0, g.pkt_len);
  }
  if (r == 0) *size_out = g.pkt_len;
}
// gsoNoneChecksum + copy to bufs[0] (tun/tun.go:532-556, gro.go:1497-1517).
__device__ void none_segment(const uint8_t* rb, const Job& j, uint8_t* dst, int lane) {
  const int plen = j.plen;
  int pf = -1;
  uint32_t pv = 0;
  if (j.flags & 1) {
    const int cs = j.cs;
    const int at = (j.cs + j.co) & 0xFFFF;
    const uint32_t initial = be16at(rb + at);
    // pass 1: sum rb[cs:plen] with the field zeroed (16-byte chunks, whole wave)
    const int rel0 = cs - (int)(((uintptr_t)rb + (uintptr_t)cs) & 15u);
    const uint8_t* a0 = rb + rel0;
    const int nch = plen > cs ? (plen - rel0 + 15) >> 4 : 0;
    uint64_t acc = 0;
    for (int c = lane; c < nch; c += 64) {
      const uint4 v = ld16(a0 + 16 * c);
      const int x0 = rel0 + 16 * c;
      uint4 w = v;
      const int j0 = at - x0, j1 = at + 1 - x0;
      if (j0 >= 0 && j0 < 16) w = set_chunk_byte(w, j0, 0);
      if (j1 >= 0 && j1 < 16) w = set_chunk_byte(w, j1, 0);
      acc += chunk_sum(w, x0, cs, plen);
    }
    uint32_t s = fold32_16(wave_sum_u32(fold64_16(acc)));
    if ((((uintptr_t)rb + (uintptr_t)cs) & 1u) == 0) s = bswap16(s);
    const uint32_t t = fold32_16(s + initial);
    pf = at;
    pv = (~t) & 0xFFFFu;
  }
  const int dalign = (int)((uintptr_t)dst & 15);
  uint8_t* dbase = dst - dalign;
  const int nk = (plen + dalign + 15) >> 4;
  uint64_t dummy = 0;
  stream_copy<false>(rb, rb, rb + plen, dbase, dalign, 0, nk, plen, plen, pf, pv, lane, dummy);
}

}  // namespace

// ---------------------------------------------------------------------------
// Row-per-segment split: one 16-lane DPP row per OUTPUT segment, 64 rows per
// 1024-thread block (wave 0 decodes the job once, LDS broadcast); grid =
// (job, group of 64 segments).  Per row:
//   * the first U payload windows are loaded speculatively (gsoSize only)
//     before the decode finishes; further batches follow the decoded bounds;
//   * the header source chunks are fetched after the barrier (L2 hits);
//   * destination chunk k = r + 16u is assembled from the dword-aligned source
//     window k and the next lane's first dword (DPP row_ror:15) with a per-row
//     byte shift, summed (v_dot2) and stored as one dwordx4;
//   * the checksums come from the row sum plus job constants plus the
//     rewritten field values (gro.go:1419-1465), and the header chunks are
//     stored last with both checksums filled in.
// Each output byte is written exactly once, each input byte read once.

__device__ __forceinline__ uint32_t add4(uint32_t acc, const uint4& v) {
  return add_halves(add_halves(add_halves(add_halves(acc, v.x), v.y), v.z), v.w);
}

// acc + the chunk's bytes selected by the 16-bit byte mask m16 (rot: the
// range pairs bytes with the opposite parity of acc's range, wgcs_common.h).
__device__ __forceinline__ uint32_t add4_masked(uint32_t acc, const uint4& v, uint32_t m16, bool rot) {
  uint32_t y0 = v.x & expand_nibble(m16 & 0xFu), y1 = v.y & expand_nibble((m16 >> 4) & 0xFu);
  uint32_t y2 = v.z & expand_nibble((m16 >> 8) & 0xFu), y3 = v.w & expand_nibble((m16 >> 12) & 0xFu);
  if (rot) {
    y0 = rotl8(y0);
    y1 = rotl8(y1);
    y2 = rotl8(y2);
    y3 = rotl8(y3);
  }
  return add_halves(add_halves(add_halves(add_halves(acc, y0), y1), y2), y3);
}

// Per-byte select: bytes whose bit is set in m16 from a, the rest from b.
__device__ __forceinline__ uint4 select_bytes(const uint4& a, const uint4& b, uint32_t m16) {
  const uint32_t m0 = expand_nibble(m16 & 0xF), m1 = expand_nibble((m16 >> 4) & 0xF);
  const uint32_t m2 = expand_nibble((m16 >> 8) & 0xF), m3 = expand_nibble((m16 >> 12) & 0xF);
  return make_uint4((a.x & m0) | (b.x & ~m0), (a.y & m1) | (b.y & ~m1), (a.z & m2) | (b.z & ~m2),
                    (a.w & m3) | (b.w & ~m3));
}

// Write byte value b at packet position pos into the chunk at position x0,
// if pos < lim (header bytes only; the payload copy wins above hdrLen).
__device__ __forceinline__ void put_byte(uint4& v, int x0, int pos, uint32_t b, int lim) {
  const int t = pos - x0;
  if (pos < lim && t >= 0 && t < 16) v = set_chunk_byte(v, t, b);
}
__device__ __forceinline__ void put_be16(uint4& v, int x0, int pos, uint32_t val, int lim) {
  put_byte(v, x0, pos, val >> 8, lim);
  put_byte(v, x0, pos + 1, val, lim);
}

template <bool NT>
__device__ __forceinline__ uint4 ld_src(const uint8_t* p) {
  if (NT) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 t = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    return make_uint4(t.x, t.y, t.z, t.w);
  }
  return ld16(p);
}

// Job-uniform header sums for the common case ("fast" header): every
// per-segment header write lands inside hdrLen at a position disjoint from the
// L4 checksum field, so the per-segment IPv4 and L4 header sums are a job
// constant plus the rewritten field values (no per-segment byte sums).
struct HdrFast {
  bool fast;
  uint32_t ip_base;   // BE words of readBuf[0:csumStart) with [2:6) and [10:12) zero (IPv4)
  uint32_t l4_base;   // BE words of readBuf[csumStart:hdrLen) pairing from csumStart, csum field and
                      // seq / UDP-length zero, FIN|PSH cleared
  uint32_t addr;      // BE words of the pseudo-header addresses
  uint32_t flags;     // readBuf[csumStart + 13] (TCP flags byte)
};

// The fast header path's geometry condition: every per-segment header write
// lands inside hdrLen, disjoint from the L4 checksum field, which lies in the
// L4 header (so the raw readBuf header bytes equal the zeroed ones outside it).
__device__ __forceinline__ bool fast_header(int cs, int hl, int ca, bool tcp) {
  const int vlo = cs + 4, vhi = tcp ? cs + 8 : cs + 6;  // per-segment L4 field bytes
  return (tcp ? cs + 14 <= hl : vhi <= hl) && (ca + 2 <= vlo || ca >= vhi) && ca >= cs &&
         (!tcp || (ca != cs + 13 && ca + 1 != cs + 13));
}

__device__ __forceinline__ HdrFast header_fast(const HdrBytes& hb, const Job& j, int lane) {
  HdrFast h;
  const int cs = j.cs, hl = j.hdr_len, ca = (j.cs + j.co) & 0xFFFF;
  const bool v4 = j.ipv == 4, tcp = j.type != GSO_UDP_L4;
  const int vlo = cs + 4, vhi = tcp ? cs + 8 : cs + 6;  // per-segment L4 field bytes
  h.fast = fast_header(cs, hl, ca, tcp);
  const int a_lo = v4 ? 12 : 8, a_hi = v4 ? 20 : 40;
  uint32_t ip = 0, l4 = 0, ad = 0;
  const uint32_t regs[4] = {hb.r0, hb.r1, hb.r2, hb.r3};
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const int x = lane + 64 * m - 10;  // readBuf position of this lane's byte
    const uint32_t b = regs[m];
    if (x < 0 || x >= hl) continue;
    const uint32_t hi8 = b << 8;
    if (v4 && x < cs && (x < 2 || x >= 6) && x != 10 && x != 11) ip += (x & 1) ? b : hi8;
    if (x >= cs && x != ca && x != ca + 1 && (x < vlo || x >= vhi)) {
      const uint32_t bb = (tcp && x == cs + 13) ? (b & ~0x09u) : b;
      l4 += ((x - cs) & 1) ? bb : (bb << 8);
    }
    if (x >= a_lo && x < a_hi) ad += (x & 1) ? b : hi8;
  }
  h.ip_base = wave_sum_u32(ip);
  h.l4_base = wave_sum_u32(l4);
  h.addr = wave_sum_u32(ad);
  h.flags = tcp ? hb(10 + cs + 13) : 0u;
  return h;
}

// Header chunks in packet coordinates (lane r: bytes [16r, 16r + 16)):
// write byte / big-endian u16 `val` at the wave-uniform position pos.
__device__ __forceinline__ void put_u(uint4& P, int r, int pos, uint32_t val, uint32_t nbytes_mask) {
  const int sh = 8 * (pos & 3);
  const uint32_t m = r == (pos >> 4) ? (nbytes_mask << sh) : 0u;
  const uint32_t v = val << sh;
  switch ((pos >> 2) & 3) {
    case 0: P.x = (P.x & ~m) | (v & m); break;
    case 1: P.y = (P.y & ~m) | (v & m); break;
    case 2: P.z = (P.z & ~m) | (v & m); break;
    default: P.w = (P.w & ~m) | (v & m); break;
  }
}
__device__ __forceinline__ void put_be16_u(uint4& P, int r, int pos, uint32_t val) {
  if ((pos & 1) == 0) {  // both bytes in one dword (pos & 3 is 0 or 2)
    put_u(P, r, pos, bswap16(val & 0xFFFFu), 0xFFFFu);
  } else {
    put_u(P, r, pos, (val >> 8) & 0xFFu, 0xFFu);
    put_u(P, r, pos + 1, val & 0xFFu, 0xFFu);
  }
}

// Job-level values decoded once per block by wave 0 and broadcast through LDS.
struct JobInfo {
  int32_t status, count, nseg, type, ipv, hdr_len, gso, cs, co, plen, flags, fast, gen;
  uint32_t id0, seq0, ip_base, l4_base, addr, tflags;
};

__device__ __forceinline__ int ufl(int x) { return __builtin_amdgcn_readfirstlane(x); }

// Row-per-segment split.  Block = 1024 threads = 64 rows of 16 lanes = 64
// consecutive output segments of one job; grid = (job, segment group).
// One decoder wave decodes the job once and broadcasts it through LDS in two
// steps (geometry, then the job-constant header sums) -- per-wave decoding
// made the CU's shared scalar unit the bottleneck (16 decodes per CU).
template <int U, bool NT, int WAVES>
__global__ __launch_bounds__(64 * WAVES) void gso_rows_kernel(const uint8_t* __restrict__ arena,
                                                        const wgcs_gso_job* __restrict__ jobs, uint32_t max_segs,
                                                        uint8_t* __restrict__ out, uint32_t out_stride,
                                                        const GsoOutPos* __restrict__ outpos,
                                                        uint32_t offset, uint32_t room, int32_t* __restrict__ sizes,
                                                        int32_t* __restrict__ count, int32_t* __restrict__ status) {
  __shared__ JobInfo ji;
  constexpr int ROWS = 4 * WAVES;   // segments per block (one 16-lane row each)
  __shared__ uint32_t s_tpay[ROWS];   // per segment of the block: row-reduced payload sum (dense header phase)
  __shared__ uint4 s_keep[ROWS][8];   // per segment: payload bytes of destination chunks 0..7
  const int lane = threadIdx.x & 63;
  const int r = lane & 15;
  const int wv = threadIdx.x >> 6;
  const uint32_t jb = blockIdx.x;
  const wgcs_gso_job job = jobs[jb];  // one scalar load of the whole descriptor, flags included
  const uint8_t* vb = arena + job.off;
  const uint32_t jlen = job.len;
  const uint8_t* rb = vb + 10;
  const uint64_t slot0 = (uint64_t)jb * max_segs;  // sizes[] index of segment 0
  // segment i of this job at out + obase + i * opitch (+ offset): fixed slots,
  // or the caller's packed per-job layout (the stager's compact D2H region)
  uint64_t obase = slot0 * out_stride;
  uint32_t opitch = out_stride;
  if (outpos) {
    obase = outpos[jb].base;
    opitch = outpos[jb].pitch;
  }
  const uint32_t seg0 = blockIdx.y * (uint32_t)ROWS + (uint32_t)wv * 4u;  // wave-uniform
  const int i = (int)seg0 + (lane >> 4);                       // this row's segment
  uint8_t* dst = out + obase + (uint64_t)i * opitch + offset;
  const int dalign = (int)((uintptr_t)dst & 15u);
  uint8_t* dbase = dst - dalign;

  // ---- decoder wave (the block's last: its rows are the least likely to
  // exist, 45 segments per job at cfg4): validation and geometry, published
  // through LDS at barrier 1; the job-constant header sums follow at barrier
  // 2, computed while the other waves stream their payload.  It decodes
  // before issuing its own speculative loads: a decode step that waited on a
  // global load would otherwise wait (vmcnt retires in order) for that batch.
  constexpr int kDec = WAVES - 1;
  HdrBytes hb;
  Job jd = {};
  bool jd_ok = false;
  if (wv == kDec) {
    __builtin_amdgcn_s_setprio(3);  // the decode chain is the block's critical path (until barrier 2)
    hb.load(vb, (int)min(jlen, 256u), lane);
    jd = decode_job(hb, jlen, job.flags, room, max_segs);
    jd_ok = jd.status == 0 || jd.status == WGCS_ERR_TOO_MANY_SEGMENTS;
    if (lane == 0) {
      ji.status = jd.status;
      ji.count = jd_ok ? jd.count : 0;
      ji.nseg = jd_ok ? jd.nseg : 0;
      ji.type = jd.type;
      ji.ipv = jd.ipv;
      ji.hdr_len = jd.hdr_len;
      ji.gso = jd.gso;
      ji.cs = jd.cs;
      ji.co = jd.co;
      ji.plen = jd.plen;
      ji.flags = jd.flags;
      ji.gen = jd.gen;
      if (blockIdx.y == 0) {
        count[jb] = ji.count;
        status[jb] = jd.status;
      }
    }
  }

  // ---- speculative first payload batch.  The source window of segment i
  // needs only gsoSize (virtio header bytes 4-5), so every row issues its
  // first U payload loads before the block barrier: the decode and the
  // barrier overlap the HBM round trip instead of preceding it.  The
  // guards keep the loads inside the job's own bytes [vb, rb + plen); bytes a
  // window picks up outside the segment are masked exactly as on the decoded
  // path (header positions, past pktLen).  GSO_NONE jobs skip it.
  int gso_s = 0, type_s = GSO_NONE;
  if (wv == kDec) {
    if (jlen >= 10) {
      type_s = (int)hb(1);
      gso_s = (int)hb.le16(4);
    }
  } else if (jlen >= 10) {
    type_s = (int)u8at(vb + 1);
    gso_s = (int)(u8at(vb + 4) | (u8at(vb + 5) << 8));
  }
  const int plen_s = jlen >= 10 ? (int)jlen - 10 : 0;
  const uint8_t* jend = rb + plen_s;
  const uint8_t* w0 = rb + (int64_t)i * gso_s - dalign;  // source of destination chunk 0 (payload positions)
  const int sb = (int)((uintptr_t)w0 & 3u);              // byte shift within dwords
  const uint8_t* abase = w0 - sb;                        // dword-aligned window base
  const uint4 z = make_uint4(0, 0, 0, 0);
  uint4 A[U];
  uint32_t E = 0;
  // RAW jobs split whatever the type byte says (gsoSplit maps non-TCP types to
  // UDP, gro.go:1398-1405): only handleVirtioRead's GSO_NONE copies one packet
  const bool splits = type_s != GSO_NONE || (job.flags & WGCS_GSO_JOB_RAW) != 0;
  const bool spec = splits && (int64_t)i * gso_s < (int64_t)plen_s;  // row-uniform
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint8_t* ca = abase + 16 * (r + 16 * u);
    A[u] = (spec && ca >= vb && ca < jend) ? ld_window<NT>(ca, jend) : z;
  }
  if (spec && r == 15) {
    const uint8_t* ce = abase + 16 * (16 * U);
    if (ce >= vb && ce < jend) E = *reinterpret_cast<const uint32_t*>(__builtin_assume_aligned(ce, 4));
  }

  // ---- speculative header chunks in packet coordinates (the fast path's;
  // bytes past hdrLen are replaced by payload bytes later): L2 hits shared by
  // the job's segments, issued after the payload batch so waiting for the
  // payload does not wait for them.
  const int hph_s = (int)((uintptr_t)rb & 15u);
  const uint8_t* hab_s = rb - hph_s + 16 * r;
  const uint8_t* hend_s = rb + min(plen_s, kMaxHdrLen + 16);
  // Issued unconditionally, only the address is selected (a chunk past
  // hend_s reads the chunk holding rb, a row that does not speculate reads
  // the job table; the fast path uses H0/H1 only when spec_ok and never their
  // bytes past hdrLen).  Together with the decoder's raised priority: 11.74 ->
  // 11.54 us on cfg4 (each change alone was slower, scripts/exp_gso.sh).
  const uint8_t* hsafe = rb - hph_s;  // the 16-byte chunk holding rb
  const uint8_t* hdummy = reinterpret_cast<const uint8_t*>(jobs);
  uint4 H0 = ld_src<NT>(spec ? (hab_s < hend_s ? hab_s : hsafe) : hdummy);
  uint4 H1 = ld_src<NT>(spec ? (hab_s + 16 < hend_s ? hab_s + 16 : hsafe) : hdummy);

  lds_barrier();  // barrier 1: geometry; the speculative loads stay in flight
  // block-uniform: whether the header phase (and so barrier 2) happens at all
  const bool hdr_phase = ufl(ji.nseg) > 0 && ufl(ji.type) != GSO_NONE && ufl(ji.gen) == 0;
  if (wv == kDec && hdr_phase) {
    const HdrFast hf = header_fast(hb, jd, lane);
    // readBuf bytes after gsoSplit zeroed the L4 checksum field (gro.go:1393;
    // the IPv4 checksum bytes 10-11 are neither id nor seq here: cs >= 20)
    const int ca = (jd.cs + jd.co) & 0xFFFF;
    auto zb = [&](int x) { return (x == ca || x == ca + 1) ? 0u : hb(10 + x); };
    const uint32_t id0 = jd.ipv == 4 ? (zb(4) << 8) | zb(5) : 0u;
    const int sq = jd.cs + 4;
    const uint32_t seq0 = jd.type != GSO_UDP_L4 ? (zb(sq) << 24) | (zb(sq + 1) << 16) | (zb(sq + 2) << 8) | zb(sq + 3) : 0u;
    if (lane == 0) {
      ji.fast = hf.fast ? 1 : 0;
      ji.id0 = id0;
      ji.seq0 = seq0;
      ji.ip_base = hf.ip_base;
      ji.l4_base = hf.l4_base;
      ji.addr = hf.addr;
      ji.tflags = hf.flags;
    }
    // barrier 2 (header constants).  Waves that retire early are not waited
    // for: s_barrier only counts the workgroup's surviving waves.
    lds_barrier();
  }
  if (wv == kDec) __builtin_amdgcn_s_setprio(0);
  Job j = {};
  j.status = ufl(ji.status);
  j.nseg = ufl(ji.nseg);
  j.type = ufl(ji.type);
  if (j.nseg == 0) return;  // error status (or an empty packet)
  j.plen = ufl(ji.plen);
  j.cs = ufl(ji.cs);
  j.co = ufl(ji.co);
  j.flags = ufl(ji.flags);
  if (j.type == GSO_NONE) {  // one packet: wave 0 of the job's first block
    if (seg0 == 0) {
      none_segment(rb, j, out + obase + offset, lane);
      if (lane == 0) sizes[slot0] = j.plen;
    }
    return;
  }
  if (seg0 >= (uint32_t)j.nseg) return;
  j.ipv = ufl(ji.ipv);
  j.hdr_len = ufl(ji.hdr_len);
  j.gso = ufl(ji.gso);
  const bool v4 = j.ipv == 4, tcp = j.type != GSO_UDP_L4;
  if (i >= j.nseg) return;  // whole rows retire; DPP below stays inside live rows
  if (ufl(ji.gen)) {  // block-uniform: no barrier 2 for general jobs
    gso_general_row(rb, j.plen, j.type, j.ipv, j.hdr_len, j.gso, j.cs, j.co, i, dst, r, &sizes[slot0 + (uint32_t)i]);
    return;
  }
  const bool spec_ok = spec && j.gso == gso_s;  // always true: both read virtio bytes 4-5

  // ---- segment geometry (row-uniform)
  const int hdr_len = j.hdr_len, cs = j.cs, plen = j.plen;
  const int csum_at = (cs + j.co) & 0xFFFF;
  const int seg_start = hdr_len + i * j.gso;
  const int seg_end = min(plen, seg_start + j.gso);
  const int seg_len = seg_end - seg_start;
  const int pkt_len = hdr_len + seg_len;
  const bool last = seg_end == plen;
  const uint64_t slot = slot0 + (uint32_t)i;
  const int nk = (pkt_len + dalign + 15) >> 4;
  const int hk = min((hdr_len + dalign + 15) >> 4, nk);
  const uint8_t* src_lo = rb + seg_start;
  const uint8_t* src_hi = rb + seg_end;


  // ---- payload stream: destination chunk k = bytes [sb, sb + 16) of the
  // dword-aligned window k and the first dword of window k + 1 (next lane, DPP)
  uint32_t acc = 0;  // L4 bytes [hdrLen, pktLen): LE words at destination addresses
  uint4 keep = z;    // payload part of header chunk r (r < hk)
  for (int k0 = 0; k0 < nk; k0 += 16 * U) {
    if (k0 > 0 || !spec_ok) {  // wave-uniform; the first batch is normally the speculative one
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint8_t* ca = abase + 16 * (k0 + r + 16 * u);
        A[u] = (ca < src_hi && ca + 16 > src_lo) ? ld_window<NT>(ca, src_hi) : z;
      }
      E = 0;
      if (r == 15) {
        const uint8_t* ce = abase + 16 * (k0 + 16 * U);
        if (ce < src_hi && ce + 4 > src_lo) E = *reinterpret_cast<const uint32_t*>(__builtin_assume_aligned(ce, 4));
      }
    }
    uint32_t Rc = row_next(A[0].x);  // lane 15: lane 0's next-u dword
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = k0 + r + 16 * u;
      const uint32_t Rx = u + 1 < U ? row_next(A[u + 1 < U ? u + 1 : u].x) : E;
      const uint32_t nx = r == 15 ? Rx : Rc;
      Rc = Rx;
      if (k < nk) {
        const uint4 v = make_uint4(__builtin_amdgcn_alignbyte(A[u].y, A[u].x, sb),
                                   __builtin_amdgcn_alignbyte(A[u].z, A[u].y, sb),
                                   __builtin_amdgcn_alignbyte(A[u].w, A[u].z, sb),
                                   __builtin_amdgcn_alignbyte(nx, A[u].w, sb));
        const int x0 = 16 * k - dalign;
        if (x0 >= hdr_len && x0 + 16 <= pkt_len) acc = add4(acc, v);
        else acc = add4_masked(acc, v, byte_bits16(hdr_len - x0, pkt_len - x0), false);
        if (k < hk) keep = v;
        else store_chunk(dbase + 16 * k, v, x0, pkt_len);
      }
    }
  }

  // ---- lane-dense header phase (fast headers of <= 113 bytes): the row
  // publishes its payload sum and the payload part of its header chunks, and
  // after barrier 2 Ld = 4 or 8 lanes per segment (instead of a whole 16-lane
  // row, of which only hk lanes hold header bytes) rewrite and store the
  // headers: 16 or 8 segments per wave, a quarter or half of the VALU issue.
  // Block-uniform; needs the decoder wave to own no segment of this block
  // (its rows publish only after barrier 2).
  const int nb = min(ROWS, j.nseg - (int)(blockIdx.y * (uint32_t)ROWS));
  const int Ld = nb <= ROWS - 4 ? (hdr_len <= 49 ? 4 : (hdr_len <= 113 ? 8 : 0)) : 0;
  if (Ld) {
    const uint32_t tp = fold32_16(row16_sum_u32(acc));
    const int sloc_r = i - (int)(blockIdx.y * (uint32_t)ROWS);
    if (r == 0) s_tpay[sloc_r] = tp;
    if (r < 8) s_keep[sloc_r][r] = keep;
  }

  // ---- job-constant header sums (barrier 2; the decoder wave passed it already)
  if (wv != kDec) lds_barrier();
  const bool fast = ufl(ji.fast) != 0;
  const uint32_t id0 = (uint32_t)ufl((int)ji.id0), seq0 = (uint32_t)ufl((int)ji.seq0);
  const uint32_t ip_base = (uint32_t)ufl((int)ji.ip_base), l4_base = (uint32_t)ufl((int)ji.l4_base);
  const uint32_t addr_sum = (uint32_t)ufl((int)ji.addr), tflags = (uint32_t)ufl((int)ji.tflags);

  if (fast && Ld) {
    const int spw = 64 / Ld;                   // segments per wave
    if (wv * spw >= nb) return;                // wave-uniform: no header of this wave
    const int sl = lane / Ld, c = lane % Ld;   // segment within the wave, header chunk
    const int sloc = wv * spw + sl;
    const bool valid2 = sloc < nb;             // lanes of live rows (Ld <= 16)
    const int i2 = (int)(blockIdx.y * (uint32_t)ROWS) + (valid2 ? sloc : 0);
    const int seg_start2 = hdr_len + i2 * j.gso;
    const int seg_end2 = min(plen, seg_start2 + j.gso);
    const int seg_len2 = seg_end2 - seg_start2;
    const int pkt_len2 = hdr_len + seg_len2;
    const bool last2 = seg_end2 == plen;
    uint8_t* dst2 = out + obase + (uint64_t)i2 * opitch + offset;
    const int dalign2 = (int)((uintptr_t)dst2 & 15u);
    uint8_t* dbase2 = dst2 - dalign2;
    const int nk2 = (pkt_len2 + dalign2 + 15) >> 4;
    const int hk2 = min((hdr_len + dalign2 + 15) >> 4, nk2);
    // header source chunks c, c + 1 (packet coordinates, wave-uniform phase):
    // the speculative H0/H1 of this wave's first row, lane c (its segment
    // speculated: it is live), fetched across lanes -- no memory round trip
    // after the barrier.  Their bytes past hdrLen are never used.
    const int hph = (int)((uintptr_t)rb & 15u);
    const uint4 G0 = make_uint4((uint32_t)__shfl((int)H0.x, c), (uint32_t)__shfl((int)H0.y, c),
                                (uint32_t)__shfl((int)H0.z, c), (uint32_t)__shfl((int)H0.w, c));
    const uint4 G1 = make_uint4((uint32_t)__shfl((int)H1.x, c), (uint32_t)__shfl((int)H1.y, c),
                                (uint32_t)__shfl((int)H1.z, c), (uint32_t)__shfl((int)H1.w, c));
    const uint32_t id = i2 > 0 ? ((id0 + 1) & 0xFFFFu) : id0;  // quirk: id0 + 1 for every i >= 1 (:1426-1431)
    const uint32_t seq = seq0 + (uint32_t)(uint16_t)((uint16_t)j.gso * (uint16_t)i2);  // uint16 product (:1445)
    const uint32_t ulen = (uint32_t)(uint16_t)(seg_len2 + (hdr_len - cs));            // UDP length (:1462-1465)
    const uint32_t tlen = (uint32_t)(uint16_t)(hdr_len - cs + seg_len2);              // transportLen (:1469-1471)
    const uint32_t proto = tcp ? 6u : 17u;
    uint32_t t_pay = s_tpay[valid2 ? sloc : 0];
    if ((((uintptr_t)dst2 + (uintptr_t)cs) & 1u) == 0) t_pay = bswap16(t_pay);  // pairing from csumStart
    const uint32_t var = tcp ? (seq >> 16) + (seq & 0xFFFFu) + (last2 ? (tflags & 0x09u) : 0u) : ulen;
    const uint32_t l4c = (~fold32_16(t_pay + fold32_16(l4_base) + var + fold32_16(addr_sum) + proto + tlen)) & 0xFFFFu;
    uint4 P = funnel(G0, G1, hph);
    if (v4) {
      const uint32_t ipc = (~fold32_16(fold32_16(ip_base) + (uint32_t)pkt_len2 + id)) & 0xFFFFu;
      put_be16_u(P, c, 2, (uint32_t)pkt_len2);  // total length (:1433)
      put_be16_u(P, c, 4, id);                  // identification (:1426-1431)
      put_be16_u(P, c, 10, ipc);                // header checksum (:1434-1436)
    } else {
      put_be16_u(P, c, 4, (uint32_t)(pkt_len2 - cs));  // payload length (:1439)
    }
    if (tcp) {
      put_be16_u(P, c, cs + 4, seq >> 16);  // sequence number (:1445-1446)
      put_be16_u(P, c, cs + 6, seq);
      put_u(P, c, cs + 13, last2 ? tflags : (tflags & ~0x09u), 0xFFu);  // FIN|PSH on the last only (:1447-1459)
    } else {
      put_be16_u(P, c, cs + 4, ulen);
    }
    put_be16_u(P, c, csum_at, l4c);  // L4 checksum (:1486-1490)
    // to the destination phase: the previous chunk of the same segment (DPP
    // row_shr:1; a group's first lane has none), merged with the payload bytes
    uint4 Pp = row_prev4(P);
    if (c == 0) Pp = z;
    const uint4 D = dalign2 ? funnel_v(Pp, P, 16 - dalign2) : P;
    const int x0h2 = 16 * c - dalign2;
    const uint32_t hmask2 = byte_bits16(-x0h2, hdr_len - x0h2);
    const uint4 keep2 = s_keep[valid2 ? sloc : 0][c];
    if (valid2 && c < hk2) store_chunk(dbase2 + 16 * c, select_bytes(D, keep2, hmask2), x0h2, pkt_len2);
    if (valid2 && c == 0) sizes[slot0 + (uint32_t)i2] = pkt_len2;
    return;
  }

  // ---- header source chunks (shared by the job's segments: L2 hits).
  // fast: packet coordinates (lane r = readBuf[16r, 16r + 16), wave-uniform
  // phase), normally the speculative H0/H1; general: destination coordinates
  // (per-row phase).
  const uint8_t* hend = rb + hdr_len;
  const int hph = fast ? (int)((uintptr_t)rb & 15u) : (int)((uintptr_t)(rb - dalign) & 15u);
  const uint8_t* hab = (fast ? rb : rb - dalign) - hph + 16 * r;
  if (!fast || !spec_ok) {  // row-uniform
    H0 = z;
    H1 = z;
    if (r < hk) {
      if (hab < hend && hab + 16 > rb) H0 = ld16(hab);
      if (hab + 16 < hend && hab + 32 > rb) H1 = ld16(hab + 16);
    }
  }

  const uint32_t id = i > 0 ? ((id0 + 1) & 0xFFFFu) : id0;  // quirk: id0 + 1 for every i >= 1 (:1426-1431)
  const uint32_t seq = seq0 + (uint32_t)(uint16_t)((uint16_t)j.gso * (uint16_t)i);  // uint16 product (:1445)
  const uint32_t ulen = (uint32_t)(uint16_t)(seg_len + (hdr_len - cs));            // UDP length (:1462-1465)
  const uint32_t tlen = (uint32_t)(uint16_t)(hdr_len - cs + seg_len);              // transportLen (:1469-1471)
  const uint32_t proto = tcp ? 6u : 17u;
  const int x0h = 16 * r - dalign;
  const uint32_t hmask = byte_bits16(-x0h, hdr_len - x0h);  // header positions of destination chunk r

  if (fast) {
    // ---- sums: payload (row reduction) + job constants + rewritten fields
    uint32_t t_pay = fold32_16(row16_sum_u32(acc));
    if ((((uintptr_t)dst + (uintptr_t)cs) & 1u) == 0) t_pay = bswap16(t_pay);  // pairing from csumStart
    const uint32_t var = tcp ? (seq >> 16) + (seq & 0xFFFFu) + (last ? (tflags & 0x09u) : 0u) : ulen;
    const uint32_t l4c = (~fold32_16(t_pay + fold32_16(l4_base) + var + fold32_16(addr_sum) + proto + tlen)) & 0xFFFFu;
    // ---- header chunk in packet coordinates, rewritten (gro.go:1418-1465, :1486-1490)
    uint4 P = funnel(H0, H1, hph);
    if (v4) {
      const uint32_t ipc = (~fold32_16(fold32_16(ip_base) + (uint32_t)pkt_len + id)) & 0xFFFFu;
      put_be16_u(P, r, 2, (uint32_t)pkt_len);  // total length (:1433)
      put_be16_u(P, r, 4, id);                 // identification (:1426-1431)
      put_be16_u(P, r, 10, ipc);               // header checksum (:1434-1436)
    } else {
      put_be16_u(P, r, 4, (uint32_t)(pkt_len - cs));  // payload length (:1439)
    }
    if (tcp) {
      put_be16_u(P, r, cs + 4, seq >> 16);  // sequence number (:1445-1446)
      put_be16_u(P, r, cs + 6, seq);
      put_u(P, r, cs + 13, last ? tflags : (tflags & ~0x09u), 0xFFu);  // FIN|PSH on the last only (:1447-1459)
    } else {
      put_be16_u(P, r, cs + 4, ulen);
    }
    put_be16_u(P, r, csum_at, l4c);  // L4 checksum (:1486-1490)
    // ---- to destination phase, merge with the payload bytes, store
    const uint4 Pp = row_prev4(P);
    const uint4 D = dalign ? funnel_v(Pp, P, 16 - dalign) : P;
    if (r < hk) store_chunk(dbase + 16 * r, select_bytes(D, keep, hmask), x0h, pkt_len);
  } else {
    // ---- general header path (unusual csum offsets / short RAW headers):
    // byte-exact replay of the reference's write order on the chunk
    const int a_lo = v4 ? 12 : 8, a_hi = v4 ? 20 : 40;
    uint32_t acc_ip = 0;
    uint4 hv = z;
    if (r < hk) {
      hv = select_bytes(funnel_v(H0, H1, hph), keep, hmask);
      // readBuf's zeroed fields (gro.go:1388,:1393), then the per-segment header writes in order
      if (v4) put_be16(hv, x0h, 10, 0, hdr_len);
      put_be16(hv, x0h, csum_at, 0, hdr_len);
      if (v4) {
        put_be16(hv, x0h, 4, id, hdr_len);
        put_be16(hv, x0h, 2, pkt_len, hdr_len);
      } else {
        put_be16(hv, x0h, 4, pkt_len - cs, hdr_len);
      }
      if (tcp) {
        put_be16(hv, x0h, cs + 4, seq >> 16, hdr_len);
        put_be16(hv, x0h, cs + 6, seq, hdr_len);
        const int fl = cs + 13 - x0h;
        if (!last && cs + 13 < hdr_len && fl >= 0 && fl < 16) hv = set_chunk_byte(hv, fl, chunk_byte(hv, fl) & ~0x09u);
      } else {
        put_be16(hv, x0h, cs + 4, ulen, hdr_len);
      }
      if (v4) acc_ip = add4_masked(0u, hv, byte_bits16(-x0h, cs - x0h), false);
      acc = add4_masked(acc, hv, byte_bits16(cs - x0h, hdr_len - x0h), false);
      acc = add4_masked(acc, hv, byte_bits16(a_lo - x0h, a_hi - x0h), (cs & 1) != 0);  // pseudo-header addresses
    }
    uint32_t t_ip = fold32_16(row16_sum_u32(acc_ip));
    if ((((uintptr_t)dst) & 1u) == 0) t_ip = bswap16(t_ip);
    uint32_t t_l4 = fold32_16(row16_sum_u32(acc));
    if ((((uintptr_t)dst + (uintptr_t)cs) & 1u) == 0) t_l4 = bswap16(t_l4);
    const uint32_t l4c = (~fold32_16(t_l4 + proto + tlen)) & 0xFFFFu;
    if (r < hk) {
      if (v4) put_be16(hv, x0h, 10, (~t_ip) & 0xFFFFu, hdr_len);
      put_be16(hv, x0h, csum_at, l4c, hdr_len);
      store_chunk(dbase + 16 * r, hv, x0h, pkt_len);
    }
  }
  if (r == 0) sizes[slot] = pkt_len;
}

hipError_t launch_gso_split_batch(const uint8_t* arena, const wgcs_gso_job* jobs, uint32_t n_jobs, uint8_t* out,
                                  uint32_t out_stride, uint32_t offset, uint32_t max_segs, int32_t* sizes,
                                  int32_t* count, int32_t* status, hipStream_t s, const GsoOutPos* outpos,
                                  uint32_t room) {
  if (n_jobs == 0 || max_segs == 0) return hipSuccess;
  if (!outpos) room = out_stride > offset ? out_stride - offset : 0;
  // 16 waves = 64 segments per 1024-thread block.  Smaller blocks (8 / 4 waves,
  // more decodes per CU) measured slower on cfg4: 12.7 / 13.0 vs 11.6 us.
  constexpr int kWaves = 16;
  const uint32_t rows = 4u * (uint32_t)kWaves;
  const uint32_t gy = (max_segs + rows - 1) / rows;
  if (gy > 65535u) return hipErrorInvalidValue;
  hipLaunchKernelGGL((gso_rows_kernel<6, true, kWaves>), dim3(n_jobs, gy), dim3(64 * kWaves), 0, s, arena, jobs,
                     max_segs, out, out_stride, outpos, offset, room, sizes, count, status);
  return hipGetLastError();
}

}  // namespace wgcs
