// gso_kernels.hip -- gfx950 GSO split (TSO/USO super-packet -> MSS segments).
//
// Device-resident batch of the reference's Tun.Read path:
//   handleVirtioRead validation/dispatch   /root/reference/tun/tun.go:514-632
//   gsoSplit                               /root/reference/tun/gro.go:1373-1493
//   gsoNoneChecksum (GSO_NONE + NEEDS_CSUM) /root/reference/tun/gro.go:1497-1517
//
// Mapping (gso_rows_kernel): one 16-lane DPP row per OUTPUT segment (slot =
// job * max_segs + i), 16 segments per 256-thread block, grid = (job,
// segment group).  For the common ("clean") job every wave derives the split
// geometry from the virtio header and the header chunks it loads (one
// 16-byte load of the virtio header + one dword-aligned 16-byte window per
// lane), issues its payload loads (dword-aligned
// 16-byte windows, U per lane in flight) and, with no decode step and no
// barrier,
//   1. shifts each window to the destination's byte phase (alignbyte with the
//      next lane's first dword via DPP row_ror), sums the L4 bytes from the
//      same registers (v_dot2) and stores full global_store_dwordx4 chunks;
//   2. computes the IPv4 and L4 checksums from the row sum plus the header
//      sums of its own header chunks and the rewritten field values, rewrites
//      the header chunk and stores it last -- every output byte written once.
// Any other job takes the decoded path: wave 0 runs the full validation and
// publishes its verdict through LDS (one barrier), the rows follow it.
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

__device__ __forceinline__ uint32_t u8at(const uint8_t* p) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)ldg8(p)); }
__device__ __forceinline__ uint32_t be16at(const uint8_t* p) { return (u8at(p) << 8) | u8at(p + 1); }

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
    r0 = lane < n ? ldg8(vb + lane) : 0u;
    r1 = lane + 64 < n ? ldg8(vb + lane + 64) : 0u;
    r2 = lane + 128 < n ? ldg8(vb + lane + 128) : 0u;
    r3 = lane + 192 < n ? ldg8(vb + lane + 192) : 0u;
  }
  __device__ __forceinline__ uint32_t operator()(int k) const {  // k wave-uniform
    if (k >= 256) return u8at(base + k);
    const int l = k & 63;
    const uint32_t v = k < 64 ? r0 : (k < 128 ? r1 : (k < 192 ? r2 : r3));
    return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
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
  int spare;     // bytes of readBuf's spare capacity after the packet (WGCS_GSO_JOB_SPARE)
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
// is the reference's uint16 sum.  The pseudo-header address slices may reach
// past len(readBuf) into the job's spare capacity (WGCS_GSO_JOB_SPARE), not
// past it.  Then: does the
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
    if (plen + j.spare < (v4 ? 20 : 40)) return false;         // address slices: up to cap(readBuf)
  }
  // (and every per-segment L4 field inside the header: a seq / UDP length /
  // flags byte past hdrLen can land past a short segment's end, which only the
  // general path writes)
  j.gen = !(j.cs >= (v4 ? 20 : 40) && ca + 2 <= j.hdr_len && j.hdr_len <= kMaxHdrLen &&
            j.cs + (tcp ? 14 : 6) <= j.hdr_len);
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
  j.spare = (int)((jflags >> 8) & 0xFFu);
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
  return ldg8(g.rb + x);
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
                                int i, uint8_t* dst, int r, int32_t* size_out, bool tails) {
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
    const uint32_t b4 = 4 < cs ? rbz(g, 4) : ldg8(dst + 4);
    const uint32_t b5 = 5 < cs ? rbz(g, 5) : ldg8(dst + 5);
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
  // The header writes that land past the packet's end (a header geometry with
  // fields beyond hdrLen and a short segment): gsoSplit writes them into
  // bufs[i] all the same, in its order -- id / length / IPv4 checksum (:1426-
  // 1439), seq + flags or UDP length (:1443-1466), the L4 checksum last
  // (:1485-1488).  Every position lies inside the slot: the decoder refused
  // (OUT_OF_RANGE) a slot shorter than segment 0's reach (split_need).  A
  // packed host region sized for the packets alone says !tails (GsoOutPos).
  if (r == 0 && tails) {
    auto put = [&](int x, uint32_t v) {
      if (x >= g.pkt_len) dst[x] = (uint8_t)v;
    };
    if (g.v4) {
      if (i > 0) {
        put(4, g.id45 >> 8);
        put(5, g.id45 & 0xFFu);
      }
      put(2, ((uint32_t)g.pkt_len >> 8) & 0xFFu);
      put(3, (uint32_t)g.pkt_len & 0xFFu);
      put(10, g.ipc >> 8);
      put(11, g.ipc & 0xFFu);
    } else {
      const uint32_t pl = (uint32_t)(g.pkt_len - cs) & 0xFFFFu;
      put(4, pl >> 8);
      put(5, pl & 0xFFu);
    }
    if (g.tcp) {
      for (int t = 0; t < 4; ++t) put(g.s4 + t, (g.seq >> (24 - 8 * t)) & 0xFFu);
      if (!g.last && g.f13 >= g.pkt_len) dst[g.f13] = (uint8_t)(ldg8(dst + g.f13) & ~0x09u);
    } else {
      put(g.s4, g.ulen >> 8);
      put(g.s4 + 1, g.ulen & 0xFFu);
    }
    put(g.ca, l4c >> 8);
    put(g.ca + 1, l4c & 0xFFu);
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
// Row-per-segment split: one 16-lane DPP row per OUTPUT segment, 16 rows per
// 256-thread block; grid = (job, group of 16 segments).  Per row:
//   * payload windows are dword-aligned 16-byte raw buffer loads over the
//     job's bytes (range-checked: nothing past the job is touched, no page
//     test), U per lane in flight;
//   * destination chunk k = r + 16u is assembled from window k and the next
//     lane's first dword (DPP row_ror:15) with a per-row byte shift, summed
//     (v_dot2) and stored as one dwordx4 (byte-exact pieces at the edges);
//   * the checksums come from the row sum plus job constants plus the
//     rewritten field values (gro.go:1419-1465), and the header bytes are
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

// Job-level values decoded once per block by the decoder wave, published
// through LDS (read by the rows before their header phase).
struct JobInfo {
  int32_t status, count, nseg;
  uint32_t shape;  // type | ipv << 8 | gen << 16 | fast << 24
  int32_t hdr_len, gso, cs, co, plen, flags;
  uint32_t id0, seq0, ip_base, l4_base, addr, tflags;
};

__device__ __forceinline__ int ufl(int x) { return __builtin_amdgcn_readfirstlane(x); }

// Buffer resource over one job's bytes [vb, vb + jlen): every dword holding a
// job byte passes the range check (num_records jlen + 3), loads past it
// return zeros instead of touching memory past the arena.  Built from
// wave-uniform values only (one descriptor per wave, no waterfall).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t job_rsrc(const uint8_t* vb, uint32_t jlen) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(vb), (short)0, (int)(jlen + 3u), 0x00020000);
}
template <bool NT>
__device__ __forceinline__ uint4 bld16(__amdgpu_buffer_rsrc_t rs, int off) {
  const auto t = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, WGCS_LD_AUX(NT));
  return make_uint4(t[0], t[1], t[2], t[3]);
}
// One batch of dword-aligned windows: lane r loads windows k0 + r + 16u at job
// offset aoff + 16 * window (lane 15 also the first dword of the window after
// the batch, E), each only when it overlaps the job bytes [lo, hi).
// A window that is not needed gets an offset past the resource's range instead
// of a branch around its load: the range check returns zeros and touches no
// memory, so the loads are issued unconditionally (no exec-mask branches, and
// the compiler can wait on them one by one with vmcnt(n)).
constexpr int kOobOffset = 0x7FFFFFF0;
template <int U, bool NT>
__device__ __forceinline__ void load_windows(__amdgpu_buffer_rsrc_t rs, int aoff, int k0, int r, int lo, int hi,
                                             uint4 (&A)[U], uint32_t& E) {
  const int o0 = aoff + 16 * (k0 + r);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int o = o0 + 256 * u;
    A[u] = bld16<NT>(rs, (o < hi && o + 16 > lo) ? o : kOobOffset);
  }
  const int oe = aoff + 16 * (k0 + 16 * U);
  E = __builtin_amdgcn_raw_buffer_load_b32(rs, (r == 15 && oe < hi && oe + 4 > lo) ? oe : kOobOffset, 0,
                                           WGCS_LD_AUX(NT));
}

// Wave-uniform: no lane of the wave has `pred` set (a scalar compare, no exec-mask branch).
__device__ __forceinline__ bool wave_none(bool pred) { return __builtin_amdgcn_ballot_w64(pred) == 0; }

// A row's source geometry for segment i: the dword-aligned window of its
// destination chunk 0 (job-relative offset aoff, byte shift sb), the job
// bytes [lo, hi) of its payload, its chunk count nk and packet length.
struct RowSrc {
  int aoff, sb, lo, hi, nk, pkt_len;
};
__device__ __forceinline__ RowSrc row_src(const uint8_t* rb, int i, int gso, int hdr_len, int plen, int dalign) {
  RowSrc g;
  const int seg_start = hdr_len + i * gso;
  const int seg_end = min(plen, seg_start + gso);
  g.pkt_len = hdr_len + (seg_end - seg_start);
  g.nk = (g.pkt_len + dalign + 15) >> 4;
  const uint8_t* w0 = rb + (int64_t)i * gso - dalign;  // source of destination chunk 0 (payload positions)
  g.sb = (int)((uintptr_t)w0 & 3u);
  g.aoff = (int)(w0 - g.sb - (rb - 10));               // its dword-aligned window, job-relative
  g.lo = 10 + seg_start;
  g.hi = 10 + seg_end;
  return g;
}

// One batch of a row's payload stream: destination chunk k = bytes [sb, sb +
// 16) of the dword-aligned source window k and the first dword of window k + 1
// (next lane, DPP row_ror).  Sums the L4 bytes [hdrLen, pktLen) from the same
// registers (v_dot2) and stores the payload bytes of every chunk (those of a
// chunk shared with the header as byte-exact pieces; the header phase stores
// the chunk's header bytes).
template <int U>
__device__ __forceinline__ void consume_batch(const uint4 (&A)[U], uint32_t E, int k0, const RowSrc& g, int hdr_len,
                                              int dalign, uint8_t* dbase, int r, uint32_t& acc) {
  const int pkt_len = g.pkt_len, nk = g.nk, sb = g.sb;
  uint32_t Rc = row_next(A[0].x);  // lane 15: lane 0's next-u dword
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int k = k0 + r + 16 * u;
    const uint32_t Rx = u + 1 < U ? row_next(A[u + 1 < U ? u + 1 : u].x) : E;
    const uint32_t nx = r == 15 ? Rx : Rc;
    Rc = Rx;
    const int x0 = 16 * k - dalign;
    const uint4 v = make_uint4(__builtin_amdgcn_alignbyte(A[u].y, A[u].x, sb),
                               __builtin_amdgcn_alignbyte(A[u].z, A[u].y, sb),
                               __builtin_amdgcn_alignbyte(A[u].w, A[u].z, sb),
                               __builtin_amdgcn_alignbyte(nx, A[u].w, sb));
    if (wave_none(x0 < hdr_len || x0 + 16 > pkt_len)) {
      // every chunk of this step in every row of the wave is whole payload
      // (the bulk of a segment): unmasked sum and a full store, no branches
      acc = add4(acc, v);
      int ko = 16 * k;
      asm volatile("" : "+v"(ko));
      st128(dbase + ko, v);
    } else if (k < nk) {
      if (x0 >= hdr_len && x0 + 16 <= pkt_len) acc = add4(acc, v);
      else acc = add4_masked(acc, v, byte_bits16(hdr_len - x0, pkt_len - x0), false);
      // the chunk's address formed here, not hoisted for all U chunks up front
      // (six 64-bit addresses held across the stream cost an occupancy step)
      int ko = 16 * k;
      asm volatile("" : "+v"(ko));
      store_chunk(dbase + ko, v, x0 - hdr_len, pkt_len - hdr_len);  // bytes [hdrLen, pktLen)
    }
  }
}

#ifndef WGCS_GSO_WT
#define WGCS_GSO_WT 1  // write-through full-chunk stores in gso_lds_kernel (0: plain stores, A/B builds)
#endif
#ifndef WGCS_GSO_WT_AUX
#define WGCS_GSO_WT_AUX 16  // the write-through stores' cache policy: 16 = sc1 (A/B builds: 0 plain, 2 nt, 17 sc0 sc1)
#endif
// Where gso_lds_kernel's row writes: its segment's destination chunks at
// dbase (= out + obase + dro), and, when `wt`, a buffer resource over the
// job's output region (out + obase) for write-through full-chunk stores
// (`sc1`: the line leaves L2 at once instead of staying dirty until the
// end-of-kernel writeback).  The stores go through the buffer intrinsic, not
// inline asm: the compiler then sees them (wait counts, and the hazard of a
// VALU overwriting a 16-byte store's data registers right behind it).
struct RowOut {
  uint4 keep;  // this lane's header-shared chunk's payload bytes (consume_batch_img)
  __amdgpu_buffer_rsrc_t rs;
  int dro;  // dbase - (out + obase), when wt
  bool wt;  // block-uniform: every offset of the job's output region fits the resource
};
__device__ __forceinline__ void store16_row(const RowOut& o, uint8_t* dbase, int ko, const uint4& v) {
  if (o.wt) {
    typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
    const u32x4v vv = {v.x, v.y, v.z, v.w};
    __builtin_amdgcn_raw_buffer_store_b128(vv, o.rs, o.dro + ko, 0, WGCS_GSO_WT_AUX);
  } else {
    st128(dbase + ko, v);
  }
}
// store_chunk with its full-chunk case through store16_row.
__device__ __forceinline__ void store_chunk_row(const RowOut& o, uint8_t* dbase, int ko, const uint4& v, int x0,
                                                int pkt_len) {
  if (x0 >= 0 && x0 + 16 <= pkt_len) store16_row(o, dbase, ko, v);
  else store_chunk(dbase + ko, v, x0, pkt_len);
}

// consume_batch for gso_lds_kernel.  A chunk the row shares with the header
// (x0 < hdrLen: only step 0 of the first batch, hdrLen + dalign <= 255) is not
// stored here: its payload bytes are kept in `keep` (lane r: chunk r) and
// finish_row stores them with the header bytes as one 16-byte store.  Whole
// payload chunks are stored write-through, the packet's last partial chunk as
// pieces.  The sums are consume_batch's.
template <int U>
__device__ __forceinline__ void consume_batch_img(const uint4 (&A)[U], uint32_t E, int k0, const RowSrc& g,
                                                  int hdr_len, int dalign, uint8_t* dbase, int r, uint32_t& acc,
                                                  RowOut& ro) {
  const int pkt_len = g.pkt_len, sb = g.sb;
  uint32_t Rc = row_next(A[0].x);  // lane 15: lane 0's next-u dword
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int k = k0 + r + 16 * u;
    const uint32_t Rx = u + 1 < U ? row_next(A[u + 1 < U ? u + 1 : u].x) : E;
    const uint32_t nx = r == 15 ? Rx : Rc;
    Rc = Rx;
    const int x0 = 16 * k - dalign;
    const uint4 v = make_uint4(__builtin_amdgcn_alignbyte(A[u].y, A[u].x, sb),
                               __builtin_amdgcn_alignbyte(A[u].z, A[u].y, sb),
                               __builtin_amdgcn_alignbyte(A[u].w, A[u].z, sb),
                               __builtin_amdgcn_alignbyte(nx, A[u].w, sb));
    int ko = 16 * k;
    asm volatile("" : "+v"(ko));
    if (wave_none(x0 < hdr_len || x0 + 16 > pkt_len)) {  // every chunk of the step whole payload
      acc = add4(acc, v);
      store16_row(ro, dbase, ko, v);
    } else {
      acc = add4_masked(acc, v, byte_bits16(hdr_len - x0, pkt_len - x0), false);
      if (u == 0) ro.keep = k0 == 0 ? v : ro.keep;
      if (x0 >= hdr_len && x0 < pkt_len) {
        if (x0 + 16 <= pkt_len) store16_row(ro, dbase, ko, v);
        else store_lo(dbase + ko, v, pkt_len - x0);  // the packet's last bytes
      }
    }
  }
}

// One row's whole payload stream, batch by batch.
template <int U, bool NT>
__device__ __forceinline__ void stream_row(const uint8_t* rb, int i, int gso, int hdr_len, int plen, int dalign,
                                           uint8_t* dbase, int r, uint32_t& acc, __amdgpu_buffer_rsrc_t rs) {
  const RowSrc g = row_src(rb, i, gso, hdr_len, plen, dalign);
  acc = 0;
  for (int k0 = 0; k0 < g.nk; k0 += 16 * U) {
    uint4 A[U];
    uint32_t E;
    load_windows<U, NT>(rs, g.aoff, k0, r, g.lo, g.hi, A, E);
    consume_batch<U>(A, E, k0, g, hdr_len, dalign, dbase, r, acc);
  }
}

// Byte `pos` (wave-uniform, < 16 * 16) of the header chunks in packet
// coordinates (lane r of each row holds readBuf[16r, 16r + 16)), from the
// wave's first row.
__device__ __forceinline__ uint32_t qdw(const uint4& Q, int dw) {  // dword dw (wave-uniform, < 64)
  return (uint32_t)__builtin_amdgcn_readlane((int)dword_at(Q, dw & 3), dw >> 2);
}
__device__ __forceinline__ uint32_t qbyte(const uint4& Q, int pos) { return (qdw(Q, pos >> 2) >> (8 * (pos & 3))) & 0xFFu; }
// Bytes [pos, pos + 4) as a little-endian u32 (two readlanes).
__device__ __forceinline__ uint32_t qle32(const uint4& Q, int pos) {
  const uint64_t w = ((uint64_t)qdw(Q, (pos >> 2) + 1) << 32) | qdw(Q, pos >> 2);
  return (uint32_t)(w >> (8 * (pos & 3)));
}
// The decoded path's decoder (wave 0 of the block): handleVirtioRead's /
// gsoSplit's checks and geometry (decode_job) and the job-constant header
// sums (header_fast), published in `ji`; count / status of the job.  Kept out
// of line: the rare path's registers do not count against the clean path's.
__device__ __noinline__ void decode_publish(const uint8_t* vb, uint32_t jlen, uint32_t jflags, uint32_t room,
                                            uint32_t max_segs, int lane, JobInfo* jip, bool first_block,
                                            int32_t* count_j, int32_t* status_j) {
  JobInfo& ji = *jip;
  __builtin_amdgcn_s_setprio(3);
  HdrBytes hb;
  hb.load(vb, (int)min(jlen, 256u), lane);
  const Job jd = decode_job(hb, jlen, jflags, room, max_segs);
  const bool ok = jd.status == 0 || jd.status == WGCS_ERR_TOO_MANY_SEGMENTS;
  uint32_t fst = 0, i0 = 0, q0 = 0;
  HdrFast hf = {};
  if (ok && jd.nseg > 0 && jd.type != GSO_NONE && !jd.gen) {
    hf = header_fast(hb, jd, lane);
    // readBuf bytes after gsoSplit zeroed the L4 checksum field (gro.go:1393;
    // the IPv4 checksum bytes 10-11 are neither id nor seq here: cs >= 20)
    const int ca = (jd.cs + jd.co) & 0xFFFF;
    auto zb = [&](int x) { return (x == ca || x == ca + 1) ? 0u : hb(10 + x); };
    const int sq = jd.cs + 4;
    i0 = jd.ipv == 4 ? (zb(4) << 8) | zb(5) : 0u;
    q0 = jd.type != GSO_UDP_L4 ? (zb(sq) << 24) | (zb(sq + 1) << 16) | (zb(sq + 2) << 8) | zb(sq + 3) : 0u;
    fst = hf.fast ? 1u : 0u;
  }
  if (lane == 0) {
    ji.status = jd.status;
    ji.count = ok ? jd.count : 0;
    ji.nseg = ok ? jd.nseg : 0;
    ji.shape = (uint32_t)(jd.type & 0xFF) | ((uint32_t)(jd.ipv & 0xFF) << 8) |
               ((uint32_t)(jd.gen ? 1 : 0) << 16) | (fst << 24);
    ji.hdr_len = jd.hdr_len;
    ji.gso = jd.gso;
    ji.cs = jd.cs;
    ji.co = jd.co;
    ji.plen = jd.plen;
    ji.flags = jd.flags;
    ji.id0 = i0;
    ji.seq0 = q0;
    ji.ip_base = fold32_16(hf.ip_base);
    ji.l4_base = fold32_16(hf.l4_base) + fold32_16(hf.addr);
    ji.tflags = hf.flags;
    if (first_block) {
      *count_j = ok ? jd.count : 0;
      *status_j = jd.status;
    }
  }
  __builtin_amdgcn_s_setprio(0);
}

// Row-per-segment split.  Block = 4 waves = 16 rows = 16 consecutive output
// segments of one job; grid = (job, segment group).
//
// Clean jobs (the common case) need no decode step and no barrier.  Every
// wave reads the virtio header (one wave-uniform load) and derives the split
// geometry; when that geometry takes the row-streaming path and its first
// segment fits the caller's room, handleVirtioRead's and gsoSplit's checks
// (tun/tun.go:557-631, gro.go:1387-1410) can fail only through the TCP data
// offset, which the wave reads from the header chunks it loads anyway
// (hdrLen = csumStart + dataOffset, tun.go:601-614).  Such a job's status is
// 0 or ErrTooManySegments from the segment count alone, and each row
// computes the header sums it needs from its own header chunks.  The row
// streams its payload (loads issued right after the virtio header arrives),
// then rewrites and stores its header chunks.
//
// Every other job (GSO_NONE, errors, unusual geometry) takes the decoded
// path: wave 0 runs decode_job and the job-constant sums and publishes them
// through LDS; after the barrier each row follows that verdict (nothing on an
// error, the byte-granular general path, or the stream with the decoded
// geometry and the general header path).
// The segment's header chunk and checksums, given the row's payload sum
// `acc` and the job-constant header values: on the fast layout the header
// chunk in packet coordinates (Q) rewritten field by field and shifted to the
// destination phase; otherwise a byte-exact replay of the reference's write
// order on the chunk in destination coordinates.  Stores the header bytes
// [0, hdrLen) of the segment (the stream stored the rest) and its size.
__device__ __forceinline__ void finish_row(bool fast, const uint4 Q, int type, int ipv, int hdr_len, int gso, int cs,
                                           int co, int plen, int i, int r, int dalign, const uint8_t* dst,
                                           uint8_t* dbase, uint32_t acc, uint32_t ip_base, uint32_t l4_base,
                                           uint32_t tflags, uint32_t id0, uint32_t seq0, int32_t* size_out,
                                           const RowOut* ro = nullptr) {
  const uint4 z = make_uint4(0, 0, 0, 0);
  // ---- segment geometry (row-uniform)
  const bool v4 = ipv == 4, tcp = type != GSO_UDP_L4;
  const int csum_at = (cs + co) & 0xFFFF;
  const int seg_start = hdr_len + i * gso;
  const int seg_end = min(plen, seg_start + gso);
  const int seg_len = seg_end - seg_start;
  const int pkt_len = hdr_len + seg_len;
  const bool last = seg_end == plen;
  const int nk = (pkt_len + dalign + 15) >> 4;
  const int hk = min((hdr_len + dalign + 15) >> 4, nk);
  const uint32_t id = i > 0 ? ((id0 + 1) & 0xFFFFu) : id0;  // quirk: id0 + 1 for every i >= 1 (:1426-1431)
  const uint32_t seq = seq0 + (uint32_t)(uint16_t)((uint16_t)gso * (uint16_t)i);  // uint16 product (:1445)
  const uint32_t ulen = (uint32_t)(uint16_t)(seg_len + (hdr_len - cs));           // UDP length (:1462-1465)
  const uint32_t tlen = (uint32_t)(uint16_t)(hdr_len - cs + seg_len);             // transportLen (:1469-1471)
  const uint32_t proto = tcp ? 6u : 17u;
  const int x0h = 16 * r - dalign;

  if (fast) {
    // ---- sums: payload (row reduction) + job constants + rewritten fields
    uint32_t t_pay = fold32_16(row16_sum_u32(acc));
    if ((((uintptr_t)dst + (uintptr_t)cs) & 1u) == 0) t_pay = bswap16(t_pay);  // pairing from csumStart
    const uint32_t var = tcp ? (seq >> 16) + (seq & 0xFFFFu) + (last ? (tflags & 0x09u) : 0u) : ulen;
    const uint32_t l4c = (~fold32_16(t_pay + l4_base + var + proto + tlen)) & 0xFFFFu;
    // ---- header chunk in packet coordinates, rewritten (gro.go:1418-1465, :1486-1490)
    uint4 P = Q;
    if (v4) {
      const uint32_t ipc = (~fold32_16(ip_base + (uint32_t)pkt_len + id)) & 0xFFFFu;
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
    // ---- to the destination phase (previous chunk of the row: DPP row_shr:1),
    // merged with the payload bytes, stored
    const uint4 Pp = row_prev4(P);
    const uint4 D = dalign ? funnel_v(Pp, P, 16 - dalign) : P;
    if (ro) {
      // gso_lds_kernel: the stream kept these chunks' payload bytes
      // (consume_batch_img); header and payload go out as one store
      if (r < hk)
        store_chunk_row(*ro, dbase, 16 * r, select_bytes(D, ro->keep, byte_bits16(-x0h, hdr_len - x0h)), x0h, pkt_len);
    } else if (r < hk) {
      store_chunk(dbase + 16 * r, D, x0h, hdr_len);  // header bytes [0, hdrLen)
    }
  } else {
    // ---- general header path (unusual csum offsets): byte-exact replay of
    // the reference's write order on the chunk (destination coordinates)
    const int a_lo = v4 ? 12 : 8, a_hi = v4 ? 20 : 40;
    uint32_t acc_ip = 0;
    uint4 hv = z;
    if (r < hk) {
      hv = Q;
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
      store_chunk(dbase + 16 * r, hv, x0h, hdr_len);  // header bytes [0, hdrLen)
    }
  }
  if (r == 0) *size_out = pkt_len;
}

// Every job that is not clean (GSO_NONE, errors, unusual geometry): wave 0
// runs the full validation (decode_publish) and publishes its verdict through
// LDS, the rows follow it.  Out of line, so that its registers do not count
// against the clean path's occupancy (it spills, if at all, only here).
// Returns the job's live segment count from the published verdict (0 for an
// error, GSO_NONE or no segment): block-uniform, so the caller's group loop
// stops after the last group that holds a segment.
template <int U, bool NT>
__device__ __noinline__ int decoded_rows(const uint8_t* vb_a, uint32_t jlen_a, uint32_t jflags_a, uint32_t room,
                                          uint32_t max_segs, int i, bool first_block, int32_t* count_j,
                                          int32_t* status_j, uint8_t* out0, uint8_t* dst, int32_t* sizes_j,
                                          uint32_t tails_a) {
  __shared__ JobInfo ji;
  const uint4 z = make_uint4(0, 0, 0, 0);
  const int lane = threadIdx.x & 63;
  const int r = lane & 15;
  const int wv = threadIdx.x >> 6;
  // the job's values are wave-uniform (arguments arrive in VGPRs)
  const uint64_t vbu = ((uint64_t)(uint32_t)ufl((int)(uint32_t)(uintptr_t)vb_a)) |
                       ((uint64_t)(uint32_t)ufl((int)(uint32_t)((uintptr_t)vb_a >> 32)) << 32);
  const uint8_t* vb = reinterpret_cast<const uint8_t*>(vbu);
  const uint32_t jlen = (uint32_t)ufl((int)jlen_a), jflags = (uint32_t)ufl((int)jflags_a);
  const uint8_t* rb = vb + 10;
  const int dalign = (int)((uintptr_t)dst & 15u);
  uint8_t* dbase = dst - dalign;
  const int hph = (int)((uintptr_t)rb & 15u);
  const uint8_t* hab = rb - hph + 16 * r;
  // ---- decoded path: wave 0 decodes, every wave follows its verdict
  if (wv == 0) decode_publish(vb, jlen, jflags, room, max_segs, lane, &ji, first_block, count_j, status_j);
  lds_barrier();  // the decoder's verdict
  const int st = ufl(ji.status);
  const int nseg = ufl(ji.nseg);
  const uint32_t shape = (uint32_t)ufl((int)ji.shape);
  const int type = (int)(shape & 0xFFu);
  if ((st != 0 && st != WGCS_ERR_TOO_MANY_SEGMENTS) || nseg == 0) return 0;
  const int plen = ufl(ji.plen);
  if (type == GSO_NONE) {  // one packet into bufs[0], by wave 0 of the job's first block
    if (first_block && wv == 0) {
      Job jn = {};
      jn.flags = ufl(ji.flags);
      jn.cs = ufl(ji.cs);
      jn.co = ufl(ji.co);
      jn.plen = plen;
      none_segment(rb, jn, out0, lane);
      if (lane == 0) *sizes_j = plen;
    }
    return 0;
  }
  if (i >= nseg) return nseg;  // whole rows retire; DPP below stays inside live rows
  const int ipv = (int)((shape >> 8) & 0xFFu);
  const bool fast = (shape >> 24) != 0;
  const int hdr_len = ufl(ji.hdr_len);
  const int gso = ufl(ji.gso);
  const int cs = ufl(ji.cs);
  const int co = ufl(ji.co);
  if ((shape >> 16) & 0xFFu) {  // block-uniform
    gso_general_row(rb, plen, type, ipv, hdr_len, gso, cs, co, i, dst, r, sizes_j + i, ufl((int)tails_a) != 0);
    return nseg;
  }
  uint32_t acc = 0;
  stream_row<U, NT>(rb, i, gso, hdr_len, plen, dalign, dbase, r, acc, job_rsrc(vb, jlen));
  // header chunks: packet coordinates on the fast layout, destination
  // coordinates for the general header path
  const uint8_t* hend = rb + hdr_len;
  const int hphd = (int)((uintptr_t)(rb - dalign) & 15u);
  const uint8_t* hb2 = fast ? hab : rb - dalign - hphd + 16 * r;
  uint4 H0 = z, H1 = z;
  if (hb2 < hend && hb2 + 16 > rb) H0 = ld16(hb2);
  if (hb2 + 16 < hend && hb2 + 32 > rb) H1 = ld16(hb2 + 16);
  const uint4 Q = fast ? funnel(H0, H1, hph) : funnel_v(H0, H1, hphd);
  const uint32_t ip_base = (uint32_t)ufl((int)ji.ip_base);
  const uint32_t l4_base = (uint32_t)ufl((int)ji.l4_base);
  const uint32_t tflags = (uint32_t)ufl((int)ji.tflags);
  const uint32_t id0 = (uint32_t)ufl((int)ji.id0);
  const uint32_t seq0 = (uint32_t)ufl((int)ji.seq0);
  finish_row(fast, Q, type, ipv, hdr_len, gso, cs, co, plen, i, r, dalign, dst, dbase, acc, ip_base, l4_base, tflags,
             id0, seq0, sizes_j + i);
  return nseg;
}

// Build-time tunables (defaults measured on cfg4):
// payload windows per lane in flight, and the occupancy the kernel is compiled
// for.  The out-of-line decoded path would otherwise set the register count
// (151 VGPRs, 3 waves per SIMD); at 5 waves (<= 96 VGPRs) the clean path runs
// without spills and the decoded path spills only inside its own call.
#ifndef WGCS_GSO_U
#define WGCS_GSO_U 6
#endif
#ifndef WGCS_GSO_WAVES
#define WGCS_GSO_WAVES 5
#endif
#ifndef WGCS_GSO_GROUPS
#define WGCS_GSO_GROUPS 3  // blocks per job (grid y); each takes every WGCS_GSO_GROUPS-th segment group
#endif
// One (job, segment-group set) of gso_rows_kernel: block `by` of `gy` blocks
// per job takes the job's segment groups by, by + gy, ...  The descriptor and
// output position come by value (the resident ring kernel passes a request's,
// gso_rows_kernel its grid's); `has_pos`: use pos, else fixed slots.
// 16 bytes at a 4-byte aligned generic pointer that points into LDS (ds reads)
__device__ __forceinline__ uint4 lds16_a4(const uint8_t* p) {
  typedef __attribute__((address_space(3))) const uint32_t l32;
  const l32* q = (const l32*)(const __attribute__((address_space(3))) uint8_t*)p;
  return make_uint4(q[0], q[1], q[2], q[3]);
}

template <int U, bool NT, int ROWS = 16>
__device__ __forceinline__ void gso_rows_body(const uint8_t* arena, const wgcs_gso_job job, uint32_t jb, int by,
                                              int gy, uint32_t max_segs, uint8_t* out, uint32_t out_stride,
                                              bool has_pos, const GsoOutPos pos, uint32_t offset, uint32_t room,
                                              int32_t* sizes, int32_t* count, int32_t* status,
                                              const uint8_t* hlds = nullptr) {
  static_assert(ROWS % 4 == 0, "4 rows per wave");  // ROWS = 4 x the workgroup's waves
#ifdef WGCS_GSO_STAMPS  // timing-only build (scripts/probe_gso_stamps.py): s_memrealtime per wave phase
  uint64_t stp[5] = {__builtin_amdgcn_s_memrealtime(), 0, 0, 0, 0};
#endif
  const int lane = threadIdx.x & 63;
  const int r = lane & 15;
  const int wv = threadIdx.x >> 6;
  const uint8_t* vb = arena + job.off;
  const uint32_t jlen = job.len;
  const uint8_t* rb = vb + 10;
  const uint64_t slot0 = (uint64_t)jb * max_segs;  // sizes[] index of segment 0
  // segment i of this job at out + obase + i * opitch (+ offset): fixed slots,
  // or the caller's packed per-job layout (the stager's compact D2H region)
  uint64_t obase = slot0 * out_stride;
  uint32_t opitch = out_stride;
  uint32_t tails = 1;  // gsoSplit's header writes past a segment's end (GsoOutPos)
  if (has_pos) {
    obase = pos.base;
    opitch = pos.pitch;
    tails = pos.flags & kOutPosTails;
  }
  // ---- header chunks in packet coordinates (lane r of each row: the
  // dword-aligned 16-byte window r from the dword holding readBuf[0]; shifted
  // to readBuf[16r, 16r + 16) with the next lane's first dword below), issued
  // first: they need only the descriptor.  A raw buffer load over the job's
  // bytes: windows past the job read as zeros.  Lane 15's last bytes
  // (readBuf[253..255]) come from the wrong lane; every use of the chunks is
  // below hdrLen <= 240.
  const int hph = (int)((uintptr_t)rb & 3u);
  const uint8_t* hbase = rb - hph;
  const __amdgpu_buffer_rsrc_t hrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(hbase), (short)0, (int)(jlen + 3u) - (int)(hbase - vb), 0x00020000);
  // (hlds: the resident ring's copy of vb[0, 272) in LDS, vb[k] at hlds[k],
  // same phase mod 16 as vb -- the header without a host-memory round trip)
  const uint4 H0 = hlds ? lds16_a4(hlds + (hbase - vb) + 16 * r) : bld16<false>(hrs, 16 * r);

  // ---- virtio header + the IP version byte: 16 bytes from the dword below
  // vb, one wave-uniform load (readable: jlen >= 14 and the arena contract)
  const bool raw = (job.flags & WGCS_GSO_JOB_RAW) != 0;
  const int plen_s = jlen > 10 ? (int)jlen - 10 : 0;
  uint32_t t1 = 0, hl = 0, g = 0, c = 0, o = 0, b0 = 0;
  if (jlen >= 14) {
    const int sh = (int)((uintptr_t)vb & 3u);
    // a range-checked vector load (zeros past the job), not a scalar one: the
    // resident ring kernel reads requests that change at the same address
    const uint4 w = hlds ? lds16_a4(hlds - sh)
                         : bld16<false>(__builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(vb - sh), (short)0,
                                                                          (int)(jlen + 3u + (uint32_t)sh), 0x00020000),
                                        0);
    const uint64_t lo = ((uint64_t)w.y << 32) | w.x, hi = ((uint64_t)w.w << 32) | w.z;
    // bytes [sh, sh + 11) of the 16: the virtio header and readBuf[0]
    const uint64_t v0 = sh ? (lo >> (8 * sh)) | (hi << (64 - 8 * sh)) : lo;  // vb[0..8)
    const uint64_t v1 = hi >> (8 * sh);                                      // vb[8..)
    t1 = (uint32_t)(v0 >> 8) & 0xFFu;
    hl = (uint32_t)(v0 >> 16) & 0xFFFFu;
    g = (uint32_t)(v0 >> 32) & 0xFFFFu;
    c = (uint32_t)(v0 >> 48) & 0xFFFFu;
    o = (uint32_t)v1 & 0xFFFFu;
    b0 = (uint32_t)(v1 >> 16) & 0xFFu;
  }
  const int type_s = raw ? ((t1 == GSO_TCPV4 || t1 == GSO_TCPV6) ? (int)t1 : GSO_UDP_L4) : (int)t1;
  const int ipv_s = raw ? ((job.flags & WGCS_GSO_JOB_V6) ? 6 : 4) : (int)(b0 >> 4);
  const bool tcp_s = type_s != GSO_UDP_L4;
  const bool ok_s = jlen >= 14 && g != 0 &&
                    (type_s == GSO_TCPV4 || type_s == GSO_TCPV6 || type_s == GSO_UDP_L4) &&
                    ((ipv_s == 4 && type_s != GSO_TCPV6) || (ipv_s == 6 && type_s != GSO_TCPV4));
  const int gso_s = (int)g, cs_s = (int)c, co_s = (int)o;
  const int hdr_s = (raw || tcp_s) ? (int)hl : ((cs_s + 8) & 0xFFFF);
  const int ca_s = (cs_s + co_s) & 0xFFFF;
  const int pkt0_s = hdr_s + min(gso_s, plen_s - hdr_s);  // segment 0, the largest
  const bool clean_s = ok_s && hdr_s < plen_s && cs_s >= (ipv_s == 4 ? 20 : 40) && ca_s + 2 <= hdr_s &&
                       hdr_s <= kMaxHdrLen && (raw || !tcp_s || (hdr_s - cs_s >= 20 && hdr_s - cs_s <= 60)) &&
                       fast_header(cs_s, hdr_s, ca_s, tcp_s) && (uint32_t)pkt0_s <= room;
  // Row i of a clean job holds a segment iff i < max_segs and hdrLen + i *
  // gsoSize < len(readBuf) (i < ceil((plen - hdrLen) / gsoSize)): a multiply,
  // no division, on the clean path.
  auto has_seg = [&](int i) { return i < (int)max_segs && hdr_s + (int64_t)i * gso_s < plen_s; };
  // Segment groups: this block takes groups blockIdx.y, + gridDim.y, ... of
  // the job's ceil(max_segs / 16).  The grid has only a few blocks per job
  // (callers size bufs for the largest read, conn.IdealBatchSize = 128 slots,
  // so most groups of a 64-KiB read are empty): groups past the job's last
  // segment under every verdict cost no dispatch and are never entered.
  // hdrLen >= csumStart + 20 (TCP, tun.go:608-613) or = csumStart + 8 (UDP) or
  // the virtio value (raw jobs) bounds the segment count from above.  Group 0
  // always runs: it writes count / status and the GSO_NONE packet.
  // Groups that may hold a segment: gbound = max(1, min(ngroups, ceil(nbound /
  // 16))) with nbound = ceil((plen - hmin) / gsoSize); group y < gbound iff y
  // == 0 or (y < ngroups and 16 y gsoSize < plen - hmin).
  const int ngroups = (int)((max_segs + ROWS - 1) / ROWS);
  const int hmin = raw ? (int)hl : (tcp_s ? cs_s + 20 : cs_s + 8);
  const bool split_type = jlen >= 14 && ok_s && cs_s + 60 <= 0xFFFF;
  const bool gso_none = jlen >= 14 && !raw && t1 == GSO_NONE;
  auto group_live = [&](int y) {
    if (y == 0) return true;
    if (gso_none || y >= ngroups) return false;
    return !split_type || (plen_s > hmin && hmin + (int64_t)y * ROWS * gso_s < plen_s);
  };
  if (!group_live(by)) return;
#ifdef WGCS_GSO_HEAD_MIN  // timing-only build: descriptor + virtio header + verdict inputs, nothing else
  if (threadIdx.x == 0 && by == 0) count[jb] = ok_s ? 45 : 0;
  if (threadIdx.x == 0 && by == 0) status[jb] = clean_s ? 0 : 1;
  return;
#endif

  uint4 Q;  // readBuf[16r, 16r + 16) (bytes below hdrLen)
  {
    const uint32_t nx = row_next(H0.x);
    Q = make_uint4(__builtin_amdgcn_alignbyte(H0.y, H0.x, hph), __builtin_amdgcn_alignbyte(H0.z, H0.y, hph),
                   __builtin_amdgcn_alignbyte(H0.w, H0.z, hph), __builtin_amdgcn_alignbyte(nx, H0.w, hph));
  }
  // the TCP data offset decides hdrLen (tun.go:601-614): block-uniform verdict
  bool clean = clean_s;
  if (clean && tcp_s && !raw) {
    const int th = (int)((qbyte(Q, cs_s + 12) >> 4) * 4);
    clean = ((cs_s + th) & 0xFFFF) == hdr_s;
  }

  // The payload loads are issued only after this verdict: no payload window
  // is live across the decoded path's call, so the clean path's registers
  // stay its own (the verdict waits on the header chunks, which arrive with
  // the virtio header).  readfirstlane makes the branch provably uniform.
  if (ufl(clean ? 1 : 0)) {
    if (by == 0 && threadIdx.x == 0) {  // the checks can only end in the segment count here
      const int nfull_s = (plen_s - hdr_s + gso_s - 1) / gso_s;
      const bool many = nfull_s > (int)max_segs;
      count[jb] = many ? (int)max_segs - 1 : nfull_s;
      status[jb] = many ? WGCS_ERR_TOO_MANY_SEGMENTS : 0;
    }
#ifdef WGCS_GSO_HEAD_VERDICT  // timing-only build: the head up to the verdict (no job sums, no stream)
    return;
#endif
    const int type = type_s, ipv = ipv_s, hdr_len = hdr_s, gso = gso_s, cs = cs_s, co = co_s, plen = plen_s;
    // job-constant header sums from this row's own header chunks (header_fast's
    // values): IPv4 header without total length / id / checksum, the L4
    // header from csumStart without checksum field, seq / UDP length and the
    // flags byte, and the pseudo-header addresses, each as BE words
    uint32_t ip_base = 0, l4_base = 0, tflags = 0, id0 = 0, seq0 = 0;
    {
      const int x0 = 16 * r;
      const bool tcp_c = type != GSO_UDP_L4;
      const int vlo = cs + 4, vhi = tcp_c ? cs + 8 : cs + 6;
      const int ca = (cs + co) & 0xFFFF;
      if (ipv == 4) {
        const uint32_t m = byte_bits16(-x0, cs - x0) & ~byte_bits16(2 - x0, 6 - x0) & ~byte_bits16(10 - x0, 12 - x0);
        ip_base = (uint32_t)ufl((int)bswap16(fold32_16(row16_sum_u32(add4_masked(0u, Q, m, false)))));
      }
      uint32_t ml4 = byte_bits16(cs - x0, hdr_len - x0) & ~byte_bits16(ca - x0, ca + 2 - x0) &
                     ~byte_bits16(vlo - x0, vhi - x0);
      if (tcp_c) ml4 &= ~byte_bits16(cs + 13 - x0, cs + 14 - x0);
      const int a_lo = ipv == 4 ? 12 : 8, a_hi = ipv == 4 ? 20 : 40;
      uint32_t s4 = add4_masked(0u, Q, ml4, false);
      s4 = add4_masked(s4, Q, byte_bits16(a_lo - x0, a_hi - x0), (cs & 1) != 0);
      uint32_t t4 = fold32_16(row16_sum_u32(s4));
      if ((cs & 1) == 0) t4 = bswap16(t4);  // pairing from csumStart (packet coordinates)
      if (tcp_c) tflags = qbyte(Q, cs + 13);
      l4_base = (uint32_t)ufl((int)t4) + (tflags & ~0x09u);
      if (ipv == 4) {
        const uint32_t b45 = qdw(Q, 1);  // readBuf[4:8)
        id0 = ((b45 & 0xFFu) << 8) | ((b45 >> 8) & 0xFFu);
      }
      if (tcp_c) seq0 = __builtin_bswap32(qle32(Q, vlo));
    }
#ifdef WGCS_GSO_STAMPS
    stp[1] = __builtin_amdgcn_s_memrealtime();
#endif
#ifdef WGCS_GSO_HEADONLY  // timing-only build: the head (decode, verdict, job sums) and nothing else
    if (ufl((int)(ip_base + l4_base + tflags + id0 + seq0)) == 0x7FFFFFFF) sizes[slot0] = 0;
    return;
#endif
    for (int grp = by; has_seg(grp * ROWS); grp += gy) {  // block-uniform
      const int i = grp * ROWS + wv * 4 + (lane >> 4);  // this row's segment
      if (has_seg(i)) {  // row-uniform
        uint8_t* dst = out + obase + (uint64_t)i * opitch + offset;
        const int dalign = (int)((uintptr_t)dst & 15u);
        uint8_t* dbase = dst - dalign;
        // ---- the payload stream
        uint32_t acc = 0;
        stream_row<U, NT>(rb, i, gso, hdr_len, plen, dalign, dbase, r, acc, job_rsrc(vb, jlen));
#ifdef WGCS_GSO_STAMPS
        stp[2] = __builtin_amdgcn_s_memrealtime();
#endif
        finish_row(true, Q, type, ipv, hdr_len, gso, cs, co, plen, i, r, dalign, dst, dbase, acc, ip_base, l4_base,
                   tflags, id0, seq0, &sizes[slot0 + (uint32_t)i]);
#ifdef WGCS_GSO_STAMPS
        stp[3] = __builtin_amdgcn_s_memrealtime();
#endif
      }
    }
#ifdef WGCS_GSO_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stp[4] = __builtin_amdgcn_s_memrealtime();
    if (lane == 0 && max_segs >= 128) {
      int32_t* sp = sizes + slot0 + 64 + (by * 4 + wv) * 5;
      for (int k = 0; k < 5; ++k) sp[k] = (int32_t)(uint32_t)stp[k];
    }
#endif
  } else {
    for (int grp = by; group_live(grp); grp += gy) {  // block-uniform
      const int i = grp * ROWS + wv * 4 + (lane >> 4);
      uint8_t* dst = out + obase + (uint64_t)i * opitch + offset;
      const int live = decoded_rows<U, NT>(vb, jlen, job.flags, room, max_segs, i, grp == 0, &count[jb], &status[jb],
                                           out + obase + offset, dst, &sizes[slot0], tails);
      lds_barrier();  // every wave is done with this group's verdict before the next one is published
      // the verdict bounds the job's segments (0 for an error / GSO_NONE): no
      // decode + barrier round for groups past it, whatever max_segs is
      if ((int64_t)(grp + gy) * ROWS >= (int64_t)ufl(live)) break;
    }
  }
}

#ifndef WGCS_RING_TU  // the batch kernels and their launchers: gso_kernels.hip only
template <int U, bool NT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WGCS_GSO_WAVES, 8))) void gso_rows_kernel(const uint8_t* __restrict__ arena,
                                                       const wgcs_gso_job* __restrict__ jobs, uint32_t max_segs,
                                                       uint8_t* __restrict__ out, uint32_t out_stride,
                                                       const GsoOutPos* __restrict__ outpos, uint32_t offset,
                                                       uint32_t room, int32_t* __restrict__ sizes,
                                                       int32_t* __restrict__ count, int32_t* __restrict__ status) {
  const uint32_t jb = blockIdx.x;
  const GsoOutPos pos = outpos ? outpos[jb] : GsoOutPos{};
  gso_rows_body<U, NT>(arena, jobs[jb], jb, (int)blockIdx.y, (int)gridDim.y, max_segs, out, out_stride,
                       outpos != nullptr, pos, offset, room, sizes, count, status);
}

#endif  // !WGCS_RING_TU
#ifdef WGCS_RING_TU  // the ring kernel: ring_kernels.hip only
// ---------------------------------------------------------------------------
// The resident per-call ring (round 6).  A launch plus a
// completion wait costs ~20 us per Go call, more than the Go
// code of one Tun.Read.  ring_kernel stays resident on a few CUs instead:
// thread 0 of every workgroup polls the request word in coherent pinned host
// memory (system-scope loads, s_sleep between polls), the workgroups run the
// request -- checksumValid of one packet (workgroup 0's first wave) or one
// handleVirtioRead (gso_rows_body: workgroup b takes segment groups b, b + nb,
// ...) -- reading the request bytes from coherent host memory and writing the
// results there, then each workgroup releases its stores at system scope and
// adds 1 to the completion word the host spins on.  Every wave leaves the
// loop on the stop word or when no request came for `idle_ticks` of
// s_memrealtime (100 MHz), so no launch can outlive its use.

typedef uint32_t u32x4s __attribute__((ext_vector_type(4)));

// checksumValid(pkt, iphLen, proto, isV6) (gro.go:554-612) by one wave: the
// batch kernel's VALIDATE arithmetic (checksum_kernels.hip) over every chunk
// with byte masks -- the main range pkt[iphLen:len] paired from iphLen, the
// pseudo-header addresses paired from their own start (rotl8 when the two
// parities differ) -- then proto + (len - iphLen).  Loads are system-scope
// (sc0 sc1) buffer loads: the bytes change between requests at one address.
__device__ uint32_t ring_validate(const uint8_t* pkt, int len, int cs, int proto, bool v6) {
  const int lane = threadIdx.x & 63;
  const int main_lo = min(cs, len), main_hi = len;
  const int addr_lo = v6 ? 8 : 12, addr_hi = v6 ? 40 : 20;
  const uintptr_t pbase = (uintptr_t)pkt;
  const bool rot_addr = (((pbase + (uintptr_t)addr_lo) ^ (pbase + (uintptr_t)main_lo)) & 1u) != 0;
  const int lo_all = min(main_lo, addr_lo), hi_all = max(main_hi, addr_hi);
  const int rel0 = lo_all - (int)((pbase + (uintptr_t)lo_all) & 15u);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(pkt + rel0), (short)0,
                                                                      hi_all - rel0, 0x00020000);
  uint32_t acc = 0;
  for (int c = lane; rel0 + 16 * c < hi_all; c += 64) {
    const int pos = rel0 + 16 * c;
    const auto t = __builtin_amdgcn_raw_buffer_load_b128(rs, 16 * c, 0, 17);
    const uint32_t w[4] = {t[0], t[1], t[2], t[3]};
    const uint32_t m16 = byte_bits16(main_lo - pos, main_hi - pos);
    const uint32_t a16 = byte_bits16(addr_lo - pos, addr_hi - pos);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      acc = add_halves(acc, w[k] & expand_nibble((m16 >> (4 * k)) & 0xFu));
      uint32_t y = w[k] & expand_nibble((a16 >> (4 * k)) & 0xFu);
      if (rot_addr) y = rotl8(y);
      acc = add_halves(acc, y);
    }
    acc = (acc >> 16) + (acc & 0xFFFFu);
  }
  uint32_t s = fold32_16(wave_sum_u32(fold32_16(acc)));
  if (((pbase + (uintptr_t)main_lo) & 1u) == 0) s = bswap16(s);
  const uint32_t t = fold32_16(s + (uint32_t)proto + ((uint32_t)(len - cs) & 0xFFFFu));
  return (t == 0xFFFFu && cs <= len) ? 1u : 0u;
}

// checksumValid of an inline request from the poll's registers: lane l of
// load j holds chunk 64 j + l, i.e. payload bytes [12 p, 12 p + 12) for
// p = 64 j + l - 8 >= 0 in its words 1-3 (word 0 is seq).  Every word starts
// at an offset that is a multiple of 4, so the 16-bit pairing is the
// packet's own; bytes past what the host wrote are masked off (main range
// [iphLen, len), addresses within the bytes carried).
__device__ uint32_t ring_validate_inline(const u32x4s (&x)[3], int len, int cs, int proto, bool v6) {
  const int lane = threadIdx.x & 63;
  const int main_lo = min(cs, len), main_hi = len;
  const int addr_lo = v6 ? 8 : 12, addr_hi = v6 ? 40 : 20;
  const bool rot_addr = ((addr_lo ^ main_lo) & 1) != 0;
  uint32_t acc = 0;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int p = 64 * j + lane - 8;
    if (p >= 0) {
#pragma unroll
      for (int m = 1; m < 4; ++m) {
        const int b0 = 12 * p + 4 * (m - 1);
        const uint32_t w = x[j][m];
        acc = add_halves(acc, w & expand_nibble(byte_bits16(main_lo - b0, main_hi - b0) & 0xFu));
        uint32_t y = w & expand_nibble(byte_bits16(addr_lo - b0, addr_hi - b0) & 0xFu);
        if (rot_addr) y = rotl8(y);
        acc = add_halves(acc, y);
      }
    }
  }
  uint32_t s = fold32_16(wave_sum_u32(fold32_16(acc)));
  if ((main_lo & 1) == 0) s = bswap16(s);
  const uint32_t t = fold32_16(s + (uint32_t)proto + ((uint32_t)(len - cs) & 0xFFFFu));
  return (t == 0xFFFFu && cs <= len) ? 1u : 0u;
}

__global__ __launch_bounds__(256) void ring_kernel(RingCtl* ctl, uint32_t last0, uint64_t idle_ticks) {
  __shared__ uint32_t s_q, s_valid;
  __shared__ uint32_t s_w[32];  // the request record's words
  __shared__ __attribute__((aligned(16))) uint32_t s_hdr[3 * kRingHdrChunks];  // a virtio read's first bytes
  RingReq* const rq = &ctl->req;
  uint32_t last = last0;
  uint64_t t_last = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    if (threadIdx.x < 64) {
      // wave 0 polls the record and the inline payload after it with three
      // system-scope 16-B loads per lane (chunk 64 j + lane) per poll, so the
      // request's fields -- and an inline packet -- arrive with its number:
      // one PCIe round trip, not one per field
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(rq, (short)0, (int)(16 * kRingPollChunks),
                                                                          0x00020000);
      const int lane = threadIdx.x;
      uint32_t q = 0;
      // 0: keep polling; 1: a new untorn record (and payload); 2: stop / idle deadline
      auto check = [&](const u32x4s (&x)[3]) -> int {
        q = (uint32_t)__builtin_amdgcn_readlane((int)x[0][0], 0);
        if (__builtin_amdgcn_readlane((int)x[0][kRqStop & 3], 0) != 0) return 2;
        // all eight chunks carry the same new seq: an untorn record
        const bool same = __builtin_amdgcn_ballot_w64(lane < 8 && x[0][0] != q) == 0;
        if (q != last && same) {
          const uint32_t op = (uint32_t)__builtin_amdgcn_readlane((int)x[0][kRqOp & 3], kRqOp >> 2);
          const uint32_t nin =
              (blockIdx.x == 0 && op == kRingOpChecksumInline)
                  ? (uint32_t)__builtin_amdgcn_readlane((int)x[0][kRqInl & 3], kRqInl >> 2)
              : op == kRingOpVirtioRead ? (uint32_t)__builtin_amdgcn_readlane((int)x[0][kRqHdrInl & 3], kRqHdrInl >> 2)
                                        : 0u;
          if (nin != 0) {
            // ... and every payload chunk the request carries
            const int nch = ((int)nin + 11) / 12;
            const bool torn = (lane >= 8 && lane - 8 < nch && x[0][0] != q) || (56 + lane < nch && x[1][0] != q) ||
                              (120 + lane < nch && x[2][0] != q);
            if (__builtin_amdgcn_ballot_w64(torn) != 0) return 0;
          }
          return 1;
        }
        if (__builtin_amdgcn_s_memrealtime() - t_last > idle_ticks) return 2;
        return 0;
      };
      // workgroup 0 reads the inline payload too; the others need only the
      // record and a virtio read's inline header (chunks < 64): their loads
      // 1-2 point past the record and return zeros without a memory access
      const int o1 = blockIdx.x == 0 ? 16 * (64 + lane) : 0x7FFFFFF0;
      const int o2 = blockIdx.x == 0 ? 16 * (128 + lane) : 0x7FFFFFF0;
      auto poll = [&](u32x4s (&x)[3]) {
        x[0] = __builtin_amdgcn_raw_buffer_load_b128(rs, 16 * lane, 0, 17);  // sc0 sc1
        x[1] = __builtin_amdgcn_raw_buffer_load_b128(rs, o1, 0, 17);
        x[2] = __builtin_amdgcn_raw_buffer_load_b128(rs, o2, 0, 17);
      };
      // two polls in flight, issued half a round trip apart: a posted request
      // is seen ~RTT/4 sooner on average than with one poll at a time
      u32x4s va[3], vb[3], v[3];
      poll(va);
      int st;
      for (;;) {
        __builtin_amdgcn_s_sleep(1);
        poll(vb);
        if ((st = check(va)) != 0) {
#pragma unroll
          for (int j = 0; j < 3; ++j) v[j] = va[j];
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        poll(va);
        if ((st = check(vb)) != 0) {
#pragma unroll
          for (int j = 0; j < 3; ++j) v[j] = vb[j];
          break;
        }
      }
      if (st == 2) q = 0xFFFFFFFFu;
      if (lane < 8) {
        s_w[4 * lane] = v[0][0];
        s_w[4 * lane + 1] = v[0][1];
        s_w[4 * lane + 2] = v[0][2];
        s_w[4 * lane + 3] = v[0][3];
      }
      // a virtio read's inline header bytes into LDS (zeros past them): word
      // 3p + m - 1 = chunk p's word m, the buffer's phase mod 16 kept
      if (st == 1 && (uint32_t)__builtin_amdgcn_readlane((int)v[0][kRqOp & 3], kRqOp >> 2) == kRingOpVirtioRead) {
        const int nch = ((int)__builtin_amdgcn_readlane((int)v[0][kRqHdrInl & 3], kRqHdrInl >> 2) + 11) / 12;
        const int p = lane - 8;
        if (p >= 0 && p < (int)kRingHdrChunks) {
          s_hdr[3 * p] = p < nch ? v[0][1] : 0u;
          s_hdr[3 * p + 1] = p < nch ? v[0][2] : 0u;
          s_hdr[3 * p + 2] = p < nch ? v[0][3] : 0u;
        }
      }
      uint32_t iv = 0;
      if (st == 1 && blockIdx.x == 0 &&
          (uint32_t)__builtin_amdgcn_readlane((int)v[0][kRqOp & 3], kRqOp >> 2) == kRingOpChecksumInline) {
        auto f = [&](uint32_t k) { return __builtin_amdgcn_readlane((int)v[0][k & 3], (int)(k >> 2)); };
        iv = ring_validate_inline(v, f(kRqLen), f(kRqCs), f(kRqProto), (f(kRqFlags) & WGCS_PKT_V6) != 0);
      }
      if (lane == 0) {
        s_q = q;
        s_valid = iv;
      }
    }
    __syncthreads();
    const uint32_t q = s_q;
    if (q == 0xFFFFFFFFu) break;  // block-uniform: every wave leaves
#ifdef WGCS_RING_STAMPS  // probe builds: s_memrealtime stamps of the request's phases
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
#endif
    auto w = [&](uint32_t k) { return (uint32_t)ufl((int)s_w[k]); };
    auto p64 = [&](uint32_t lo, uint32_t hi) { return (uint64_t)w(lo) | ((uint64_t)w(hi) << 32); };
    // request pointers as global-address-space ones: the inlined body then
    // emits global_load / global_store, not flat (which also waits on lgkmcnt)
    typedef __attribute__((address_space(1))) uint8_t g8;
    auto gptr = [&](uint32_t lo, uint32_t hi) { return (uint8_t*)(g8*)(uintptr_t)p64(lo, hi); };
    const uint32_t op = w(kRqOp);
    uint32_t valid = 0;
    if (op == kRingOpChecksumInline) {
      valid = s_valid;  // workgroup 0's wave 0 checked it from the poll's registers
    } else if (op == kRingOpChecksumValid) {
      if (blockIdx.x == 0 && threadIdx.x < 64)
        valid = ring_validate(gptr(kRqPktLo, kRqPktHi), (int)w(kRqLen),
                              (int)w(kRqCs), (int)w(kRqProto), (w(kRqFlags) & WGCS_PKT_V6) != 0);
    } else if (op == kRingOpVirtioRead) {
      const wgcs_gso_job job = {0, w(kRqVlen), w(kRqJflags)};
      const GsoOutPos pos = {0, w(kRqPitch), w(kRqPosFlags)};
      int32_t* h = (int32_t*)(__attribute__((address_space(1))) int32_t*)(uintptr_t)p64(kRqMetaLo, kRqMetaHi);
      const uint32_t kb = w(kRqKbufs);
      const uint8_t* vb = gptr(kRqVbufLo, kRqVbufHi);
      // the inline header: vb[k] at LDS byte (vb & 15) + k
      const uint8_t* hl = w(kRqHdrInl) ? reinterpret_cast<const uint8_t*>(s_hdr) + ((uintptr_t)vb & 15u) : nullptr;
      gso_rows_body<WGCS_GSO_U, false, 4 * kRingWaves>(vb, job, 0, (int)blockIdx.x, (int)gridDim.x, kb,
                                                         gptr(kRqOutLo, kRqOutHi), 0, true, pos, 0, w(kRqRoom), h,
                                                         h + kb, h + kb + 1, hl);
    }
    // completion: every wave's stores done; a request that stored results
    // releases them at system scope (the fence's own wait made explicit:
    // MI355X_MICROARCH.md); then {seq, valid} in ONE 8-byte write-through
    // store on this workgroup's own line, which the host spins on
#ifdef WGCS_RING_STAMPS
    const uint64_t t2 = __builtin_amdgcn_s_memrealtime();
#endif
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
#ifdef WGCS_RING_STAMPS
      const uint64_t t3 = __builtin_amdgcn_s_memrealtime();
#endif
#ifndef WGCS_RING_NOFENCE  // A/B builds: timing without the system-scope release (not exact output)
      if (op == kRingOpVirtioRead) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
#endif
#ifdef WGCS_RING_STAMPS
      {  // {body issued, drained, released, idle before} in 10-ns ticks from the request's start
        const uint64_t t4 = __builtin_amdgcn_s_memrealtime();
        const u32x4s st = {(uint32_t)(t2 - t1), (uint32_t)(t3 - t1), (uint32_t)(t4 - t1), (uint32_t)(t1 - t_last)};
        const __amdgpu_buffer_rsrc_t ss = __builtin_amdgcn_make_buffer_rsrc(&ctl->dn[blockIdx.x], (short)0, 64,
                                                                            0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(st, ss, 16, 0, 17);
      }
#endif
      typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
      const __amdgpu_buffer_rsrc_t ds = __builtin_amdgcn_make_buffer_rsrc(&ctl->dn[blockIdx.x], (short)0, 64,
                                                                          0x00020000);
      const u32x2 w = {q, valid};
      __builtin_amdgcn_raw_buffer_store_b64(w, ds, 0, 0, 17);  // sc0 sc1
    }
    last = q;
    t_last = __builtin_amdgcn_s_memrealtime();
  }
  if (threadIdx.x == 0)
    __hip_atomic_fetch_add(&ctl->dn[blockIdx.x].exited, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

hipError_t launch_ring(RingCtl* ctl, uint32_t nb, uint32_t last, uint64_t idle_ticks, hipStream_t s) {
  if (nb == 0 || nb > kRingMaxBlocks) return hipErrorInvalidValue;
  hipLaunchKernelGGL(ring_kernel, dim3(nb), dim3(64 * kRingWaves), 0, s, ctl, last, idle_ticks);
  return hipGetLastError();
}

#endif  // WGCS_RING_TU
#ifndef WGCS_RING_TU
// ---------------------------------------------------------------------------
// Job staged whole in LDS (round 5): one workgroup of NW waves per job.
//
// gso_rows_kernel's payload loads wait on a dependent chain: the job
// descriptor, then the virtio header and header chunks, then the verdict and
// the segment geometry; only then does a row know which bytes to load
// (≈ 4.7 µs of a one-stream cfg4 launch).  Here the payload
// loads depend on the descriptor alone: every wave issues, right after its
// header loads, LDS-DMA loads (global_load_lds_dwordx4) of its share of the
// job's 16-byte chunks into a 65-KiB LDS image of the job, whatever the
// geometry turns out to be.  The head (verdict, segment count, job-constant
// sums) runs while those loads are in flight; then one vmcnt(0) + barrier,
// and every row streams its segments out of LDS through the same consume /
// finish code as the register path (dword-aligned 16-byte windows, shifted to
// the destination phase, summed, stored; header chunk last).  So every input
// byte is read from HBM once, by one load issued at the start of the launch.
//
// A job larger than the image (> 65,545 bytes at a 15-byte phase) streams
// its rows from HBM as gso_rows_kernel does; every job that is not clean
// takes the decoded path (decoded_rows) with NW * 4 rows per group.
constexpr int kVmcnt0 = 0x0F70;  // s_waitcnt vmcnt(0) expcnt(7) lgkmcnt(15): gfx9 encoding, loads / stores only
constexpr int kImgBytes = 66560;  // 4,160 chunks: a 65,545-byte job ([virtio hdr | 65,535 B]) at any 16-B phase

// 16 bytes at the 4-byte aligned LDS offset o of the image (two ds_read2_b32).
__device__ __forceinline__ uint4 img16(const uint8_t* img, int o) {
  typedef unsigned int u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
  const u32x4a4 t = *reinterpret_cast<const u32x4a4*>(__builtin_assume_aligned(img + o, 4));
  return make_uint4(t.x, t.y, t.z, t.w);
}
__device__ __forceinline__ uint32_t img4(const uint8_t* img, int o) {
  return *reinterpret_cast<const uint32_t*>(__builtin_assume_aligned(img + o, 4));
}

// ---- the staged image (round 6).  One loader wave issues every LDS-DMA load
// of a part itself, through inline asm: hipcc's wait-count pass then does not
// know that LDS-DMA is pending, so it puts no vmcnt(0) in front of the LDS
// accesses that follow (with the builtin it waits for the whole image before
// the first one).  The loader publishes its progress stage by stage -- a
// counted `s_waitcnt vmcnt(N)` (its own DMA only: it issues no vector store
// before its last wait) and then an LDS word -- and the row waves poll that
// word, so the rows of the first segments stream out while the later bytes
// of the read are still landing.
typedef uint32_t u32x4s __attribute__((ext_vector_type(4)));
// Buffer resource words (wave-uniform): base, stride 0, num_records, the
// same config dword as __builtin_amdgcn_make_buffer_rsrc(..., 0x00020000).
__device__ __forceinline__ u32x4s rsrc_words(const void* base, uint32_t nrec) {
  const uint64_t a = (uint64_t)(uintptr_t)base;
  return u32x4s{(uint32_t)ufl((int)(uint32_t)a), (uint32_t)ufl((int)((uint32_t)(a >> 32) & 0xFFFFu)),
                (uint32_t)ufl((int)nrec), 0x00020000u};
}
// The LDS byte address of a __shared__ object (what M0 takes).
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)ufl((int)(uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p);
}
// buffer_load_dwordx4 ... lds: 16 bytes per lane from rsrc + voff into LDS at
// m0v + 16 * lane (the builtin's instruction, issued where hipcc cannot see it).
template <bool NT>
__device__ __forceinline__ void dma16_asm(const u32x4s& rs, int voff, uint32_t m0v) {
  if (NT)
    asm volatile("s_mov_b32 m0, %2\n\tbuffer_load_dwordx4 %0, %1, 0 offen nt lds" ::"v"(voff), "s"(rs), "s"(m0v)
                 : "memory", "m0");
  else
    asm volatile("s_mov_b32 m0, %2\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(rs), "s"(m0v)
                 : "memory", "m0");
}
template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N <= 63, "gfx9 vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// The loader's stage waits: after DMA [0, T) of K have landed (its vmcnt
// down to K - T), T is stored in the LDS word; every D instructions.
// The stage word: relaxed workgroup-scope atomics on an LDS pointer (plain
// ds_read_b32 / ds_write_b32; a volatile or flat access gets a vmcnt(0)
// from the memory legalizer, which would wait for the whole image).
typedef __attribute__((address_space(3))) int32_t* lds_flag_t;
__device__ __forceinline__ void flag_put(lds_flag_t f, int v) {
  __hip_atomic_store(f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ int flag_get(lds_flag_t f) {
  return __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
template <int K, int D, int S>
__device__ __forceinline__ void publish_stages(lds_flag_t landed, int lane) {
  if constexpr (S < K) {
    constexpr int T = S + D < K ? S + D : K;
    vm_wait<K - T>();
    if (lane == 0) flag_put(landed, T);
    publish_stages<K, D, T>(landed, lane);
  }
}

// The loader, throttled: at most W of its image DMA instructions in flight
// (W KiB; three loaders per CU), so that the chip's memory queues stay
// shallow -- every CU dumping its whole image at once queues ~18 MB, and a
// request issued behind that (the head's input, a stage's bytes) waits ~3 us
// for it.  The header DMA (issued before the call) is waited first and
// published as `hland`; then DMA d is issued once DMA d - W has landed, and
// `landed` counts landed instructions in steps of D.
template <int K, int W, int D, int d>
__device__ __forceinline__ void loader_issue(const u32x4s& rs, uint32_t l0, int lane, lds_flag_t landed) {
  if constexpr (d < K) {
    constexpr int done = d - W + 1;  // DMA [0, done) landed after this wait (the header DMA too)
    if constexpr (done > 0) {
      vm_wait<W - 1>();
      if constexpr (done % D == 0) {
        if (lane == 0) flag_put(landed, done);
      }
    }
    dma16_asm<true>(rs, 16 * (64 * d + lane), l0 + 1024 * d);
    loader_issue<K, W, D, d + 1>(rs, l0, lane, landed);
  }
}

// load_windows from the LDS image (job byte x at image offset ibias + x).
// Unlike the HBM form, windows outside the row's payload bytes [lo, hi) are
// read too (from LDS, no memory traffic) and not zeroed: consume_batch masks
// every byte of a chunk outside [hdrLen, pktLen) -- the bytes such a window
// contributes -- out of every sum and store.  Offsets below the image (a
// window before the payload) clamp to 0; the image array has room for every
// window past the job's end (>= 1,552 bytes of slack, gso_lds_kernel).
template <int U>
__device__ __forceinline__ void img_windows(const uint8_t* img, int ibias, int aoff, int k0, int r, uint4 (&A)[U],
                                            uint32_t& E) {
  const int o0 = ibias + aoff + 16 * (k0 + r);
#pragma unroll
  for (int u = 0; u < U; ++u) A[u] = img16(img, max(o0 + 256 * u, 0));
  E = img4(img, max(ibias + aoff + 16 * (k0 + 16 * U), 0));  // used by lane 15 only
}

template <int U>
__device__ __forceinline__ void stream_row_img(const uint8_t* img, int ibias, const uint8_t* rb, int i, int gso,
                                               int hdr_len, int plen, int dalign, uint8_t* dbase, int r,
                                               uint32_t& acc, RowOut& ro) {
  const RowSrc g = row_src(rb, i, gso, hdr_len, plen, dalign);
  acc = 0;
  for (int k0 = 0; k0 < g.nk; k0 += 16 * U) {
    uint4 A[U];
    uint32_t E;
    img_windows<U>(img, ibias, g.aoff, k0, r, A, E);
    consume_batch_img<U>(A, E, k0, g, hdr_len, dalign, dbase, r, acc, ro);
  }
}

// The head's inputs: the header chunks (lane r of each row: readBuf[16r, 16r +
// 16) from the dword holding it) and the 16 bytes from the dword holding vb[0].
struct HeadIn {
  uint4 H0, w;
};
// The head's results in registers (wave-uniform except Q: lane r of each
// row holds readBuf[16r, 16r + 16)).
struct HeadRes {
  int clean, type, ipv, hdr_len, gso, cs, co, plen;
  uint32_t ip_base, l4_base, tflags, id0, seq0;
  uint4 Q;
};
// The head's results, published by the head wave through LDS.
struct LdsHead {
  int32_t clean;  // 1: the row-streaming path (a clean job, gso_rows_kernel's criterion)
  int32_t type, ipv, hdr_len, gso, cs, co, plen;
  uint32_t ip_base, l4_base, tflags, id0, seq0;
  uint4 q[16];  // readBuf[16r, 16r + 16) per row lane r (P > 1 with WGCS_GSO_QLDS)
  int32_t landed;           // staged: the loader's DMA instructions landed so far
  int32_t hready;           // staged: 1 once the head wave has published everything above
  int32_t hland;            // staged: 1 once the loader's header DMA (hbuf) has landed
  int32_t hgeo;             // staged: 1 once the head wave has published the verdict and geometry
  uint4 hbuf[64];           // staged: the read's first KiB from its 16-B aligned start (the head's input)
};

// Launch shape: P = 3 workgroups of 4 waves per read (round 5, late):
// 6.35-6.46 us per cfg4 launch on four streams against 6.73-7.31 for one
// workgroup of 8 waves, 9.72-9.88 against 9.13-9.18 on one stream, the same
// HBM bytes (profiles/r5_gso_p3_ab*.jsonl, r5_pmc/); several reads in flight
// (the bench's four streams, a stager's batches) is the regime this serves.
#ifndef WGCS_GSO_LDS_WAVES
#define WGCS_GSO_LDS_WAVES 4
#endif
#ifndef WGCS_GSO_PARTS
#define WGCS_GSO_PARTS 3
#endif
#ifndef WGCS_GSO_QLDS
#define WGCS_GSO_QLDS 1  // P > 1: wave 0 publishes the header chunks through LDS (0: every wave loads them)
#endif
#ifndef WGCS_GSO_SHEAD
#define WGCS_GSO_SHEAD 1  // P > 1: the head's loads through the scalar path
#endif
#ifndef WGCS_GSO_STAGED
#define WGCS_GSO_STAGED 0  // P > 1: 1 = one loader wave, the image published stage by stage (round 6 A/B; slower)
#endif
#ifndef WGCS_GSO_STAGE_DMA
#define WGCS_GSO_STAGE_DMA 2  // staged: LDS-DMA instructions (KiB) per published stage
#endif
#ifndef WGCS_GSO_INFLIGHT
#define WGCS_GSO_INFLIGHT 8  // staged: the loader's image DMA instructions (KiB) in flight at once
#endif
#ifndef WGCS_GSO_PART_XCD
#define WGCS_GSO_PART_XCD 1  // P > 1: a job's parts on one XCD (0: consecutive blocks)
#endif
// One workgroup of NW waves per job.  Wave 0 issues the header loads, then
// every wave its share of the LDS-DMA loads of the whole job; wave 0 runs the
// head (verdict, segment count, job-constant header sums) while they are in
// flight and publishes it through LDS; one vmcnt(0) + barrier; then every row
// streams its segments out of the image (header chunks read from it as well)
// with write-through full-chunk stores: the segment stores follow the loads in
// this kernel, so the lines go to HBM while the rows still work instead of
// in one end-of-kernel writeback of every segment (≈ 17 MB for cfg4).
// P > 1 (round 5): P workgroups per job, each staging about 1/P of the job
// (part p: the segments whose payload starts in job bytes [p H, (p + 1) H),
// H = len / P rounded up to 16, plus one segment's worth past that for the
// last one), so a block holds 1/P of the LDS and rows -- P = 2: 40 KB, 4
// blocks per CU instead of 2 -- and its rows run one pass.  The parts of a job
// are dealt to one XCD (their shared header lines and boundary bytes meet in
// one L2).  Every part runs the head; part 0 writes count / status and runs
// the decoded path of a job that is not clean.  A row whose bytes lie outside
// its part's image (gsoSize > 1,536) streams from HBM.
template <int NW, int U, bool NT, int P>
#ifdef WGCS_GSO_LDS_WPE  // A/B builds: waves per SIMD to compile for (VGPR budget)
#define WGCS_GSO_LDS_ATTR __attribute__((amdgpu_waves_per_eu(WGCS_GSO_LDS_WPE, 8)))
#else
#define WGCS_GSO_LDS_ATTR
#endif
__global__ __launch_bounds__(NW * 64) WGCS_GSO_LDS_ATTR void gso_lds_kernel(const uint8_t* __restrict__ arena,
                                                           const wgcs_gso_job* __restrict__ jobs, uint32_t max_segs,
                                                           uint8_t* __restrict__ out, uint32_t out_stride,
                                                           const GsoOutPos* __restrict__ outpos, uint32_t offset,
                                                           uint32_t room, int32_t* __restrict__ sizes,
                                                           int32_t* __restrict__ count, int32_t* __restrict__ status, uint32_t n_jobs) {
  constexpr int ROWS = NW * 4;  // 16-lane rows per workgroup
  // a part's staged bytes: H (at most kImgBytes / P rounded up) + 48 before +
  // kPartTail past its end; the image also holds 1,552 bytes of window slack
  constexpr int kPartTail = 1536 + 32;
  constexpr int kStage = P == 1 ? kImgBytes : ((kImgBytes + P - 1) / P + 15) / 16 * 16 + 48 + kPartTail + 16;
  constexpr int kIters = ((kStage + 1552) / 16 + NW * 64 - 1) / (NW * 64);  // LDS-DMA instructions per wave
  constexpr int kArr = kIters * NW * 64 * 16;                      // every slot a DMA writes
  static_assert(kArr >= kStage + 1552, "image slack for the windows past a job's end");
  __shared__ __attribute__((aligned(16))) uint8_t img[kArr];
  __shared__ LdsHead hd;
#ifdef WGCS_GSO_STAMPS  // timing-only build (scripts/probe_gso_stamps.py, LDS kernel: NWAVES=NW)
  uint64_t stp[5] = {__builtin_amdgcn_s_memrealtime(), 0, 0, 0, 0};
#endif
  const int lane = threadIdx.x & 63;
  const int r = lane & 15;
  const int wv = threadIdx.x >> 6;
  uint32_t jb = blockIdx.x;
  int part = 0;
  if (P > 1) {  // blocks b, b + 8, ... share an XCD: job (k / P) * 8 + b % 8, part k % P (k = b / 8)
    if (WGCS_GSO_PART_XCD) {
      const uint32_t k = blockIdx.x >> 3;
      jb = (k / P) * 8 + (blockIdx.x & 7u);
      part = (int)(k % P);
    } else {
      jb = blockIdx.x / P;
      part = (int)(blockIdx.x % P);
    }
    if (jb >= n_jobs) return;  // the grid is padded to a multiple of 8 jobs
  }
  const wgcs_gso_job job = jobs[jb];
  const uint8_t* vb = arena + job.off;
  const uint32_t jlen = job.len;
  const uint8_t* rb = vb + 10;
  const uint64_t slot0 = (uint64_t)jb * max_segs;
  uint64_t obase = slot0 * out_stride;
  uint32_t opitch = out_stride;
  uint32_t tails = 1;
  if (outpos) {
    obase = outpos[jb].base;
    opitch = outpos[jb].pitch;
    tails = outpos[jb].flags & kOutPosTails;
  }
  const int ibias = (int)((uintptr_t)vb & 15u);
  const int nch = (int)((jlen + (uint32_t)ibias + 15u) >> 4);
  // this part's image: chunks [q_lo, q_lo + q_n) of the job (chunk q = the
  // aligned 16 bytes at (vb & ~15) + 16 q); job byte x at image offset x + ib_p
  const int H = P == 1 ? 0 : (int)(((jlen + P - 1) / P + 15u) & ~15u);
  int q_lo = 0, q_n = nch;
  if (P > 1) {
    q_lo = max(0, (part * H + ibias) / 16 - 3);
    const int q_hi = part == P - 1 ? nch : min(nch, ((part + 1) * H + kPartTail + ibias + 15) / 16);
    q_n = max(0, q_hi - q_lo);
  }
  const int ib_p = ibias - 16 * q_lo;
  const bool use_img = P == 1 ? (jlen >= 14 && nch <= kImgBytes / 16)  // block-uniform
                              : (jlen >= 14 && q_n <= kStage / 16);
  const bool raw = (job.flags & WGCS_GSO_JOB_RAW) != 0;
  // Staged (P > 1, round 6): wave 0 is the loader and issues nothing else
  // before its stage waits; wave 1 runs the head (its loads are the
  // compiler's, waited on inside the head: none is pending where the loader's
  // code continues, so hipcc puts no vmcnt(0) behind the loader's DMA).
  constexpr bool STG = P > 1 && WGCS_GSO_STAGED != 0;
  constexpr int kHeadWave = STG ? 1 : 0;
  constexpr int kDma = (kStage + 1023) / 1024;  // staged: the loader's LDS-DMA instructions (1 KiB each)
  static_assert(!STG || (NW >= 2 && kDma <= 63 && kDma * 1024 <= kArr), "staged image: roles, vmcnt, image size");
  // ---- the head wave (wave 0; staged: wave 1): header chunks (as gso_rows_kernel) and the virtio header +
  // readBuf[0] (16 bytes from the dword holding vb[0], range-checked: zeros
  // past the job), issued ahead of its bulk loads so that the head waits for
  // them alone (a counted vmcnt)
  const int hph = (int)((uintptr_t)rb & 3u);
  const uint8_t* hbase = rb - hph;
  const __amdgpu_buffer_rsrc_t hrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(hbase), (short)0, (int)(jlen + 3u) - (int)(hbase - vb), 0x00020000);
  const int sh = (int)((uintptr_t)vb & 3u);
  uint4 H0 = make_uint4(0, 0, 0, 0), w = make_uint4(0, 0, 0, 0);
  if (P > 1 && !WGCS_GSO_QLDS && wv != kHeadWave) H0 = bld16<false>(hrs, 16 * r);  // the header chunks (Q) of every row
  // P > 1, a read long enough (WGCS_GSO_SHEAD): the head's inputs through the
  // scalar path (s_load from uniform addresses), so they do not queue in the
  // CU's vector-memory pipeline behind the LDS-DMA of the blocks already on
  // it; the 64 header dwords become per-lane chunks by selects
  const bool shead = P > 1 && WGCS_GSO_SHEAD && jlen >= 288;  // block-uniform
  // (by value in and out: a lambda writing the outer H0 / w by reference put
  // them in scratch memory, whose loads then queued behind the bulk DMA)
  auto head_loads = [&]() -> HeadIn {
  uint4 H0 = make_uint4(0, 0, 0, 0), w = make_uint4(0, 0, 0, 0);
  if (STG && shead) {
    // staged: the loader's first DMA instruction brings the read's first KiB
    // into hd.hbuf ahead of its bulk; the head reads its inputs from there
    // (s_load's of the same bytes queue behind every CU's bulk DMA: ~3 us)
    while (ufl(flag_get((lds_flag_t)&hd.hland)) == 0) __builtin_amdgcn_s_sleep(1);
    asm volatile("" ::: "memory");
#if defined(WGCS_GSO_STAMPS) && WGCS_GSO_STAMPS == 3  // head wave: T2 header seen
    stp[2] = __builtin_amdgcn_s_memrealtime();
#endif
    const uint8_t* hb8 = reinterpret_cast<const uint8_t*>(hd.hbuf);
    w = img16(hb8, ibias - sh);
    H0 = img16(hb8, ibias + 10 - hph + 16 * r);
  } else if (!shead) {
    H0 = bld16<false>(hrs, 16 * r);
    const __amdgpu_buffer_rsrc_t vrs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t*>(vb - sh), (short)0, (int)(jlen + 3u + (uint32_t)sh), 0x00020000);
    w = bld16<false>(vrs, 0);
  } else {
    typedef const __attribute__((address_space(4))) uint32_t* cptr;  // constant space: s_load
    const cptr vp = (cptr)(const void*)(vb - sh);
    w = make_uint4(vp[0], vp[1], vp[2], vp[3]);
    const cptr hp = (cptr)(const void*)hbase;
    uint32_t hv[64];
#pragma unroll
    for (int k = 0; k < 64; ++k) hv[k] = hp[k];
#pragma unroll
    for (int k = 0; k < 16; ++k) {  // lane r of each row takes dwords 4r .. 4r + 3
      const bool m = r == k;
      H0.x = m ? hv[4 * k] : H0.x;
      H0.y = m ? hv[4 * k + 1] : H0.y;
      H0.z = m ? hv[4 * k + 2] : H0.z;
      H0.w = m ? hv[4 * k + 3] : H0.w;
    }
  }
  return HeadIn{H0, w};
  };
  // ---- every wave: its share of the whole job into the LDS image.  Chunk q
  // = the aligned 16 bytes at (vb & ~15) + 16 q, image offset 16 q (job byte x
  // at ibias + x); an aligned chunk holding a job byte lies in that byte's
  // page.  kIters instructions per wave unconditionally, through a
  // range-checked resource over the job's chunks (loads past it are dropped;
  // a job too large for the image gets an empty range): a fixed count of
  // loads behind wave 0's header loads.
  auto bulk_loads = [&]() {
  if (STG) {
    if (wv == 0) {  // the loader: the read's first KiB (the head's input), then the part's chunks in order
      const u32x4s hrs4 = rsrc_words(vb - ibias, jlen + (uint32_t)ibias);
      dma16_asm<false>(hrs4, 16 * lane, lds_addr(hd.hbuf));
      const u32x4s irs4 = rsrc_words(vb - ibias + 16 * q_lo, use_img ? 16 * q_n : 0);
      const uint32_t l0 = lds_addr(img);
      if constexpr (STG) {
        constexpr int W = WGCS_GSO_INFLIGHT < kDma ? WGCS_GSO_INFLIGHT : kDma;
        // the first W image DMAs, then the header's wait (the oldest), then the rest throttled
#pragma unroll
        for (int d = 0; d < W; ++d) dma16_asm<NT>(irs4, 16 * (64 * d + lane), l0 + 1024 * d);
        vm_wait<W>();
        if (lane == 0) flag_put((lds_flag_t)&hd.hland, 1);
#if defined(WGCS_GSO_STAMPS) && WGCS_GSO_STAMPS == 3  // loader: T2 header landed
        stp[2] = __builtin_amdgcn_s_memrealtime();
#endif
        loader_issue<kDma, W, WGCS_GSO_STAGE_DMA, W>(irs4, l0, lane, (lds_flag_t)&hd.landed);
      }
    }
  } else {
    const __amdgpu_buffer_rsrc_t irs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t*>(vb - ibias + 16 * q_lo), (short)0, use_img ? 16 * q_n : 0, 0x00020000);
#pragma unroll
    for (int it = 0; it < kIters; ++it) {
      const int q0 = (it * NW + wv) * 64;  // this wave-instruction's first chunk (1 KiB of LDS)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(irs, (__attribute__((address_space(3))) void*)(img + 16 * q0), 16,
                                               16 * (q0 + lane), 0, 0, NT ? 2 : 0);
    }
  }
  };
  // ---- the head wave: the head, while the bulk loads are in flight
  // publish: this wave writes count / status (part 0) and the LDS copy
  // the job-constant header sums (as gso_rows_kernel) of a clean job: only
  // finish_row needs them, so the staged row waves compute them after their
  // first payload stream (the loads and stores of it do not wait for them)
  auto head_sums = [&](HeadRes& h) {
    const bool tcp_s = h.type != GSO_UDP_L4;
    const uint4 Q = h.Q;
    const int cs = h.cs, hdr_len = h.hdr_len, ipv = h.ipv;
    const int x0 = 16 * r;
    const int vlo = cs + 4, vhi = tcp_s ? cs + 8 : cs + 6;
    const int ca = (cs + h.co) & 0xFFFF;
    uint32_t ip_base = 0, l4_base = 0, tflags = 0, id0 = 0, seq0 = 0;
    if (ipv == 4) {
      const uint32_t m = byte_bits16(-x0, cs - x0) & ~byte_bits16(2 - x0, 6 - x0) & ~byte_bits16(10 - x0, 12 - x0);
      ip_base = (uint32_t)ufl((int)bswap16(fold32_16(row16_sum_u32(add4_masked(0u, Q, m, false)))));
    }
    uint32_t ml4 = byte_bits16(cs - x0, hdr_len - x0) & ~byte_bits16(ca - x0, ca + 2 - x0) &
                   ~byte_bits16(vlo - x0, vhi - x0);
    if (tcp_s) ml4 &= ~byte_bits16(cs + 13 - x0, cs + 14 - x0);
    const int a_lo = ipv == 4 ? 12 : 8, a_hi = ipv == 4 ? 20 : 40;
    uint32_t s4 = add4_masked(0u, Q, ml4, false);
    s4 = add4_masked(s4, Q, byte_bits16(a_lo - x0, a_hi - x0), (cs & 1) != 0);
    uint32_t t4 = fold32_16(row16_sum_u32(s4));
    if ((cs & 1) == 0) t4 = bswap16(t4);
    if (tcp_s) tflags = qbyte(Q, cs + 13);
    l4_base = (uint32_t)ufl((int)t4) + (tflags & ~0x09u);
    if (ipv == 4) {
      const uint32_t b45 = qdw(Q, 1);
      id0 = ((b45 & 0xFFu) << 8) | ((b45 >> 8) & 0xFFu);
    }
    if (tcp_s) seq0 = __builtin_bswap32(qle32(Q, vlo));
    h.ip_base = ip_base;
    h.l4_base = l4_base;
    h.tflags = tflags;
    h.id0 = id0;
    h.seq0 = seq0;
  };
  // the LDS copy of the head's results and the hready word (the loader and,
  // unstaged, every wave read it)
  auto publish_geo = [&](const HeadRes& h) {  // the verdict and geometry (staged: + the hgeo word)
    if (lane == 0) {
      hd.clean = h.clean;
      hd.type = h.type;
      hd.ipv = h.ipv;
      hd.hdr_len = h.hdr_len;
      hd.gso = h.gso;
      hd.cs = h.cs;
      hd.co = h.co;
      hd.plen = h.plen;
    }
    if (STG) {
      asm volatile("" ::: "memory");
      if (lane == 0) flag_put((lds_flag_t)&hd.hgeo, 1);
    }
  };
  auto head_publish = [&](const HeadRes& h) {  // the sums and Q (staged: + the hready word); unstaged: all
    if (!STG) publish_geo(h);
    if (lane == 0) {
      hd.ip_base = h.ip_base;
      hd.l4_base = h.l4_base;
      hd.tflags = h.tflags;
      hd.id0 = h.id0;
      hd.seq0 = h.seq0;
    }
    if (P > 1 && WGCS_GSO_QLDS) {  // the head's Q (every row of the wave holds it; row 0 publishes)
      if (lane < 16) hd.q[lane] = h.Q;
    }
    if (STG) {  // after every field above (one wave's LDS writes complete in order)
      asm volatile("" ::: "memory");
      if (lane == 0) flag_put((lds_flag_t)&hd.hready, 1);
#if defined(WGCS_GSO_STAMPS) && WGCS_GSO_STAMPS == 3  // head wave: T3 head published
      stp[3] = __builtin_amdgcn_s_memrealtime();
#endif
    }
  };
  // The verdict and geometry (and count / status when `publish`); with
  // `sums` also the job-constant header sums.
  auto head = [&](const uint4 H0, const uint4 w, bool publish, bool sums) -> HeadRes {
    // the virtio header words become scalars only here, behind the bulk loads
    // (a wave-uniform load's value is otherwise moved into SGPRs at the load,
    // with a vmcnt(0) in front of every bulk load)
    uint4 wq = w;
    asm volatile("" : "+v"(wq.x), "+v"(wq.y), "+v"(wq.z), "+v"(wq.w));
    wq = make_uint4((uint32_t)ufl((int)wq.x), (uint32_t)ufl((int)wq.y), (uint32_t)ufl((int)wq.z),
                    (uint32_t)ufl((int)wq.w));
    uint32_t t1 = 0, hl = 0, g = 0, c = 0, o = 0, b0 = 0;
    if (jlen >= 14) {
      const uint64_t lo = ((uint64_t)wq.y << 32) | wq.x, hi = ((uint64_t)wq.w << 32) | wq.z;
      const uint64_t v0 = sh ? (lo >> (8 * sh)) | (hi << (64 - 8 * sh)) : lo;
      const uint64_t v1 = hi >> (8 * sh);
      t1 = (uint32_t)(v0 >> 8) & 0xFFu;
      hl = (uint32_t)(v0 >> 16) & 0xFFFFu;
      g = (uint32_t)(v0 >> 32) & 0xFFFFu;
      c = (uint32_t)(v0 >> 48) & 0xFFFFu;
      o = (uint32_t)v1 & 0xFFFFu;
      b0 = (uint32_t)(v1 >> 16) & 0xFFu;
    }
    const int plen_s = jlen > 10 ? (int)jlen - 10 : 0;
    const int type_s = raw ? ((t1 == GSO_TCPV4 || t1 == GSO_TCPV6) ? (int)t1 : GSO_UDP_L4) : (int)t1;
    const int ipv_s = raw ? ((job.flags & WGCS_GSO_JOB_V6) ? 6 : 4) : (int)(b0 >> 4);
    const bool tcp_s = type_s != GSO_UDP_L4;
    const bool ok_s = jlen >= 14 && g != 0 && (type_s == GSO_TCPV4 || type_s == GSO_TCPV6 || type_s == GSO_UDP_L4) &&
                      ((ipv_s == 4 && type_s != GSO_TCPV6) || (ipv_s == 6 && type_s != GSO_TCPV4));
    const int gso_s = (int)g, cs_s = (int)c, co_s = (int)o;
    const int hdr_s = (raw || tcp_s) ? (int)hl : ((cs_s + 8) & 0xFFFF);
    const int ca_s = (cs_s + co_s) & 0xFFFF;
    const int pkt0_s = hdr_s + min(gso_s, plen_s - hdr_s);
    const bool clean_s = ok_s && hdr_s < plen_s && cs_s >= (ipv_s == 4 ? 20 : 40) && ca_s + 2 <= hdr_s &&
                         hdr_s <= kMaxHdrLen && (raw || !tcp_s || (hdr_s - cs_s >= 20 && hdr_s - cs_s <= 60)) &&
                         fast_header(cs_s, hdr_s, ca_s, tcp_s) && (uint32_t)pkt0_s <= room;
    uint4 Q;
    {
      const uint32_t nx = row_next(H0.x);
      Q = make_uint4(__builtin_amdgcn_alignbyte(H0.y, H0.x, hph), __builtin_amdgcn_alignbyte(H0.z, H0.y, hph),
                     __builtin_amdgcn_alignbyte(H0.w, H0.z, hph), __builtin_amdgcn_alignbyte(nx, H0.w, hph));
    }
    bool clean = clean_s;
    if (clean && tcp_s && !raw) {  // the TCP data offset decides hdrLen (tun.go:601-614)
      const int th = (int)((qbyte(Q, cs_s + 12) >> 4) * 4);
      clean = ((cs_s + th) & 0xFFFF) == hdr_s;
    }
    if (ufl(clean ? 1 : 0)) {
      if (publish && lane == 0 && part == 0) {  // the checks can only end in the segment count here (gso_rows_kernel)
        const int nfull_s = (plen_s - hdr_s + gso_s - 1) / gso_s;
        const bool many = nfull_s > (int)max_segs;
        count[jb] = many ? (int)max_segs - 1 : nfull_s;
        status[jb] = many ? WGCS_ERR_TOO_MANY_SEGMENTS : 0;
      }
    }
    HeadRes res = {clean ? 1 : 0, type_s, ipv_s, hdr_s, gso_s, cs_s, co_s, plen_s, 0u, 0u, 0u, 0u, 0u, Q};
    if (sums && res.clean) head_sums(res);
    return res;
  };
  // the head's results from the LDS copy (after the barrier / the hready word)
  auto sums_from_lds = [&](HeadRes& h) {
    h.ip_base = (uint32_t)ufl((int)hd.ip_base);
    h.l4_base = (uint32_t)ufl((int)hd.l4_base);
    h.tflags = (uint32_t)ufl((int)hd.tflags);
    h.id0 = (uint32_t)ufl((int)hd.id0);
    h.seq0 = (uint32_t)ufl((int)hd.seq0);
    h.Q = (P > 1 && WGCS_GSO_QLDS) ? hd.q[r] : make_uint4(0, 0, 0, 0);
  };
  auto head_from_lds = [&]() -> HeadRes {
    HeadRes h;
    h.clean = ufl(hd.clean);
    h.type = ufl(hd.type);
    h.ipv = ufl(hd.ipv);
    h.hdr_len = ufl(hd.hdr_len);
    h.gso = ufl(hd.gso);
    h.cs = ufl(hd.cs);
    h.co = ufl(hd.co);
    h.plen = ufl(hd.plen);
    h.ip_base = (uint32_t)ufl((int)hd.ip_base);
    h.l4_base = (uint32_t)ufl((int)hd.l4_base);
    h.tflags = (uint32_t)ufl((int)hd.tflags);
    h.id0 = (uint32_t)ufl((int)hd.id0);
    h.seq0 = (uint32_t)ufl((int)hd.seq0);
    h.Q = (P > 1 && WGCS_GSO_QLDS) ? hd.q[r] : make_uint4(0, 0, 0, 0);
    return h;
  };
  HeadRes hr = {};
  if (STG) {  // the loader's DMA; the head wave's loads and head in ONE branch (waited inside it)
    // the two LDS words start at 0 before any wave may poll them (the
    // barrier waits on LDS and scalar loads only: the job descriptor)
    if (threadIdx.x == 0) {
      flag_put((lds_flag_t)&hd.landed, 0);
      flag_put((lds_flag_t)&hd.hready, 0);
      flag_put((lds_flag_t)&hd.hland, 0);
      flag_put((lds_flag_t)&hd.hgeo, 0);
    }
    lds_barrier();
#if defined(WGCS_GSO_STAMPS) && WGCS_GSO_STAMPS == 3  // per role: T1 past the init barrier
    stp[1] = __builtin_amdgcn_s_memrealtime();
#endif
    if (wv == 0) {
      bulk_loads();
    } else {
      // every row wave runs the head itself from the header bytes (no wait
      // for one head wave, no LDS round trip); the head wave also publishes
      // it for the loader
      if (wv == kHeadWave) {
        // the verdict and geometry first (the other row waves start their
        // payload streams on them), then the header sums and Q, which only
        // finish_row needs
        HeadIn hi = head_loads();
#ifdef WGCS_GSO_HEAD_TWICE  // timing-only build: the fast head run twice (is the first run instruction-fetch bound?)
        hr = head(hi.H0, hi.w, false, false);
        stp[2] = __builtin_amdgcn_s_memrealtime();
        asm volatile("" : "+v"(hi.H0.x), "+v"(hi.w.x), "+v"(hi.w.y));
        if (ufl(hr.gso) == 0x7FFFFFFF) hi.w.x = 0;
#endif
        hr = head(hi.H0, hi.w, true, false);
        publish_geo(hr);
        if (hr.clean) head_sums(hr);
        head_publish(hr);
      } else {
        while (ufl(flag_get((lds_flag_t)&hd.hgeo)) == 0) __builtin_amdgcn_s_sleep(1);
        asm volatile("" ::: "memory");
        hr = head_from_lds();  // the sums and Q in it are read again once hready is set (ensure_sums)
      }
    }
  } else {
    HeadIn hi = {make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0)};
    if (wv == kHeadWave) hi = head_loads();
    __builtin_amdgcn_sched_barrier(0);  // keep the header loads ahead of the bulk loads
    bulk_loads();
    if (wv == kHeadWave) head_publish(head(hi.H0, hi.w, true, true));
  }
#ifdef WGCS_GSO_STAMPS
  if (WGCS_GSO_STAMPS != 3) stp[1] = __builtin_amdgcn_s_memrealtime();
#endif
  // ---- every wave's bulk loads have landed (the compiler's own s_waitcnt,
  // not inline asm: its wait-count pass then knows no LDS-DMA is pending and
  // puts no vmcnt(0) -- which would also wait for the row's earlier stores --
  // in front of the image reads of the row loop); the barrier publishes the
  // image and the head
  const lds_flag_t landed = (lds_flag_t)&hd.landed;
  if (STG) {
    // no barrier: the loader publishes its stages while the head wave still
    // works; every wave but the head wave waits for the head's word
    if constexpr (STG) {
      if (wv == 0) {  // the last W instructions' stages (the loader issued every DMA already)
        constexpr int W = WGCS_GSO_INFLIGHT < kDma ? WGCS_GSO_INFLIGHT : kDma;
        constexpr int D = WGCS_GSO_STAGE_DMA;
        publish_stages<kDma, D, (kDma - W) / D * D>(landed, lane);  // ends at vmcnt(0)
#if defined(WGCS_GSO_STAMPS) && WGCS_GSO_STAMPS == 3  // loader: T3 all landed
        stp[3] = __builtin_amdgcn_s_memrealtime();
#endif
      }
    }
    if (wv == 0) {  // the loader takes the head wave's copy
      while (ufl(flag_get((lds_flag_t)&hd.hready)) == 0) __builtin_amdgcn_s_sleep(1);
      asm volatile("" ::: "memory");
      hr = head_from_lds();
    }
#if defined(WGCS_GSO_STAMPS) && WGCS_GSO_STAMPS == 3  // row waves: T2 head computed
    if (wv > 1) stp[2] = __builtin_amdgcn_s_memrealtime();
#endif
#ifdef WGCS_GSO_STAMPS  // staged: T1 head known, T2 the wave's first rows may start (loader: all landed)
    if (WGCS_GSO_STAMPS != 3) stp[1] = __builtin_amdgcn_s_memrealtime();
#endif
  } else {
    __builtin_amdgcn_s_waitcnt(kVmcnt0);
    lds_barrier();
    hr = head_from_lds();
  }
#ifdef WGCS_GSO_STAMPS
  if (WGCS_GSO_STAMPS != 3) stp[2] = __builtin_amdgcn_s_memrealtime();
#endif
  if (ufl(hr.clean)) {
    const int type = ufl(hr.type), ipv = ufl(hr.ipv), hdr_len = ufl(hr.hdr_len), gso = ufl(hr.gso);
    const int cs = ufl(hr.cs), co = ufl(hr.co), plen = ufl(hr.plen);
    // staged: the head wave computes the header sums now and publishes the
    // head for the loader; the other row waves after their first payload stream
    bool sums = !STG || wv == 0 || wv == kHeadWave;
    uint32_t ip_base = (uint32_t)ufl((int)hr.ip_base), l4_base = (uint32_t)ufl((int)hr.l4_base);
    uint32_t tflags = (uint32_t)ufl((int)hr.tflags), id0 = (uint32_t)ufl((int)hr.id0);
    uint32_t seq0 = (uint32_t)ufl((int)hr.seq0);
    auto has_seg = [&](int i) { return i < (int)max_segs && hdr_len + (int64_t)i * gso < plen; };
    // readBuf[16r, 16r + 16): from the image, or (a job too large for it)
    // from HBM as gso_rows_kernel reads it
    uint4 Q;
    if (P > 1 && WGCS_GSO_QLDS) {  // the wave's own head (staged) or the head wave's LDS copy
      Q = hr.Q;
    } else if (P > 1) {  // from the header loads every wave issued first
      const uint32_t nx = row_next(H0.x);
      Q = make_uint4(__builtin_amdgcn_alignbyte(H0.y, H0.x, hph), __builtin_amdgcn_alignbyte(H0.z, H0.y, hph),
                     __builtin_amdgcn_alignbyte(H0.w, H0.z, hph), __builtin_amdgcn_alignbyte(nx, H0.w, hph));
    } else if (use_img) {
      const int dq = ibias + 10 + 16 * r, s = dq & 3;
      const uint4 T = img16(img, dq - s);
      const uint32_t T4 = img4(img, dq - s + 16);
      Q = make_uint4(__builtin_amdgcn_alignbyte(T.y, T.x, s), __builtin_amdgcn_alignbyte(T.z, T.y, s),
                     __builtin_amdgcn_alignbyte(T.w, T.z, s), __builtin_amdgcn_alignbyte(T4, T.w, s));
    } else {
      const uint4 Hq = bld16<false>(hrs, 16 * r);
      const uint32_t nx = row_next(Hq.x);
      Q = make_uint4(__builtin_amdgcn_alignbyte(Hq.y, Hq.x, hph), __builtin_amdgcn_alignbyte(Hq.z, Hq.y, hph),
                     __builtin_amdgcn_alignbyte(Hq.w, Hq.z, hph), __builtin_amdgcn_alignbyte(nx, Hq.w, hph));
    }
    auto ensure_sums = [&]() {
      if (STG && !sums) {
        while (ufl(flag_get((lds_flag_t)&hd.hready)) == 0) __builtin_amdgcn_s_sleep(1);
        asm volatile("" ::: "memory");
        sums_from_lds(hr);
        Q = hr.Q;
        ip_base = (uint32_t)ufl((int)hr.ip_base);
        l4_base = (uint32_t)ufl((int)hr.l4_base);
        tflags = (uint32_t)ufl((int)hr.tflags);
        id0 = (uint32_t)ufl((int)hr.id0);
        seq0 = (uint32_t)ufl((int)hr.seq0);
        sums = true;
      }
    };
    // write-through stores through a resource over the job's output region
    // when every row offset fits it (block-uniform; else plain stores)
    // (based at out + obase rounded down to 16 bytes: every row's dbase lies
    // at a non-negative 16-byte multiple from it)
    const bool wt = WGCS_GSO_WT && (uint64_t)max_segs * opitch + offset < 0x7FFF0000ull;
    uint8_t* const obase16 = out + obase - ((uintptr_t)(out + obase) & 15u);
    const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(obase16, (short)0, 0x7FFFFFFF, 0x00020000);
    // this part's segments: payload start (job byte 10 + hdrLen + i gso) in
    // [part H, (part + 1) H)
    int i0 = 0, i1 = 0x7FFFFFFF;
    if (P > 1) {
      const int64_t a = (int64_t)part * H - 10 - hdr_len, b = a + H;
      // ceil(x / gso) in 32 bits where x fits (every read the image holds): a
      // 64-bit division is a long serial chain on this critical path
      auto cdiv = [&](int64_t x) -> int {
        if (x <= 0) return 0;
        if (x < 0x40000000) return (int)(((uint32_t)x + (uint32_t)gso - 1u) / (uint32_t)gso);
        return (int)min((x + gso - 1) / gso, (int64_t)0x7FFFFFFF);
      };
      i0 = cdiv(a);
      if (part < P - 1) i1 = cdiv(b);
    }
    const int lo_b = 16 * q_lo - ibias, hi_b = 16 * (q_lo + q_n) - ibias;  // staged job bytes
    // staged: the loader (wave 0) takes the last rows of a pass, the other
    // waves the first ones in order, so they start on the stages that land first
    // (the head wave, which computes the sums first, takes the rows before the loader's)
    const int slotw = (STG ? (wv == 0 ? NW - 1 : wv == kHeadWave ? NW - 2 : wv - 2) : wv) * 4;
    for (int i = i0 + slotw + (lane >> 4); i < i1 && has_seg(i); i += ROWS) {  // row-uniform
      if (STG && use_img) {
        // every payload byte of the wave's rows landed: job bytes up to the
        // end of its last row's segment (+ the window's next dword), image
        // offset ib_p + x, in loader instructions of 1 KiB
        const int il = min(ufl(i - (lane >> 4)) + 3, i1 - 1);
        const int64_t se = min((int64_t)plen, (int64_t)hdr_len + (int64_t)(il + 1) * gso);
        const int need = ufl((int)min((int64_t)kDma, ((int64_t)ib_p + 10 + se + 4 + 1023) >> 10));
        while (ufl(flag_get(landed)) < need) __builtin_amdgcn_s_sleep(1);
        asm volatile("" ::: "memory");
#ifdef WGCS_GSO_STAMPS
        if (wv != 0 && i - (lane >> 4) == i0 + slotw) stp[WGCS_GSO_STAMPS == 3 ? 3 : 2] = __builtin_amdgcn_s_memrealtime();
#endif
      }
      uint8_t* dst = out + obase + (uint64_t)i * opitch + offset;
      const int dalign = (int)((uintptr_t)dst & 15u);
      uint8_t* dbase = dst - dalign;
      uint32_t acc = 0;
      bool in_img = use_img;
      if (P > 1 && in_img) {  // the row's payload windows staged, and every window it reads inside the image
        const RowSrc g = row_src(rb, i, gso, hdr_len, plen, dalign);
        in_img = g.lo - 18 >= lo_b && (g.hi + 20 <= hi_b || q_lo + q_n >= nch) &&
                 ib_p + g.aoff + 16 * ((g.nk + 16 * U - 1) / (16 * U) * 16 * U) + 4 <= kArr;
      }
      RowOut ro;
      ro.keep = make_uint4(0, 0, 0, 0);
      ro.rs = ors;
      ro.dro = (int)(dbase - obase16);
      ro.wt = wt;
      if (in_img) {
#ifndef WGCS_GSO_PROBE_NOSTREAM  // timing-only builds (not exact output): the row's parts alone
        stream_row_img<U>(img, ib_p, rb, i, gso, hdr_len, plen, dalign, dbase, r, acc, ro);
#endif
      } else {
        stream_row<U, NT>(rb, i, gso, hdr_len, plen, dalign, dbase, r, acc, job_rsrc(vb, jlen));
      }
      ensure_sums();  // one place: the header sums' code is inlined once
#ifndef WGCS_GSO_PROBE_NOFINISH
      if (in_img)
        finish_row(true, Q, type, ipv, hdr_len, gso, cs, co, plen, i, r, dalign, dst, dbase, acc, ip_base, l4_base,
                   tflags, id0, seq0, &sizes[slot0 + (uint32_t)i], &ro);
      else
        finish_row(true, Q, type, ipv, hdr_len, gso, cs, co, plen, i, r, dalign, dst, dbase, acc, ip_base, l4_base,
                   tflags, id0, seq0, &sizes[slot0 + (uint32_t)i]);
#else
      if (r == 0) sizes[slot0 + (uint32_t)i] = (int32_t)acc;
#endif
    }
#ifdef WGCS_GSO_STAMPS
    if (WGCS_GSO_STAMPS != 3) stp[3] = __builtin_amdgcn_s_memrealtime();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stp[4] = __builtin_amdgcn_s_memrealtime();
    if (lane == 0 && max_segs >= 128 && part * NW + wv < 12) {
      int32_t* sp = sizes + slot0 + 64 + (part * NW + wv) * 5;
      for (int k = 0; k < 5; ++k) sp[k] = (int32_t)(uint32_t)stp[k];
    }
#endif
  } else if (part == 0) {
    // every other job: the decoded path, NW * 4 rows per group (the image's
    // loads have drained above, so no LDS-DMA write can land after the
    // workgroup retires)
    for (int grp = 0;; ++grp) {  // block-uniform
      const int i = grp * ROWS + wv * 4 + (lane >> 4);
      uint8_t* dst = out + obase + (uint64_t)i * opitch + offset;
      const int live = decoded_rows<U, NT>(vb, jlen, job.flags, room, max_segs, i, grp == 0, &count[jb], &status[jb],
                                           out + obase + offset, dst, &sizes[slot0], tails);
      lds_barrier();
      if ((int64_t)(grp + 1) * ROWS >= (int64_t)ufl(live)) break;
    }
  }
}

// WGCS_GSO_KERNEL=rows selects the round-4 grid (A/B builds and probes)
static int gso_use_rows() {
  static const int use_rows = [] {
    const char* e = getenv("WGCS_GSO_KERNEL");
    return e && e[0] == 'r' ? 1 : 0;
  }();
  return use_rows;
}

void gso_kernel_shape(int* lds_waves, int* parts, int* u, int* rows) {
  if (lds_waves) *lds_waves = WGCS_GSO_LDS_WAVES;
  if (parts) *parts = WGCS_GSO_PARTS;
  if (u) *u = WGCS_GSO_U;
  if (rows) *rows = gso_use_rows();
}

hipError_t launch_gso_split_batch(const uint8_t* arena, const wgcs_gso_job* jobs, uint32_t n_jobs, uint8_t* out,
                                  uint32_t out_stride, uint32_t offset, uint32_t max_segs, int32_t* sizes,
                                  int32_t* count, int32_t* status, hipStream_t s, const GsoOutPos* outpos,
                                  uint32_t room) {
  if (n_jobs == 0 || max_segs == 0) return hipSuccess;
  if (!outpos) room = out_stride > offset ? out_stride - offset : 0;
  const int use_rows = gso_use_rows();
  if (!use_rows) {
    constexpr int NW = WGCS_GSO_LDS_WAVES;
    constexpr int P = WGCS_GSO_PARTS;
    if (P == 1) {
      hipLaunchKernelGGL((gso_lds_kernel<NW, WGCS_GSO_U, true, 1>), dim3(n_jobs), dim3(NW * 64), 0, s, arena, jobs,
                         max_segs, out, out_stride, outpos, offset, room, sizes, count, status, n_jobs);
    } else {  // (n_jobs rounded up to 8) x P blocks
      // in 64 bits before the check (n_jobs + 7 wrapped in 32)
      const uint64_t nblk = ((uint64_t)n_jobs + 7u) / 8u * 8u * (uint64_t)P;
      if (nblk > 0x7FFFFFFFull) return hipErrorInvalidValue;
      hipLaunchKernelGGL((gso_lds_kernel<NW, WGCS_GSO_U, true, P>), dim3((uint32_t)nblk), dim3(NW * 64), 0,
                         s, arena, jobs, max_segs, out, out_stride, outpos, offset, room, sizes, count, status, n_jobs);
    }
    return hipGetLastError();
  }
  // 16 segments (4 waves) per block and group; a few blocks per job, each
  // looping over its groups (a 65,535-B read at MSS 1460 has 3 groups)
  const uint32_t ngroups = (max_segs + 15) / 16;
  const uint32_t gy = ngroups < (uint32_t)WGCS_GSO_GROUPS ? ngroups : (uint32_t)WGCS_GSO_GROUPS;
  hipLaunchKernelGGL((gso_rows_kernel<WGCS_GSO_U, true>), dim3(n_jobs, gy), dim3(256), 0, s, arena, jobs, max_segs, out,
                     out_stride, outpos, offset, room, sizes, count, status);
  return hipGetLastError();
}

#endif  // !WGCS_RING_TU
}  // namespace wgcs
