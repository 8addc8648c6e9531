// gso_kernels.hip -- gfx950 GSO split (TSO/USO super-packet -> MSS segments).
//
// Device-resident batch of the reference's Tun.Read path:
//   handleVirtioRead validation/dispatch   /root/reference/tun/tun.go:514-632
//   gsoSplit                               /root/reference/tun/gro.go:1373-1493
//   gsoNoneChecksum (GSO_NONE + NEEDS_CSUM) /root/reference/tun/gro.go:1497-1517
//
// Mapping: one wave64 per OUTPUT segment ("slot" = job * max_segs + i).  Each
// wave re-derives its job's validation result with wave-uniform scalar code
// (a few header bytes, L2-resident after the first wave of the job), then:
//   1. assembles the patched headers of its segment in LDS (byte-parallel,
//      laid out at the destination's 16-byte phase) and computes the IPv4
//      header checksum and the pseudo-header address sum from it;
//   2. streams the payload: aligned 16-byte source loads, a 1-lane DPP/shuffle
//      funnel shift to the destination phase, full global_store_dwordx4 (byte
//      stores only on the packet's first/last partial chunk), summing the L4
//      bytes from the same registers;
//   3. writes the final L4 checksum into the LDS header, then stores the
//      header chunks -- so every output byte is written exactly once.
// Reference quirks reproduced bit-for-bit: IPv4 ID is
// id0 + 1 for every segment i >= 1; TCP seq uses a uint16 product
// gsoSize * uint16(i); FIN/PSH cleared on all but the last segment; no UDP
// 0 -> 0xFFFF substitution; ErrTooManySegments returns n = max_segs - 1.
#include <hip/hip_runtime.h>

#include "../../include/wgcsum.h"
#include "wgcs_common.h"
#include "wgcs_copy.h"
#include "wgcs_kernels.h"

namespace wgcs {

namespace {

constexpr int kHdrLds = 256;   // LDS bytes per wave for the segment headers
constexpr int kMaxHdrLen = 240;  // hdrLen + dest phase (<= 15) must fit kHdrLds

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
};

// Segment count / ErrTooManySegments (gro.go:1406-1410) + output room.
__device__ void count_segments(Job& j, uint32_t out_room, uint32_t max_segs) {
  const int plen = j.plen;
  long nseg = 0;
  if (j.hdr_len < plen) nseg = j.gso == 0 ? 0x7FFFFFFF : ((long)plen - j.hdr_len + j.gso - 1) / j.gso;
  if (nseg > 0) {
    const int first = j.hdr_len + min(j.gso, plen - j.hdr_len);
    if ((uint32_t)first > out_room) { j.status = WGCS_ERR_OUT_OF_RANGE; return; }
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

// gsoSplit's own slice bounds (gro.go:1388-1402,:1419,:1442,:1474-1475) and
// this kernel's header limits (Linux never produces violating TCP/UDP GSO
// headers).
__device__ bool split_bounds_ok(const Job& j) {
  const int plen = j.plen;
  const int csum_at = (j.cs + j.co) & 0xFFFF;
  const bool tcp = j.type != GSO_UDP_L4;
  if (j.cs > plen || j.hdr_len < j.cs || csum_at + 2 > plen || (tcp && j.cs + 8 > plen)) return false;
  if (j.ipv == 4 ? (plen < 20 || j.cs < 20) : (plen < 40 || j.cs < 40)) return false;
  if (csum_at + 2 > j.hdr_len || j.hdr_len > kMaxHdrLen) return false;
  return true;
}

// handleVirtioRead's checks (tun/tun.go:522-630) + this kernel's limits.
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
    if (!split_bounds_ok(j)) { j.status = WGCS_ERR_OUT_OF_RANGE; return j; }
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
  if (!split_bounds_ok(j)) { j.status = WGCS_ERR_OUT_OF_RANGE; return j; }
  count_segments(j, out_room, max_segs);
  return j;
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

// Per-job plan written by gso_plan_kernel, read by every segment wave.
struct GsoPlan {
  int32_t status, count, nseg, type;
  int32_t flags, ipv, hdr_len, gso;
  int32_t cs, co, plen, csum_at;
  uint32_t id0, first_seq, ip_base, addr_sum;  // ip_base: IPv4 header words with [2:6) and [10:12) zero
};
static_assert(sizeof(GsoPlan) == 64, "plan layout");
constexpr int kTplBytes = 256;  // header template per job (readBuf[:hdrLen] with the zeroed fields)

// Wave per job: handleVirtioRead validation, header template, header sums.
__global__ __launch_bounds__(256) void gso_plan_kernel(const uint8_t* __restrict__ arena,
                                                       const wgcs_gso_job* __restrict__ jobs, uint32_t n_jobs,
                                                       uint32_t room, uint32_t max_segs, GsoPlan* __restrict__ plans,
                                                       uint8_t* __restrict__ tpl, int32_t* __restrict__ count,
                                                       int32_t* __restrict__ status) {
  const int lane = threadIdx.x & 63;
  const uint32_t wave = (uint32_t)uni((int)(blockIdx.x * 4 + (threadIdx.x >> 6)));
  const uint32_t nwaves = gridDim.x * 4;
  for (uint32_t jb = wave; jb < n_jobs; jb += nwaves) {
    const uint8_t* vb = arena + jobs[jb].off;
    const uint32_t jlen = jobs[jb].len;
    HdrBytes hb;
    hb.load(vb, (int)min(jlen, 256u), lane);
    const Job j = decode_job(hb, jlen, jobs[jb].flags, room, max_segs);
    const bool ok = j.status == 0 || j.status == WGCS_ERR_TOO_MANY_SEGMENTS;
    GsoPlan P = {};
    P.status = j.status;
    P.count = ok ? j.count : 0;
    P.nseg = ok ? j.nseg : 0;
    P.type = j.type;
    P.flags = j.flags;
    P.ipv = j.ipv;
    P.hdr_len = j.hdr_len;
    P.gso = j.gso;
    P.cs = j.cs;
    P.co = j.co;
    P.plen = j.plen;
    P.csum_at = (j.cs + j.co) & 0xFFFF;
    if (ok && j.type != GSO_NONE) {
      const bool v4 = j.ipv == 4;
      P.id0 = v4 ? hb.be16(10 + 4) : 0;
      P.first_seq = j.type != GSO_UDP_L4 ? hb.be32(10 + j.cs + 4) : 0;
      // template byte x = readBuf[x] with readBuf's zeroed fields (gro.go:1388,:1393)
      uint8_t* t = tpl + (uint64_t)jb * kTplBytes;
      for (int x0 = 0; x0 < j.hdr_len; x0 += 64) {
        const int x = x0 + lane;
        uint32_t b = hb.lane_byte(min(10 + x, 255));
        if ((v4 && (x == 10 || x == 11)) || x == P.csum_at || x == P.csum_at + 1) b = 0;
        if (x < j.hdr_len) t[x] = (uint8_t)b;
      }
      // IPv4 header words with [2:6) and [10:12) zero; pseudo-header address words
      const int a_lo = v4 ? 12 : 8, a_hi = v4 ? 20 : 40;
      uint32_t ipw = 0, adw = 0;
      for (int r = 0; r < 2; ++r) {  // header bytes [0, 256): two rounds of 64 words
        const int x = 2 * lane + 128 * r;
        const uint32_t hi = hb.lane_byte(min(10 + x, 255)), lo = hb.lane_byte(min(11 + x, 255));
        const uint32_t w = (hi << 8) | (x + 1 < j.cs ? lo : 0u);
        if (v4 && x < j.cs && x != 2 && x != 4 && x != 10) ipw += w;
        if (x >= a_lo && x < a_hi) adw += w;
      }
      P.ip_base = fold32_16(wave_sum_u32(ipw));
      P.addr_sum = fold32_16(wave_sum_u32(adw));
    }
    if (lane == 0) {
      plans[jb] = P;
      count[jb] = P.count;
      status[jb] = P.status;
    }
  }
}

// One output segment (gro.go:1408-1491 for one i), in two phases: seg_begin
// computes the segment geometry and issues its payload loads; seg_finish
// builds the header while they land, streams the payload to the destination
// and writes the checksums.
struct Seg {
  const uint8_t* rb;     // readBuf (after the virtio header)
  const uint8_t* t;      // header template of the job
  const uint8_t* pay0;   // source of packet position x >= hdr_len is pay0 + x
  uint8_t* dst;          // destination packet start
  int i, pkt_len, seg_len, dalign, nk, hk;
  long seg_start, seg_end;
  bool active, none;
  CopyBatch pay;
};

__device__ __forceinline__ Seg seg_begin(const uint8_t* __restrict__ arena, const wgcs_gso_job* __restrict__ jobs,
                                         const GsoPlan& P, const uint8_t* tpl, uint8_t* out, uint32_t slot, uint32_t jb,
                                         int i, uint32_t out_stride, uint32_t offset, bool in_range, int lane) {
  Seg g;
  g.active = in_range && i < P.nseg;
  g.none = P.type == GSO_NONE;
  g.i = i;
  g.rb = arena + jobs[jb].off + 10;
  g.t = tpl + (uint64_t)jb * kTplBytes;
  g.dst = out + (uint64_t)slot * out_stride + offset;
  g.seg_start = (long)P.hdr_len + (long)i * P.gso;
  g.seg_end = min((long)P.plen, g.seg_start + P.gso);
  g.seg_len = (int)(g.seg_end - g.seg_start);
  g.pkt_len = P.hdr_len + g.seg_len;
  g.dalign = (int)((uintptr_t)g.dst & 15);
  g.nk = (g.pkt_len + g.dalign + 15) >> 4;
  g.hk = min((P.hdr_len + g.dalign + 15) >> 4, g.nk);
  g.pay0 = g.rb + (long)i * P.gso;
  if (g.active && !g.none)
    g.pay = copy_batch_load(g.pay0, g.rb + g.seg_start, g.rb + g.seg_end, g.dalign, g.hk, g.nk, lane);
  return g;
}

__device__ void seg_finish(const Seg& g, const GsoPlan& j, uint8_t* lds, int32_t* sizes, uint32_t slot, int lane) {
  if (!g.active) return;
  if (g.none) {
    Job jj = {};
    jj.flags = j.flags;
    jj.cs = j.cs;
    jj.co = j.co;
    jj.plen = j.plen;
    none_segment(g.rb, jj, g.dst, lane);
    if (lane == 0) sizes[slot] = j.plen;
    return;
  }
  const bool v4 = j.ipv == 4;
  const bool tcp = j.type != GSO_UDP_L4;
  const int hdr_len = j.hdr_len, cs = j.cs, iph = cs;
  const int pkt_len = g.pkt_len, dalign = g.dalign, nk = g.nk, hk = g.hk, i = g.i;
  const int csum_at = j.csum_at;
  const uint32_t id = i > 0 ? ((j.id0 + 1) & 0xFFFF) : j.id0;  // quirk: id0 + 1 for every i >= 1
  const uint32_t seq = j.first_seq + (uint32_t)(uint16_t)((uint16_t)j.gso * (uint16_t)i);  // uint16 product
  const bool last = g.seg_end == j.plen;
  const uint32_t ulen = (uint32_t)(uint16_t)(g.seg_len + (hdr_len - cs));
  const uint32_t ipc = (~fold32_16(j.ip_base + (uint32_t)pkt_len + id)) & 0xFFFF;  // (:1433-1436)
  uint8_t* dbase = g.dst - dalign;

  // ---- 1. patched header (+ the payload bytes sharing its last chunk) into LDS
  for (int L = lane; L < 16 * hk; L += 64) {
    const int x = L - dalign;
    uint32_t b = 0;
    if (x >= 0 && x < pkt_len) {
      if (x < hdr_len) {
        b = g.t[x];
        if (v4) {
          if (x == 2) b = (uint32_t)pkt_len >> 8;  // total length (:1433)
          if (x == 3) b = (uint32_t)pkt_len & 0xFF;
          if (x == 4) b = id >> 8;                 // identification (:1426-1431)
          if (x == 5) b = id & 0xFF;
          if (x == 10) b = ipc >> 8;               // header checksum (:1434-1436)
          if (x == 11) b = ipc & 0xFF;
        } else {
          if (x == 4) b = (uint32_t)(pkt_len - iph) >> 8 & 0xFF;  // payload length (:1439)
          if (x == 5) b = (uint32_t)(pkt_len - iph) & 0xFF;
        }
        if (tcp) {
          if (x >= cs + 4 && x < cs + 8) b = (seq >> (8 * (cs + 7 - x))) & 0xFF;  // (:1445-1446)
          if (x == cs + 13 && !last) b &= ~(uint32_t)0x09;                       // clear FIN|PSH (:1447-1459)
        } else {
          if (x >= cs + 4 && x < cs + 6) b = (ulen >> (8 * (cs + 5 - x))) & 0xFF;  // UDP length (:1462-1465)
        }
      } else {
        b = g.pay0[x];
      }
    }
    lds[L] = (uint8_t)b;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

  // ---- 2. L4 sum: header chunks from LDS, payload chunks streamed + stored
  uint64_t acc = 0;
  uint4 hv = make_uint4(0, 0, 0, 0);
  if (lane < hk) {
    hv = *reinterpret_cast<const uint4*>(lds + 16 * lane);
    acc += chunk_sum(hv, 16 * lane - dalign, cs, pkt_len);
  }
  copy_batch_store<true>(g.pay, dbase, dalign, nk, pkt_len, cs, lane, acc);
  if (nk > hk + 128)  // segments longer than 2 KiB: stream the rest
    stream_copy<true>(g.pay0, g.rb + g.seg_start, g.rb + g.seg_end, dbase, dalign, hk + 128, nk, pkt_len, cs, -1, 0,
                      lane, acc);
  uint32_t s = fold32_16(wave_sum_u32(fold64_16(acc)));
  if ((((uintptr_t)g.dst + (uintptr_t)cs) & 1u) == 0) s = bswap16(s);
  const uint32_t tlen = (uint32_t)(uint16_t)(hdr_len - cs + g.seg_len);  // transportLen (:1469-1471)
  const uint32_t tt = fold32_16(s + j.addr_sum + (tcp ? 6u : 17u) + tlen);
  const uint32_t l4c = (~tt) & 0xFFFF;  // ^checksum(pkt[csumStart:pktLen], pseudo) (:1480-1488)

  // ---- 3. final checksum into the header chunk, then store the header chunks
  if (lane < hk) {
    const int x0 = 16 * lane - dalign;
    const int j0 = csum_at - x0, j1 = csum_at + 1 - x0;
    if (j0 >= 0 && j0 < 16) hv = set_chunk_byte(hv, j0, l4c >> 8);
    if (j1 >= 0 && j1 < 16) hv = set_chunk_byte(hv, j1, l4c);
    store_chunk(dbase + 16 * lane, hv, x0, pkt_len);
  }
  if (lane == 0) sizes[slot] = pkt_len;
  __builtin_amdgcn_wave_barrier();  // the LDS header region is reused by the next segment
}

__global__ __launch_bounds__(256) void gso_split_kernel(const uint8_t* __restrict__ arena,
                                                        const wgcs_gso_job* __restrict__ jobs, uint32_t n_jobs,
                                                        const GsoPlan* __restrict__ plans,
                                                        const uint8_t* __restrict__ tpl, uint8_t* __restrict__ out,
                                                        uint32_t out_stride, uint32_t offset, uint32_t max_segs,
                                                        int32_t* __restrict__ sizes) {
  __shared__ __attribute__((aligned(16))) uint8_t lds_all[4][kHdrLds];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  uint8_t* lds = lds_all[wv];
  const uint32_t wave = (uint32_t)uni((int)(blockIdx.x * 4 + wv));
  const uint32_t nwaves = gridDim.x * 4;
  const uint32_t total = n_jobs * max_segs;
  for (uint32_t sa = wave; sa < total; sa += nwaves) {
    const uint32_t ja = sa / max_segs;
    const GsoPlan PA = plans[ja];
    const int i = (int)(sa - ja * max_segs);
    if (i >= PA.nseg) continue;
    const Seg A = seg_begin(arena, jobs, PA, tpl, out, sa, ja, i, out_stride, offset, true, lane);
    seg_finish(A, PA, lds, sizes, sa, lane);
  }
}

size_t gso_workspace_bytes(uint32_t n_jobs) { return (size_t)n_jobs * (sizeof(GsoPlan) + kTplBytes); }

hipError_t launch_gso_split_batch(const uint8_t* arena, const wgcs_gso_job* jobs, uint32_t n_jobs, uint8_t* out,
                                  uint32_t out_stride, uint32_t offset, uint32_t max_segs, int32_t* sizes,
                                  int32_t* count, int32_t* status, void* workspace, hipStream_t s, int num_cu) {
  if (n_jobs == 0 || max_segs == 0) return hipSuccess;
  GsoPlan* plans = reinterpret_cast<GsoPlan*>(workspace);
  uint8_t* tpl = reinterpret_cast<uint8_t*>(plans + n_jobs);
  const uint32_t room = out_stride > offset ? out_stride - offset : 0;
  uint32_t g1 = (n_jobs + 3) / 4;
  if (g1 > (uint32_t)num_cu * 8) g1 = (uint32_t)num_cu * 8;
  hipLaunchKernelGGL(gso_plan_kernel, dim3(g1), dim3(256), 0, s, arena, jobs, n_jobs, room, max_segs, plans, tpl,
                     count, status);
  const uint64_t slots = (uint64_t)n_jobs * max_segs;
  uint64_t want = (slots + 3) / 4;
  const uint64_t cap = (uint64_t)num_cu * 8;
  const int grid = (int)(want < cap ? want : cap);
  hipLaunchKernelGGL(gso_split_kernel, dim3(grid), dim3(256), 0, s, arena, jobs, n_jobs, plans, tpl, out, out_stride,
                     offset, max_segs, sizes);
  return hipGetLastError();
}

}  // namespace wgcs
