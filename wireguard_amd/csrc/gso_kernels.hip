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
constexpr int kSlotsPerWave = 2;  // output segments per wave (amortizes the header decode)

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

__device__ void gso_segment(const uint8_t* rb, const HdrBytes& hb, const Job& j, int i, uint8_t* dst, uint8_t* lds,
                            int lane) {
  const bool v4 = j.ipv == 4;
  const bool tcp = j.type != GSO_UDP_L4;
  const int hdr_len = j.hdr_len, cs = j.cs, plen = j.plen;
  const int iph = cs;
  const long seg_start = (long)hdr_len + (long)i * j.gso;
  const int seg_end = (int)min((long)plen, seg_start + j.gso);
  const int seg_len = seg_end - (int)seg_start;
  const int pkt_len = hdr_len + seg_len;
  const int csum_at = (cs + j.co) & 0xFFFF;
  // per-segment header values (gro.go:1419-1466)
  const uint32_t id0 = v4 ? hb.be16(10 + 4) : 0;
  const uint32_t id1 = (id0 + 1) & 0xFFFF;                                     // quirk: +1 for every i >= 1
  const uint32_t first_seq = tcp ? hb.be32(10 + cs + 4) : 0;
  const uint32_t seq = first_seq + (uint32_t)(uint16_t)((uint16_t)j.gso * (uint16_t)i);  // uint16 product
  const bool last = seg_end == plen;
  const uint32_t ulen = (uint32_t)(uint16_t)(seg_len + (hdr_len - cs));
  const int dalign = (int)((uintptr_t)dst & 15);
  uint8_t* dbase = dst - dalign;
  const int nk = (pkt_len + dalign + 15) >> 4;
  const int hk = min((hdr_len + dalign + 15) >> 4, nk);  // chunks assembled in LDS
  const uint8_t* pay_src0 = rb + (long)i * j.gso;  // source of position x >= hdr_len

  // ---- 1. patched header (+ the payload bytes sharing its last chunk) into LDS
  for (int L = lane; L < 16 * hk; L += 64) {
    const int x = L - dalign;
    uint32_t b = 0;
    if (x >= 0 && x < pkt_len) {
      if (x < hdr_len) {
        b = rb[x];
        if (x >= csum_at && x < csum_at + 2) b = 0;  // readBuf csum field zeroed (gro.go:1393)
        if (v4) {
          if (x == 10 || x == 11) b = 0;           // readBuf[10:12] zeroed (:1388)
          if (x == 2) b = (uint32_t)pkt_len >> 8;  // total length (:1433)
          if (x == 3) b = (uint32_t)pkt_len & 0xFF;
          if (i > 0 && x == 4) b = id1 >> 8;       // identification (:1426-1431)
          if (i > 0 && x == 5) b = id1 & 0xFF;
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
        b = pay_src0[x];
      }
    }
    lds[L] = (uint8_t)b;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

  // ---- 2. IPv4 header checksum and pseudo-header address sum (BE words)
  const int a_lo = v4 ? 12 : 8, a_hi = v4 ? 20 : 40;
  uint32_t ipw = 0, adw = 0;
  for (int x = 2 * lane; x < iph; x += 128) {
    const uint32_t hi = lds[x + dalign];
    const uint32_t lo = (x + 1 < iph) ? lds[x + 1 + dalign] : 0u;
    if (v4) ipw += (hi << 8) | lo;
    if (x >= a_lo && x < a_hi) adw += (hi << 8) | lo;
  }
  const uint32_t ip_sum = fold32_16(wave_sum_u32(ipw));
  const uint32_t addr_sum = fold32_16(wave_sum_u32(adw));
  if (v4 && lane == 0) {
    const uint32_t ipc = (~ip_sum) & 0xFFFF;  // ^checksum(pkt[:iphLen], 0) (:1434-1436)
    lds[10 + dalign] = (uint8_t)(ipc >> 8);
    lds[11 + dalign] = (uint8_t)ipc;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

  // ---- 3. L4 sum: header chunks from LDS, payload chunks streamed + stored
  uint64_t acc = 0;
  uint4 hv = make_uint4(0, 0, 0, 0);
  if (lane < hk) {
    hv = *reinterpret_cast<const uint4*>(lds + 16 * lane);
    acc += chunk_sum(hv, 16 * lane - dalign, cs, pkt_len);
  }
  stream_copy<true>(pay_src0, rb + seg_start, rb + seg_end, dbase, dalign, hk, nk, pkt_len, cs, -1, 0, lane, acc);
  uint32_t s = fold32_16(wave_sum_u32(fold64_16(acc)));
  if ((((uintptr_t)dst + (uintptr_t)cs) & 1u) == 0) s = bswap16(s);
  const uint32_t proto = tcp ? 6u : 17u;
  const uint32_t tlen = (uint32_t)(uint16_t)(hdr_len - cs + seg_len);  // transportLen (:1469-1471)
  const uint32_t t = fold32_16(s + addr_sum + proto + tlen);
  const uint32_t l4c = (~t) & 0xFFFF;  // ^checksum(pkt[csumStart:pktLen], pseudo) (:1480-1488)

  // ---- 4. final checksum into the header chunk, then store the header chunks
  if (lane < hk) {
    const int x0 = 16 * lane - dalign;
    const int j0 = csum_at - x0, j1 = csum_at + 1 - x0;
    if (j0 >= 0 && j0 < 16) hv = set_chunk_byte(hv, j0, l4c >> 8);
    if (j1 >= 0 && j1 < 16) hv = set_chunk_byte(hv, j1, l4c);
    store_chunk(dbase + 16 * lane, hv, x0, pkt_len);
  }
}

}  // namespace

__global__ __launch_bounds__(256) void gso_split_kernel(const uint8_t* __restrict__ arena,
                                                        const wgcs_gso_job* __restrict__ jobs, uint32_t n_jobs,
                                                        uint8_t* __restrict__ out, uint32_t out_stride,
                                                        uint32_t offset, uint32_t max_segs, int32_t* __restrict__ sizes,
                                                        int32_t* __restrict__ count, int32_t* __restrict__ status) {
  __shared__ __attribute__((aligned(16))) uint8_t lds_all[4][kHdrLds];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  uint8_t* lds = lds_all[wv];
  const uint64_t wave = (uint64_t)uni((int)(blockIdx.x * 4 + wv));
  const uint64_t nwaves = (uint64_t)gridDim.x * 4;
  const uint32_t room = out_stride > offset ? out_stride - offset : 0;
  const uint32_t groups_per_job = (max_segs + kSlotsPerWave - 1) / kSlotsPerWave;
  const uint64_t total_groups = (uint64_t)n_jobs * groups_per_job;
  for (uint64_t g = wave; g < total_groups; g += nwaves) {
    const uint32_t jb = (uint32_t)(g / groups_per_job);
    const int i0 = (int)(g - (uint64_t)jb * groups_per_job) * kSlotsPerWave;
    const uint64_t joff = jobs[jb].off;
    const uint32_t jlen = jobs[jb].len;
    const uint32_t jflags = jobs[jb].flags;
    const uint8_t* vb = arena + joff;
    HdrBytes hb;
    hb.load(vb, (int)min(jlen, 256u), lane);
    const Job j = decode_job(hb, jlen, jflags, room, max_segs);
    if (i0 == 0 && lane == 0) {
      count[jb] = j.status && j.status != WGCS_ERR_TOO_MANY_SEGMENTS ? 0 : j.count;
      status[jb] = j.status;
    }
    if (j.status && j.status != WGCS_ERR_TOO_MANY_SEGMENTS) continue;
    const int i_end = min(i0 + kSlotsPerWave, j.nseg);
    for (int i = i0; i < i_end; ++i) {
      const uint64_t slot = (uint64_t)jb * max_segs + i;
      uint8_t* dst = out + slot * (uint64_t)out_stride + offset;
      if (j.type == GSO_NONE) {
        none_segment(vb + 10, j, dst, lane);
        if (lane == 0) sizes[slot] = j.plen;
      } else {
        gso_segment(vb + 10, hb, j, i, dst, lds, lane);
        if (lane == 0) {
          const long seg_start = (long)j.hdr_len + (long)i * j.gso;
          const long seg_end = min((long)j.plen, seg_start + j.gso);
          sizes[slot] = (int32_t)(j.hdr_len + (seg_end - seg_start));
        }
      }
    }
  }
}

hipError_t launch_gso_split_batch(const uint8_t* arena, const wgcs_gso_job* jobs, uint32_t n_jobs, uint8_t* out,
                                  uint32_t out_stride, uint32_t offset, uint32_t max_segs, int32_t* sizes,
                                  int32_t* count, int32_t* status, hipStream_t s, int num_cu) {
  if (n_jobs == 0 || max_segs == 0) return hipSuccess;
  const uint64_t groups = (uint64_t)n_jobs * ((max_segs + kSlotsPerWave - 1) / kSlotsPerWave);
  uint64_t want = (groups + 3) / 4;
  const uint64_t cap = (uint64_t)num_cu * 8;
  const int grid = (int)(want < cap ? want : cap);
  hipLaunchKernelGGL(gso_split_kernel, dim3(grid), dim3(256), 0, s, arena, jobs, n_jobs, out, out_stride, offset,
                     max_segs, sizes, count, status);
  return hipGetLastError();
}

}  // namespace wgcs
