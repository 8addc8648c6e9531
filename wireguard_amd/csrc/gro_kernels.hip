// gro_kernels.hip -- gfx950 GRO coalesce: builds the super-packets that
// handleGRO hands to the TUN fd (/root/reference/tun/gro.go:1326-1367), from
// the host's coalescing plan.
//
// The order-dependent flow-table logic (tcpGRO / udpGRO, gro.go:801-1095) runs
// on the host (gro_host.cpp) with checksumValid precomputed on the GPU; this
// kernel does the per-byte part of coalescing: the payload appends of
// coalesceTCPPackets / coalesceUDPPackets (gro.go:630-783) as one gather, and
// applyTCPCoalesce / applyUDPCoalesce (gro.go:1099-1268): IPv4 total length +
// header checksum or IPv6 payload length, UDP length, PSH, the virtio header,
// and the uncomplemented pseudo-header checksum in the L4 checksum field.
// One wave64 per output item header and one per payload piece (the host
// computes every piece's destination), so an item's pieces copy in parallel;
// pieces move with aligned 16-byte loads/stores (wgcs_copy.h).
#include <hip/hip_runtime.h>

#include "../../include/wgcsum.h"
#include "wgcs_common.h"
#include "wgcs_copy.h"
#include "wgcs_kernels.h"

namespace wgcs {

namespace {

struct HdrPatch {
  int iph, hdr_len, csum_at;
  uint32_t pkt_len;
  bool v6, udp, psh;
};

// Header byte x of the output packet before the two computed checksums
// (IPv4 header checksum and L4 pseudo-header partial are zero here).
__device__ __forceinline__ uint32_t patched(const uint8_t* head, const HdrPatch& h, int x) {
  uint32_t b = head[x];
  if (!h.v6) {
    if (x == 2) b = (h.pkt_len >> 8) & 0xFF;  // total length, uint16(len(pkt)) (gro.go:1131 / :1214)
    if (x == 3) b = h.pkt_len & 0xFF;
    if (x == 10 || x == 11) b = 0;   // :1134 / :1217
  } else {
    const uint32_t pl = h.pkt_len - (uint32_t)h.iph;  // payload length (:1124-1127 / :1207-1210)
    if (x == 4) b = (pl >> 8) & 0xFF;
    if (x == 5) b = pl & 0xFF;
  }
  if (h.udp) {
    const uint32_t ul = h.pkt_len - (uint32_t)h.iph;  // UDP length (:1229-1232)
    if (x == h.iph + 4) b = (ul >> 8) & 0xFF;
    if (x == h.iph + 5) b = ul & 0xFF;
  } else if (h.psh && x == h.iph + 13) {
    b |= 0x08;  // PSH appended (gro.go:724-729)
  }
  if (x == h.csum_at || x == h.csum_at + 1) b = 0;
  return b;
}

}  // namespace

__global__ __launch_bounds__(256) void gro_coalesce_kernel(const uint8_t* __restrict__ stage,
                                                           const GroItem* __restrict__ items, uint32_t n_items,
                                                           const GroSeg* __restrict__ segs, uint32_t n_segs,
                                                           uint8_t* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(blockIdx.x * 4 + (threadIdx.x >> 6)));
  if (wave >= n_items) {  // payload piece (coalesceTCPPackets / coalesceUDPPackets appends, gro.go:630-783)
    const uint32_t k = wave - n_items;
    if (k < n_segs) {
      const GroSeg sg = segs[k];
      copy_range(stage + sg.src_off, (int)sg.len, out + sg.dst_off, lane);
    }
    return;
  }
  {
    const uint32_t it = wave;
    const GroItem g = items[it];
    const uint8_t* head = stage + g.head_off;
    HdrPatch h;
    h.iph = g.iph;
    h.hdr_len = g.iph + g.l4h;
    h.v6 = g.kind & GRO_KIND_V6;
    h.udp = g.kind & GRO_KIND_UDP;
    h.psh = g.kind & GRO_KIND_PSH;
    h.csum_at = g.iph + (h.udp ? 6 : 16);
    h.pkt_len = g.pkt_len;
    uint8_t* o = out + g.out_off;
    if (g.kind & GRO_KIND_RAW) {  // coalesced, never applied (gro.go:1335-1337 returned first)
      for (int x = lane; x < h.hdr_len; x += 64) {
        uint32_t b = head[x];
        if (!h.udp && h.psh && x == h.iph + 13) b |= 0x08;  // PSH (gro.go:724-729)
        o[10 + x] = (uint8_t)b;
      }
      return;
    }
    // IPv4 header checksum: ^checksum(pkt[:iphLen], 0) after the patches
    uint32_t ipw = 0, adw = 0;
    const int a_lo = h.v6 ? 8 : 12, a_hi = h.v6 ? 40 : 20;
    for (int x = 2 * lane; x < h.iph; x += 128) {
      const uint32_t w = (patched(head, h, x) << 8) | (x + 1 < h.iph ? patched(head, h, x + 1) : 0u);
      if (!h.v6) ipw += w;
      if (x >= a_lo && x < a_hi) adw += w;
    }
    const uint32_t ipc = (~fold32_16(wave_sum_u32(ipw))) & 0xFFFF;
    // checksum([]byte{}, pseudoHeaderChecksumNoFold(src, dst, proto, len-iph)), not complemented
    const uint32_t pcs =
        fold32_16(fold32_16(wave_sum_u32(adw)) + (h.udp ? 17u : 6u) + ((h.pkt_len - (uint32_t)h.iph) & 0xFFFF));
    // virtio_net_hdr (gro.go:1107-1117 / :1191-1201), native byte order
    if (lane < 10) {
      const uint32_t gso_type = h.udp ? 5u : (h.v6 ? 4u : 1u);
      const uint32_t f[5] = {(uint32_t)h.hdr_len, g.gso_size, (uint32_t)h.iph, h.udp ? 6u : 16u, 0u};
      uint32_t b;
      if (lane == 0) b = 1;  // VIRTIO_NET_HDR_F_NEEDS_CSUM
      else if (lane == 1) b = gso_type;
      else b = (f[(lane - 2) >> 1] >> (8 * (lane & 1))) & 0xFF;
      o[lane] = (uint8_t)b;
    }
    for (int x = lane; x < h.hdr_len; x += 64) {
      uint32_t b = patched(head, h, x);
      if (!h.v6 && x == 10) b = ipc >> 8;
      if (!h.v6 && x == 11) b = ipc & 0xFF;
      if (x == h.csum_at) b = pcs >> 8;
      if (x == h.csum_at + 1) b = pcs & 0xFF;
      o[10 + x] = (uint8_t)b;
    }
  }
}

hipError_t launch_gro_coalesce(const uint8_t* stage, const GroItem* items, uint32_t n_items, const GroSeg* segs,
                               uint32_t n_segs, uint8_t* out, hipStream_t s) {
  if (n_items == 0) return hipSuccess;
  const uint32_t grid = (n_items + n_segs + 3) / 4;  // one wave per item header + one per piece
  hipLaunchKernelGGL(gro_coalesce_kernel, dim3(grid), dim3(256), 0, s, stage, items, n_items, segs, n_segs, out);
  return hipGetLastError();
}

}  // namespace wgcs
