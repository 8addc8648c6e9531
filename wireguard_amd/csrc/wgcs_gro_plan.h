// wgcs_gro_plan.h -- the host half of handleGRO (/root/reference/tun/gro.go:
// 1326-1367): the order-dependent flow-table decisions of tcpGRO / udpGRO
// (gro.go:801-1095: flows keyed by addresses, ports and ack, sequence
// adjacency, PSH, capacity, prepend swaps), on headers and lengths only.  No
// payload byte is touched: appends are recorded as a gather plan of pieces per
// output buffer, and apply{TCP,UDP}Coalesce (gro.go:1099-1268) becomes one
// GroItem per merged buffer for the GPU coalesce kernel (gro_kernels.hip).
// checksumValid (gro.go:554-612) comes in as precomputed bits (`valid`): the
// reference validates before it mutates (gro.go:665-681, :709-723, :767-775),
// so bits computed up front by the VALIDATE kernel are exact; the bits a plan
// depended on are recorded (`consulted`) so a plan made on assumed bits can be
// checked.  Shared by wgcs_handle_gro (gro_host.cpp) and the Tun.Write stager
// (wstager.cpp).
#pragma once

#include <stdint.h>

#include <algorithm>
#include <cstring>
#include <unordered_map>
#include <vector>

#include "wgcs_host.h"

namespace wgcs {
namespace gro {

constexpr int kVnetLen = 10;
constexpr uint8_t kFin = 0x01, kPsh = 0x08, kAck = 0x10;
enum Cand { NOT_CAND = 0, TCP4 = 1, TCP6 = 2, UDP4 = 3, UDP6 = 4 };
enum GroResult { NOOP, INSERT, COALESCED };
enum CanCoalesce { PREPEND = -1, UNAVAILABLE = 0, APPEND = 1 };
enum CoalesceResult { INSUFF_CAP, PSH_ENDING, ITEM_BAD, PKT_BAD, SUCCESS };

inline uint16_t be16(const uint8_t* p) { return (uint16_t)((p[0] << 8) | p[1]); }
inline uint32_t be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

struct FlowKey {  // tcpFlowKey / udpFlowKey (gro.go:96-127, :252-275); ack = 0 for UDP
  uint8_t src[16], dst[16];
  uint16_t sport, dport;
  uint32_t ack;
  uint8_t v6;
  bool operator==(const FlowKey& o) const {
    return !memcmp(src, o.src, 16) && !memcmp(dst, o.dst, 16) && sport == o.sport && dport == o.dport &&
           ack == o.ack && v6 == o.v6;
  }
};
struct FlowHash {
  size_t operator()(const FlowKey& k) const {
    uint64_t h = 1469598103934665603ull;
    auto mix = [&](const uint8_t* p, size_t n) {
      for (size_t i = 0; i < n; ++i) h = (h ^ p[i]) * 1099511628211ull;
    };
    mix(k.src, 16);
    mix(k.dst, 16);
    mix((const uint8_t*)&k.sport, 2);
    mix((const uint8_t*)&k.dport, 2);
    mix((const uint8_t*)&k.ack, 4);
    h ^= k.v6;
    return (size_t)h;
  }
};

struct Item {  // tcpGROItem (gro.go:131-149) / udpGROItem (:279-293)
  FlowKey key;
  uint32_t seq = 0;
  uint16_t bufs_index = 0, num_merged = 0, gso_size = 0;
  uint8_t iph = 0, l4h = 0;
  bool psh = false, csum_bad = false;
};

struct Piece {
  int pkt;  // original packet index (its bytes are at stage_off[pkt])
  uint32_t start, len;
};
struct Content {  // the bytes a Go buffer holds: pieces in order + PSH OR'ed into its header
  std::vector<Piece> pieces;
  bool psh = false;
};

struct Planner {
  uint8_t** bufs;
  size_t* lens;
  size_t* caps;
  int n, offset;
  std::vector<const uint8_t*> orig;   // original packet starts (host)
  std::vector<uint8_t> valid;          // checksumValid per original index (GPU, or assumed)
  std::vector<uint8_t> consulted;      // validity bits the decisions depended on
  std::vector<Content> content;        // per slot, swapped with bufs
  std::unordered_map<FlowKey, std::vector<Item>, FlowHash> tcp, udp;

  bool V(int i) {  // checksumValid of the packet at slot i, recording that the plan used it
    consulted[i] = 1;
    return valid[i] != 0;
  }

  // header bytes of the buffer now at `slot` (the head packet's original header)
  const uint8_t* head(int slot) const { return orig[content[slot].pieces[0].pkt]; }
  size_t plen(int slot) const { return lens[slot] - (size_t)offset; }

  void swap_slots(int a, int b) {
    std::swap(bufs[a], bufs[b]);
    std::swap(lens[a], lens[b]);
    std::swap(caps[a], caps[b]);
    std::swap(content[a], content[b]);
  }

  static FlowKey key_of(const uint8_t* pkt, int src_off, int alen, int l4_off, bool tcp) {
    FlowKey k;
    memset(&k, 0, sizeof k);
    memcpy(k.src, pkt + src_off, (size_t)alen);
    memcpy(k.dst, pkt + src_off + alen, (size_t)alen);
    k.sport = be16(pkt + l4_off);
    k.dport = be16(pkt + l4_off + 2);
    k.ack = tcp ? be32(pkt + l4_off + 8) : 0;
    k.v6 = alen == 16;
    return k;
  }

  // gro.go:392-427
  static bool ip_headers_can_coalesce(const uint8_t* a, size_t la, const uint8_t* b, size_t lb) {
    if (la < 9 || lb < 9) return false;
    if (a[0] >> 4 == 6) {
      if (a[0] != b[0] || a[1] >> 4 != b[1] >> 4) return false;
      if (a[7] != b[7]) return false;
    } else {
      if (a[1] != b[1]) return false;
      if (a[6] >> 5 != b[6] >> 5) return false;
      if (a[8] != b[8]) return false;
    }
    return true;
  }

  // gro.go:433-512
  int tcp_can_coalesce(const uint8_t* pkt, size_t pl, uint8_t iph, uint8_t th, uint32_t seq, bool psh, uint16_t gso,
                       const Item& it) const {
    const uint8_t* tgt = head(it.bufs_index);
    const size_t tl = plen(it.bufs_index);
    if (th != it.l4h) return UNAVAILABLE;
    if (th > 20 && memcmp(pkt + iph + 20, tgt + it.iph + 20, (size_t)(th - 20))) return UNAVAILABLE;
    if (!ip_headers_can_coalesce(pkt, pl, tgt, tl)) return UNAVAILABLE;
    const uint16_t lhs = (uint16_t)(it.gso_size + (uint16_t)(it.gso_size * it.num_merged));
    if (seq == it.seq + (uint32_t)lhs) {
      if (it.psh) return UNAVAILABLE;
      if ((tl - (size_t)(iph + th)) % it.gso_size != 0) return UNAVAILABLE;
      if (gso > it.gso_size) return UNAVAILABLE;
      return APPEND;
    } else if (seq + (uint32_t)gso == it.seq) {
      if (psh) return UNAVAILABLE;
      if (gso < it.gso_size) return UNAVAILABLE;
      if (gso > it.gso_size && it.num_merged > 0) return UNAVAILABLE;
      return PREPEND;
    }
    return UNAVAILABLE;
  }

  // gro.go:630-741 (payload copies become pieces)
  int coalesce_tcp(int mode, int bi, uint16_t gso, uint32_t seq, bool psh, Item& it) {
    const size_t pl = plen(bi);
    const uint32_t hdrs = (uint8_t)(it.iph + it.l4h);
    const size_t pay = pl - hdrs;
    const size_t new_len = plen(it.bufs_index) + pay;
    if (mode == PREPEND) {
      if (caps[bi] - (size_t)offset < new_len) return INSUFF_CAP;
      if (psh) return PSH_ENDING;
      if (it.num_merged == 0 && !V(it.bufs_index)) return ITEM_BAD;
      if (!V(bi)) return PKT_BAD;
      it.seq = seq;
      const size_t item_pay = new_len - pl;
      Content& dst = content[bi];
      const Content& src = content[it.bufs_index];
      const Piece& h0 = src.pieces[0];  // drop the item's headers (gro.go:690-693)
      dst.pieces.push_back({h0.pkt, h0.start + hdrs, h0.len - hdrs});
      dst.pieces.insert(dst.pieces.end(), src.pieces.begin() + 1, src.pieces.end());
      lens[bi] += item_pay;
      swap_slots(it.bufs_index, bi);  // gro.go:696-697
    } else {
      if (caps[it.bufs_index] - (size_t)offset < new_len) return INSUFF_CAP;
      if (it.num_merged == 0 && !V(it.bufs_index)) return ITEM_BAD;
      if (!V(bi)) return PKT_BAD;
      if (psh) {
        it.psh = true;
        content[it.bufs_index].psh = true;  // pktHead[iphLen+13] |= PSH (gro.go:724-729)
      }
      content[it.bufs_index].pieces.push_back({bi, hdrs, (uint32_t)pay});
      lens[it.bufs_index] += pay;
    }
    it.gso_size = std::max(it.gso_size, gso);
    it.num_merged++;
    return SUCCESS;
  }

  // gro.go:801-963
  int tcp_gro(int bi, bool v6) {
    const uint8_t* pkt = orig[bi];
    const size_t pl = plen(bi);
    if (pl > 65535) return NOOP;
    int iph = (uint8_t)((pkt[0] & 0x0F) * 4);
    if (v6) {
      iph = 40;
      if ((int)be16(pkt + 4) != (int)pl - iph) return NOOP;
    } else if ((size_t)be16(pkt + 2) != pl) {
      return NOOP;
    }
    if (pl < (size_t)iph) return NOOP;
    const int th = (uint8_t)((pkt[iph + 12] >> 4) * 4);
    if (th < 20 || th > 60) return NOOP;
    if (pl < (size_t)(iph + th)) return NOOP;
    if (!v6 && ((pkt[6] & 0x20) || (uint8_t)(pkt[6] << 3) || pkt[7])) return NOOP;
    const uint8_t flags = pkt[iph + 13];
    bool psh = false;
    if (flags != kAck) {
      if (flags != (kAck | kPsh)) return NOOP;
      psh = true;
    }
    const uint16_t gso = (uint16_t)(pl - (size_t)iph - (size_t)th);
    if (gso < 1) return NOOP;
    const uint32_t seq = be32(pkt + iph + 4);
    const int src_off = v6 ? 8 : 12, alen = v6 ? 16 : 4;
    const FlowKey key = key_of(pkt, src_off, alen, iph, true);
    Item ni;
    ni.key = key;
    ni.bufs_index = (uint16_t)bi;
    ni.gso_size = gso;
    ni.iph = (uint8_t)iph;
    ni.l4h = (uint8_t)th;
    ni.seq = seq;
    ni.psh = (flags & kPsh) != 0;
    auto f = tcp.find(key);
    if (f == tcp.end()) {
      tcp[key].push_back(ni);
      return INSERT;
    }
    std::vector<Item>& items = f->second;
    for (int i = (int)items.size() - 1; i >= 0; --i) {
      Item item = items[i];
      const int can = tcp_can_coalesce(pkt, pl, (uint8_t)iph, (uint8_t)th, seq, psh, gso, item);
      if (can == UNAVAILABLE) continue;
      const int r = coalesce_tcp(can, bi, gso, seq, psh, item);
      if (r == SUCCESS) {
        items[i] = item;
        return COALESCED;
      }
      if (r == ITEM_BAD) items.erase(items.begin() + i);  // deleteAt (gro.go:241-247)
      else if (r == PKT_BAD) return NOOP;
    }
    items.push_back(ni);
    return INSERT;
  }

  // gro.go:971-1095
  int udp_gro(int bi, bool v6) {
    const uint8_t* pkt = orig[bi];
    const size_t pl = plen(bi);
    if (pl > 65535) return NOOP;
    int iph = (uint8_t)((pkt[0] & 0x0F) * 4);
    if (v6) {
      iph = 40;
      if ((int)be16(pkt + 4) != (int)pl - iph) return NOOP;
    } else if ((size_t)be16(pkt + 2) != pl) {
      return NOOP;
    }
    if (pl < (size_t)(iph + 8)) return NOOP;
    if (!v6 && ((pkt[6] & 0x20) || (uint8_t)(pkt[6] << 3) || pkt[7])) return NOOP;
    const uint16_t gso = (uint16_t)(pl - (size_t)iph - 8);
    if (gso < 1) return NOOP;
    const int src_off = v6 ? 8 : 12, alen = v6 ? 16 : 4;
    const FlowKey key = key_of(pkt, src_off, alen, iph, false);
    Item ni;
    ni.key = key;
    ni.bufs_index = (uint16_t)bi;
    ni.gso_size = gso;
    ni.iph = (uint8_t)iph;
    ni.l4h = 8;
    auto f = udp.find(key);
    if (f == udp.end()) {
      udp[key].push_back(ni);
      return INSERT;
    }
    std::vector<Item>& items = f->second;
    Item item = items.back();
    bool bad = false;
    // udpPacketsCanCoalesce (gro.go:519-544)
    const uint8_t* tgt = head(item.bufs_index);
    const size_t tl = plen(item.bufs_index);
    bool can = ip_headers_can_coalesce(pkt, pl, tgt, tl) && (tl - (size_t)(iph + 8)) % item.gso_size == 0 &&
               gso <= item.gso_size;
    if (can) {
      // coalesceUDPPackets (gro.go:745-783)
      const uint32_t hdrs = (uint8_t)(item.iph + 8);
      const size_t pay = pl - hdrs;
      int r;
      if (caps[item.bufs_index] - (size_t)offset < tl + pay) r = INSUFF_CAP;
      else if (item.num_merged == 0 && (item.csum_bad || !V(item.bufs_index))) r = ITEM_BAD;
      else if (!V(bi)) r = PKT_BAD;
      else {
        content[item.bufs_index].pieces.push_back({bi, hdrs, (uint32_t)pay});
        lens[item.bufs_index] += pay;
        item.num_merged++;
        r = SUCCESS;
      }
      if (r == SUCCESS) {
        items.back() = item;
        return COALESCED;
      }
      if (r == PKT_BAD) bad = true;
    }
    ni.csum_bad = bad;
    items.push_back(ni);
    return INSERT;
  }
};

// gro.go:1280-1317
inline int gro_candidate(const uint8_t* pkt, size_t len, bool can_udp) {
  if (len < 28) return NOT_CAND;
  switch (pkt[0] >> 4) {
    case 4:
      if ((pkt[0] & 0x0F) != 5) return NOT_CAND;
      if (pkt[9] == 6 && len >= 40) return TCP4;
      if (pkt[9] == 17 && can_udp) return UDP4;
      break;
    case 6:
      if (pkt[6] == 6 && len >= 60) return TCP6;
      if (pkt[6] == 17 && len >= 48 && can_udp) return UDP6;
      break;
  }
  return NOT_CAND;
}

// The host half of one handleGRO: flow decisions (gro.go:1334-1363) and the
// applyTCPCoalesce / applyUDPCoalesce gather plan (:1364-1366) for the given
// validity bits.  Nothing is written to the caller's bytes here (only the
// bufs/lens/caps slice headers move, as the Go code moves them).
struct Plan {
  std::vector<int> to_write, zero_hdr;  // slots to write; slots whose virtio header is all-zero
  std::vector<GroItem> items;
  std::vector<GroSeg> segs;
  std::vector<int> item_slot;
  uint64_t out_bytes = 0;
};

// raw: the loop stopped at packet `n_eff` with "invalid offset" (gro.go:1335-
// 1337): no apply* runs, so every buffer whose bytes the coalescing changed
// (appends, prepend swaps, PSH) becomes a RAW item holding exactly those bytes.
inline void make_plan(Planner& P, const std::vector<int>& cand, const std::vector<uint64_t>& stage_off, int n_eff, bool raw,
               Plan& out) {
  for (int i = 0; i < n_eff; ++i) {
    int res = NOOP;
    switch (cand[i]) {
      case TCP4: res = P.tcp_gro(i, false); break;
      case TCP6: res = P.tcp_gro(i, true); break;
      case UDP4: res = P.udp_gro(i, false); break;
      case UDP6: res = P.udp_gro(i, true); break;
    }
    if (res == NOOP) out.zero_hdr.push_back(i);  // gro.go:1350-1358
    if (res == NOOP || res == INSERT) out.to_write.push_back(i);
  }
  auto emit = [&](int slot, const Item& it, bool udp, bool raw_item) {
    const Content& c = P.content[slot];
    GroItem gi;
    memset(&gi, 0, sizeof gi);
    gi.out_off = out.out_bytes;
    gi.head_off = (uint32_t)stage_off[c.pieces[0].pkt];
    gi.pkt_len = (uint32_t)(P.lens[slot] - P.offset);
    gi.iph = it.iph;
    gi.l4h = it.l4h;
    gi.gso_size = it.gso_size;
    gi.kind = (uint8_t)((it.key.v6 ? GRO_KIND_V6 : 0) | (udp ? GRO_KIND_UDP : 0) | (c.psh ? GRO_KIND_PSH : 0) |
                        (raw_item ? GRO_KIND_RAW : 0));
    gi.seg_first = (uint32_t)out.segs.size();
    const uint32_t hdr = (uint32_t)it.iph + it.l4h;
    uint64_t dst = out.out_bytes + kVnetLen + hdr;
    for (size_t k = 0; k < c.pieces.size(); ++k) {  // piece 0 = head packet; its header is rebuilt
      Piece pc = c.pieces[k];
      if (k == 0) {
        pc.start += hdr;
        pc.len -= hdr;
      }
      if (pc.len) out.segs.push_back({(uint32_t)(stage_off[pc.pkt] + pc.start), pc.len, (uint32_t)dst, 0u});
      dst += pc.len;
    }
    gi.seg_count = (uint32_t)out.segs.size() - gi.seg_first;
    out.items.push_back(gi);
    out.item_slot.push_back(slot);
    out.out_bytes += (kVnetLen + gi.pkt_len + 15) & ~(uint64_t)15;
  };
  auto apply = [&](std::unordered_map<FlowKey, std::vector<Item>, FlowHash>& table, bool udp) {
    for (auto& kv : table) {
      for (const Item& it : kv.second) {
        const int slot = it.bufs_index;
        const Content& c = P.content[slot];
        if (raw) {
          if (c.pieces.size() > 1 || c.psh) emit(slot, it, udp, true);
        } else if (it.num_merged == 0) {
          out.zero_hdr.push_back(slot);
        } else {
          emit(slot, it, udp, false);
        }
      }
    }
  };
  apply(P.tcp, false);
  apply(P.udp, true);
}

inline void init_planner(Planner& P, uint8_t** bufs, size_t* lens, size_t* caps, int n, int offset,
                  const std::vector<const uint8_t*>& orig, const std::vector<uint8_t>& valid) {
  P.bufs = bufs;
  P.lens = lens;
  P.caps = caps;
  P.n = n;  // packets the loop reaches
  P.offset = offset;
  P.orig = orig;
  P.valid = valid;
  P.consulted.assign(n, 0);
  P.content.assign(n, Content());
  for (int i = 0; i < n; ++i) P.content[i].pieces.push_back({i, 0, (uint32_t)(lens[i] - offset)});
}

}  // namespace gro
}  // namespace wgcs
