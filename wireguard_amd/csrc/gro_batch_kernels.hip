// gro_batch_kernels.hip -- gfx950 device-resident batched handleGRO: many
// Tun.Write calls (/root/reference/tun/tun.go:654-700) whose packets are
// already in HBM, one workgroup per call, everything on the GPU.
//
// handleGRO (gro.go:1326-1367) is order-dependent inside one call (flow
// table, sequence adjacency, prepend swaps) but calls are independent, so the
// batch maps to one 256-thread block per call:
//   1. every thread takes one buffer: slice header, handleGRO's offset check;
//      then one 16-lane DPP row per packet reads the packet once: groCandidate
//      (gro.go:1280-1317), the tcpGRO / udpGRO pre-checks that end in
//      groResultNoop, the header fields the table needs (seq, gsoSize, PSH,
//      the IP fields ipHeadersCanCoalesce compares) from its first 64 bytes,
//      and checksumValid (gro.go:554-612) of every candidate from all of them
//      -- exact up front because the reference validates before it mutates
//      (gro.go:665-681, :709-723, :767-775);
//   2. flow ids: each packet finds the first earlier packet of its table with
//      the same flow key (tcpFlowKey / udpFlowKey, gro.go:96-127, :252-275);
//   3. the loop of handleGRO over those precomputed fields, one thread per
//      flow (flows never interact): tcpGRO / udpGRO with the flow's items as a
//      linked list in LDS, coalesceTCPPackets / coalesceUDPPackets as piece
//      lists (no byte moves yet), the prepend swaps of bufs; toWrite in
//      packet order by a wave ballot;
//   4. every wave applies it in place, one buffer each: the pieces the
//      reference appended behind the buffer's own packet (copied from the
//      original packet bytes), then applyTCPCoalesce / applyUDPCoalesce's
//      header rewrite and virtio header (gro.go:1099-1268); a buffer that a
//      prepend moved out of its item gets the appends it had received; then
//      the slice headers.
// Reads of step 4 never overlap its writes: pieces are read from packet bytes
// below a buffer's original length (never written: only item heads' headers
// and bytes past a buffer's original length are), in the buffer's own region.
#include <hip/hip_runtime.h>

#include "../../include/wgcsum.h"
#include "wgcs_common.h"
#include "wgcs_copy.h"
#include "wgcs_kernels.h"
#include "wgcs_rows.h"

namespace wgcs {

namespace {

constexpr int kMaxB = WGCS_GRO_MAX_CALL;  // buffers per call (one per thread)
constexpr int kNone = -1;
constexpr int kVnet = 10;
constexpr int kCoopMin = 16;  // packets of a flow from which one wave walks it (r4_gro_walk: 16x8 walks 22 -> 4 us)
enum : uint8_t { C_NOT = 0, C_TCP4 = 1, C_TCP6 = 2, C_UDP4 = 3, C_UDP6 = 4 };
enum { R_NOOP = 0, R_INSERT = 1, R_COALESCED = 2 };
enum { CC_PREPEND = -1, CC_UNAV = 0, CC_APPEND = 1 };
enum { CR_INSUFF = 0, CR_PSH = 1, CR_ITEM_BAD = 2, CR_PKT_BAD = 3, CR_OK = 4 };

struct GroSmem {
  uint64_t boff[kMaxB];                 // arena offset of each original buffer
  uint32_t blen[kMaxB], bcap[kMaxB];    // its slice length / capacity
  uint32_t seq[kMaxB], ipattr[kMaxB], keyh[kMaxB], opth[kMaxB];
  union {
    uint32_t kw[kMaxB][10];  // step 2: flow key words (addresses, ports, ack for TCP)
    uint4 rec[kMaxB];        // step 3: the walker's per-packet record (PktRec), one ds_read_b128
  };
  uint32_t slen[kMaxB];                 // len(bufs[s]) of the slice now at position s
  uint32_t it_seq[kMaxB];
  uint32_t m_pos[kMaxB];            // materializations: first byte of the pieces in the buffer
  uint16_t gso[kMaxB], flow[kMaxB], pstart[kMaxB], plen[kMaxB], it_nm[kMaxB], it_gso[kMaxB];
  int16_t pnext[kMaxB], sbuf[kMaxB], shead[kMaxB], stail[kMaxB];
  int16_t it_slot[kMaxB], it_prev[kMaxB], it_next[kMaxB], fl_head[kMaxB], fl_tail[kMaxB];
  int16_t to_write[kMaxB], scount[kMaxB];
  int16_t fnext[kMaxB];                 // next packet of the same flow (kNone: last)
  // materializations (<= n: one per final item or per prepend, each the
  // work of a distinct packet); m_item: -1 = plain
  int16_t m_buf[kMaxB], m_first[kMaxB], m_count[kMaxB], m_item[kMaxB];
  uint8_t m_psh[kMaxB];
  uint8_t cand[kMaxB], noop[kMaxB], iph[kMaxB], th[kMaxB], psh[kMaxB], valid[kMaxB], spsh[kMaxB], szero[kMaxB];
  uint8_t swalk[kMaxB];  // slot s's pieces moved since they were appended (a prepend): finish_item walks them
  uint8_t it_iph[kMaxB], it_l4h[kMaxB], it_psh[kMaxB], it_bad[kMaxB], it_alive[kMaxB], it_cand[kMaxB];
  uint8_t res[kMaxB];                   // groResult of each packet (R_*)
  int16_t ndst[kMaxB];                  // piece p's destination buffer in its final item (-1: none)
  uint32_t npos[kMaxB];                 // ... and its first byte there
  // long TCP flows walked by a whole wave (Planner::run_flow_wave): the flow's
  // packet count, its items as an array (fitem[fbase[f] .. fbase[f] + fnit[f])
  // in insertion order), the list of such flows
  uint8_t hdr[16][80];    // step 1: each row's packet bytes 0..63 (its first five aligned chunks)
  uint32_t fsize[kMaxB];  // packets of the flow
  int16_t fbase[kMaxB], fnit[kMaxB], fitem[kMaxB], coop[kMaxB];
  int n_eff, n_write, n_mat, n_coop, fitem_top;
};

__device__ __forceinline__ uint32_t be16g(const uint8_t* p) { return ((uint32_t)p[0] << 8) | p[1]; }

__device__ __forceinline__ uint32_t fnv(uint32_t h, uint32_t b) { return (h ^ b) * 16777619u; }

// Orders one wave's LDS accesses across its lanes: the wave-cooperative walk
// (run_flow_wave, tcp_gro_wave, append_run) hands LDS state from lane 0 to
// every lane and back.  A wave's LDS operations execute in issue order; this
// keeps the compiler from moving a lane's read above another lane's write to
// a location it cannot prove aliased (a wavefront-scope acquire-release fence
// emits no instruction, the wave barrier pins the schedule).  ADVICE r4.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// ---- the handleGRO loop over the precomputed fields (one thread per flow) ---

struct Planner {
  GroSmem& S;
  const uint8_t* arena;
  int offset;

  __device__ const uint8_t* pkt(int p) const { return arena + S.boff[p] + offset; }
  __device__ int plen_slot(int s) const { return (int)S.slen[s] - offset; }

  __device__ void insert(int bi, int f, uint8_t bad) {  // tcpGROTable.insert / udpGROTable.insert
    const int it = bi;  // an item is named after the packet that inserted it
    init_item(bi, bad);
    S.it_next[it] = kNone;
    S.it_prev[it] = S.fl_tail[f];
    if (S.fl_tail[f] != kNone) S.it_next[S.fl_tail[f]] = (int16_t)it;
    else S.fl_head[f] = (int16_t)it;
    S.fl_tail[f] = (int16_t)it;
  }

  __device__ void init_item(int bi, uint8_t bad) {  // the new item's fields (gro.go:216-225, :358-364)
    const int it = bi;
    S.it_slot[it] = (int16_t)bi;
    S.it_seq[it] = S.seq[bi];
    S.it_nm[it] = 0;
    S.it_gso[it] = S.gso[bi];
    S.it_iph[it] = S.iph[bi];
    S.it_l4h[it] = S.cand[bi] <= C_TCP6 ? S.th[bi] : 8;
    S.it_psh[it] = S.psh[bi];
    S.it_bad[it] = bad;
    S.it_alive[it] = 1;
    S.it_cand[it] = S.cand[bi];
  }

  // A buffer's bytes as the reference leaves them: its own packet (in place)
  // followed by `count` pieces starting at node `first`; item >= 0: also the
  // apply* header rewrite and virtio header of that item.
  __device__ void materialize(int buf, int first, int count, uint32_t pos, uint8_t pshf, int item) {
    const int k = atomicAdd(&S.n_mat, 1);
    S.m_buf[k] = (int16_t)buf;
    S.m_first[k] = (int16_t)first;
    S.m_count[k] = (int16_t)count;
    S.m_pos[k] = pos;
    S.m_psh[k] = pshf;
    S.m_item[k] = (int16_t)item;
  }

  __device__ void unlink(int it, int f) {  // tcpGROTable.deleteAt (gro.go:241-247)
    const int p = S.it_prev[it], n = S.it_next[it];
    if (p != kNone) S.it_next[p] = (int16_t)n;
    else S.fl_head[f] = (int16_t)n;
    if (n != kNone) S.it_prev[n] = (int16_t)p;
    else S.fl_tail[f] = (int16_t)p;
    S.it_alive[it] = 0;
  }

  __device__ bool options_equal(int bi, int tgt, int tgt_iph) const {  // gro.go:442-448
    const int n = S.th[bi] - 20;
    if (S.opth[bi] != S.opth[tgt]) return false;
    const uint8_t* a = pkt(bi) + S.iph[bi] + 20;
    const uint8_t* b = pkt(tgt) + tgt_iph + 20;
    for (int k = 0; k < n; ++k)
      if (a[k] != b[k]) return false;
    return true;
  }

  // tcpPacketsCanCoalesce (gro.go:433-512)
  __device__ int tcp_can(int bi, int it) const {
    const int s = S.it_slot[it];
    const int tgt = S.shead[s];  // the buffer's head packet: its header
    if (S.th[bi] != S.it_l4h[it]) return CC_UNAV;
    if (S.th[bi] > 20 && !options_equal(bi, tgt, S.it_iph[it])) return CC_UNAV;
    if (S.ipattr[bi] != S.ipattr[tgt]) return CC_UNAV;  // ipHeadersCanCoalesce (gro.go:392-427)
    const uint32_t g = S.it_gso[it];
    const uint16_t lhs = (uint16_t)(g + (uint16_t)(g * S.it_nm[it]));
    if (S.seq[bi] == S.it_seq[it] + (uint32_t)lhs) {
      if (S.it_psh[it]) return CC_UNAV;
      if ((plen_slot(s) - (S.iph[bi] + S.th[bi])) % (int)g != 0) return CC_UNAV;
      if (S.gso[bi] > g) return CC_UNAV;
      return CC_APPEND;
    }
    if (S.seq[bi] + S.gso[bi] == S.it_seq[it]) {
      if (S.psh[bi]) return CC_UNAV;
      if (S.gso[bi] < g) return CC_UNAV;
      if (S.gso[bi] > g && S.it_nm[it] > 0) return CC_UNAV;
      return CC_PREPEND;
    }
    return CC_UNAV;
  }

  // coalesceTCPPackets (gro.go:630-741): appends become pieces
  __device__ int tcp_coalesce(int mode, int bi, int it) {
    const int s = S.it_slot[it];
    const int pl = plen_slot(bi);
    const int hdrs = (uint8_t)(S.it_iph[it] + S.it_l4h[it]);
    const int pay = pl - hdrs;
    const int new_len = plen_slot(s) + pay;
    if (mode == CC_PREPEND) {
      if ((int)S.bcap[S.sbuf[bi]] - offset < new_len) return CR_INSUFF;
      if (S.psh[bi]) return CR_PSH;
      if (S.it_nm[it] == 0 && !S.valid[s]) return CR_ITEM_BAD;
      if (!S.valid[bi]) return CR_PKT_BAD;
      S.it_seq[it] = S.seq[bi];
      const int item_pay = new_len - pl;
      const int h0 = S.shead[s];  // the item's head loses its headers (gro.go:690-693)
      // the item's buffer leaves the table holding what the appends wrote into
      // it (and the PSH they set): it keeps those bytes (gro.go:696-697)
      if (S.scount[s] > 1 || S.spsh[s])
        materialize(S.sbuf[s], S.pnext[h0], S.scount[s] - 1, S.plen[h0], S.spsh[s], kNone);
      S.pstart[h0] = (uint16_t)(S.pstart[h0] + hdrs);
      S.plen[h0] = (uint16_t)(S.plen[h0] - hdrs);
      S.pnext[S.stail[bi]] = (int16_t)h0;
      S.stail[bi] = S.stail[s];
      S.slen[bi] += (uint32_t)item_pay;
      S.scount[bi] = (int16_t)(S.scount[bi] + S.scount[s]);
      // bufs[item.bufsIndex], bufs[pktBuffsIndex] = ... (gro.go:696-697)
      int16_t t16;
      uint32_t t32;
      uint8_t t8;
      t16 = S.sbuf[s]; S.sbuf[s] = S.sbuf[bi]; S.sbuf[bi] = t16;
      t32 = S.slen[s]; S.slen[s] = S.slen[bi]; S.slen[bi] = t32;
      t16 = S.shead[s]; S.shead[s] = S.shead[bi]; S.shead[bi] = t16;
      t16 = S.stail[s]; S.stail[s] = S.stail[bi]; S.stail[bi] = t16;
      t8 = S.spsh[s]; S.spsh[s] = S.spsh[bi]; S.spsh[bi] = t8;
      t16 = S.scount[s]; S.scount[s] = S.scount[bi]; S.scount[bi] = t16;
      S.swalk[s] = 1;  // every piece now sits behind the new head
    } else {
      if ((int)S.bcap[S.sbuf[s]] - offset < new_len) return CR_INSUFF;
      if (S.it_nm[it] == 0 && !S.valid[s]) return CR_ITEM_BAD;
      if (!S.valid[bi]) return CR_PKT_BAD;
      if (S.psh[bi]) {  // pktHead[iphLen+13] |= PSH (gro.go:724-729)
        S.it_psh[it] = 1;
        S.spsh[s] = 1;
      }
      S.pstart[bi] = (uint16_t)hdrs;
      S.plen[bi] = (uint16_t)pay;
      S.pnext[bi] = kNone;
      S.ndst[bi] = S.sbuf[s];  // its place in the item's buffer: behind everything before it
      S.npos[bi] = S.slen[s] - (uint32_t)offset;
      S.pnext[S.stail[s]] = (int16_t)bi;
      S.stail[s] = (int16_t)bi;
      S.scount[s]++;
      S.slen[s] += (uint32_t)pay;
    }
    if (S.gso[bi] > S.it_gso[it]) S.it_gso[it] = S.gso[bi];
    S.it_nm[it]++;
    return CR_OK;
  }

  // tcpGRO (gro.go:801-963) after its pre-checks (step 1)
  __device__ int tcp_gro(int bi) {
    const int f = S.flow[bi];
    int it = S.fl_tail[f];
    while (it != kNone) {  // items of the flow, last to first
      const int prev = S.it_prev[it];
      const int can = tcp_can(bi, it);
      if (can != CC_UNAV) {
        const int r = tcp_coalesce(can, bi, it);
        if (r == CR_OK) return R_COALESCED;
        if (r == CR_ITEM_BAD) unlink(it, f);  // deleteAt
        else if (r == CR_PKT_BAD) return R_NOOP;
      }
      it = prev;
    }
    insert(bi, f, 0);
    return R_INSERT;
  }

  // The flow's last item, cached in registers for the in-order append fast
  // path below (it = kNone: nothing cached / no item).
  struct TailCache {
    int it, s, tgt, stail, scount, buf;
    uint32_t l4h, iphit, ipattr, g, nm, seq, psh, slen, cap, valid_s;
    bool dirty;  // running fields newer than LDS
    bool mult;   // the item's payload is a multiple of its gsoSize
  };

  __device__ void load_tail(TailCache& c, int f) const {
    c.dirty = false;
    c.it = S.fl_tail[f];
    if (c.it == kNone) return;
    const int it = c.it;
    c.s = S.it_slot[it];
    c.l4h = S.it_l4h[it];
    c.iphit = S.it_iph[it];
    c.g = S.it_gso[it];
    c.nm = S.it_nm[it];
    c.seq = S.it_seq[it];
    c.psh = S.it_psh[it];
    const int s = c.s;
    c.tgt = S.shead[s];
    c.buf = S.sbuf[s];
    c.slen = S.slen[s];
    c.cap = S.bcap[S.sbuf[s]];
    c.valid_s = S.valid[s] && !S.it_bad[it];  // it_bad: a UDP item inserted after a bad-checksum packet (TCP: 0)
    c.stail = S.stail[s];
    c.scount = S.scount[s];
    c.ipattr = S.ipattr[c.tgt];
    c.mult = c.g != 0 && ((int)c.slen - offset - (int)(uint8_t)(c.iphit + c.l4h)) % (int)c.g == 0;
  }

  // tcpGRO when packet bi appends to the flow's last item -- the in-order
  // bulk case: tcpPacketsCanCoalesce's append branch and coalesceTCPPackets'
  // checks (gro.go:433-512, :709-734) in the reference's order for that item,
  // from registers: the item in `c`, the packet in its record R (PktRec, one
  // LDS read, prefetched by the walker a step ahead).  Returns false whenever
  // any of them fails (or TCP options are present), and the general path
  // (tcp_gro) then decides from LDS exactly as before.  The item's running
  // fields (tail, count, length, numMerged) stay in `c` until flush_tail.
  __device__ bool tcp_append_fast(TailCache& c, int bi, const uint4& R) {
    if (c.it == kNone) return false;
    const uint32_t th = R.w & 0xFFu, iph = (R.w >> 8) & 0xFFu;
    const uint32_t gso = R.z & 0xFFFFu;
    const uint16_t lhs = (uint16_t)(c.g + (uint16_t)(c.g * c.nm));
    // th == l4h and equal IP attributes (version included, so iph == the
    // item's): the appended payload is the packet's gsoSize
    const int plen_s = (int)c.slen - offset;
    const int pay = (int)gso;
    // every check of the append branch at once (no early exits: one lane
    // walks, and each exit would be an exec-mask branch); c.mult is
    // len(pktTarget[iphLen+tcphLen:]) % gsoSize == 0 (gro.go:479-484), kept
    // incrementally instead of a division per packet
    const bool ok = th == c.l4h && th <= 20 && R.y == c.ipattr && R.x == c.seq + (uint32_t)lhs && !c.psh &&
                    c.mult && gso <= c.g && (int)c.cap - offset >= plen_s + pay &&  // coalesceInsufficientCap
                    (c.nm != 0 || c.valid_s) &&                                      // coalesceItemInvalidCSum
                    ((R.w >> 24) & 1u);                                              // coalescePktInvalidCSum
    if (!ok) return false;
    (void)iph;
    if ((R.w >> 16) & 1u) {  // pktHead[iphLen+13] |= PSH (gro.go:724-729)
      S.it_psh[c.it] = 1;
      S.spsh[c.s] = 1;
      c.psh = 1;
    }
    S.pstart[bi] = (uint16_t)(c.iphit + c.l4h);
    S.plen[bi] = (uint16_t)pay;  // S.pnext[bi] is kNone since step 1
    S.ndst[bi] = (int16_t)c.buf;
    S.npos[bi] = c.slen - (uint32_t)offset;
    S.pnext[c.stail] = (int16_t)bi;
    c.stail = bi;
    ++c.scount;
    c.slen += (uint32_t)pay;
    ++c.nm;
    c.mult = pay == (int)c.g;  // a multiple before, so a multiple after iff this payload is gsoSize
    c.dirty = true;
    return true;
  }

  // the item's running fields back into LDS (before the general path reads them)
  __device__ void flush_tail(TailCache& c) {
    if (!c.dirty) return;
    S.stail[c.s] = (int16_t)c.stail;
    S.scount[c.s] = (int16_t)c.scount;
    S.slen[c.s] = c.slen;
    S.it_nm[c.it] = (uint16_t)c.nm;
    c.dirty = false;
  }

  // udpGRO (gro.go:971-1095) after its pre-checks
  __device__ int udp_gro(int bi) {
    const int f = S.flow[bi];
    const int it = S.fl_tail[f];
    if (it == kNone) {
      insert(bi, f, 0);
      return R_INSERT;
    }
    const int s = S.it_slot[it];
    const int tgt = S.shead[s];
    const int tl = plen_slot(s);
    uint8_t bad = 0;
    // udpPacketsCanCoalesce (gro.go:519-544)
    if (S.ipattr[bi] == S.ipattr[tgt] && (tl - (S.iph[bi] + 8)) % (int)S.it_gso[it] == 0 && S.gso[bi] <= S.it_gso[it]) {
      // coalesceUDPPackets (gro.go:745-783)
      const int hdrs = (uint8_t)(S.it_iph[it] + 8);
      const int pay = plen_slot(bi) - hdrs;
      if ((int)S.bcap[S.sbuf[s]] - offset < tl + pay) {
      } else if (S.it_nm[it] == 0 && (S.it_bad[it] || !S.valid[s])) {
      } else if (!S.valid[bi]) {
        bad = 1;
      } else {
        S.pstart[bi] = (uint16_t)hdrs;
        S.plen[bi] = (uint16_t)pay;
        S.pnext[bi] = kNone;
        S.ndst[bi] = S.sbuf[s];
        S.npos[bi] = S.slen[s] - (uint32_t)offset;
        S.pnext[S.stail[s]] = (int16_t)bi;
        S.stail[s] = (int16_t)bi;
        S.scount[s]++;
        S.slen[s] += (uint32_t)pay;
        S.it_nm[it]++;
        return R_COALESCED;
      }
    }
    insert(bi, f, bad);
    return R_INSERT;
  }

  // The loop of handleGRO (gro.go:1334-1363) restricted to the packets of
  // one flow (first packet f).  Flows never interact: a packet only meets the
  // items of its own flow key, and the buffers it swaps or appends into are
  // its own flow's, so every flow of a call runs on its own thread.
  __device__ void run_flow(int f) {
    const bool tcp = S.cand[f] <= C_TCP6;
    if (!tcp) {
      for (int i = f; i != kNone; i = S.fnext[i]) S.res[i] = (uint8_t)udp_gro(i);
      return;
    }
    TailCache c;
    c.it = kNone;
    c.dirty = false;
    bool fresh = false;  // c mirrors the flow's last item
    uint4 R = S.rec[f];
    for (int i = f; i != kNone;) {  // the flow's packets in order (fnext links)
      const int nx = (int)(int16_t)(R.z >> 16);
      const uint4 Rn = nx != kNone ? S.rec[nx] : R;  // the next record, a step ahead
      if (!fresh) {
        load_tail(c, f);
        fresh = true;
      }
      if (tcp_append_fast(c, i, R)) {
        S.res[i] = R_COALESCED;
      } else {
        flush_tail(c);
        S.res[i] = (uint8_t)tcp_gro(i);
        fresh = false;  // inserts, prepends, deletes: reload from LDS
      }
      i = nx;
      R = Rn;
    }
    flush_tail(c);
  }

  // tcpGRO's item loop for packet bi against the items of flow f, one lane per
  // item (lane k: the k-th item from the last, gro.go:903-951): every lane
  // evaluates tcpPacketsCanCoalesce and coalesceTCPPackets' checks for its
  // item from the state before this packet, without side effects, so the
  // loop's outcome is decided at once: the first item (from the last) whose
  // coalesce would succeed or find the packet's checksum invalid ends it; the
  // items before it whose own checksum is invalid are deleted (deleteAt, the
  // loop goes on past them); no such item: the packet is inserted.  Then lane 0
  // applies the outcome.  Returns the groResult.
  enum { W_SKIP = 0, W_DEL = 1, W_STOP = 2, W_OK = 3 };
  // tail_app: 1 when bi appended to the flow's last item, 0 when not, -1 when
  // not known here (the one-lane loop)
  __device__ int tcp_gro_wave(int bi, int f, int lane, int& tail_app) {
    tail_app = -1;
    const int base = S.fbase[f];
    int nit = S.fnit[f];
    int result = R_INSERT, mode = CC_UNAV, it_ok = kNone;
    if (nit > 64 || nit <= 2) {  // wave-uniform: more items than lanes, or too few to share -- lane 0 runs the loop
      if (lane == 0) {
        for (int p = nit - 1; p >= 0; --p) {
          const int it = S.fitem[base + p];
          const int can = tcp_can(bi, it);
          if (can == CC_UNAV) continue;
          const int r = tcp_coalesce(can, bi, it);
          if (r == CR_OK) {
            result = R_COALESCED;
            break;
          }
          if (r == CR_ITEM_BAD) {  // deleteAt: the items after it close up
            S.it_alive[it] = 0;
            for (int q = p; q + 1 < nit; ++q) S.fitem[base + q] = S.fitem[base + q + 1];
            --nit;
          } else if (r == CR_PKT_BAD) {
            result = R_NOOP;
            break;
          }
        }
        if (result == R_INSERT) {
          init_item(bi, 0);
          S.fitem[base + nit] = (int16_t)bi;
          ++nit;
        }
        S.fnit[f] = (int16_t)nit;
        S.fl_tail[f] = nit ? S.fitem[base + nit - 1] : (int16_t)kNone;
      }
      wave_lds_sync();
      return __builtin_amdgcn_readfirstlane(result);
    }
    {  // nit <= 64: one lane per item
      const int k = lane;
      int code = W_SKIP, can = CC_UNAV, it = kNone;
      const uint4 R = S.rec[bi];  // the packet: {seq, ipattr, gsoSize, th | iph | PSH | valid}
      const uint32_t pth = R.w & 0xFFu;
      if (k < nit) {
        // tcp_can and coalesceTCPPackets' checks without early exits, so
        // each lane issues its item's LDS reads together (three dependent
        // levels: item, slot, head packet / buffer), not one round trip per check
        it = S.fitem[base + nit - 1 - k];
        const int s = S.it_slot[it];
        const uint32_t l4h = S.it_l4h[it], g = S.it_gso[it], nm = S.it_nm[it], iseq = S.it_seq[it];
        const bool ipsh = S.it_psh[it] != 0;
        const int hdrs = (uint8_t)(S.it_iph[it] + l4h);
        const int tgt = S.shead[s];
        const int plen_s = plen_slot(s);
        const bool vs = S.valid[s] != 0;
        const uint32_t tattr = S.ipattr[tgt];
        const int cap_s = (int)S.bcap[S.sbuf[s]] - offset;
        const int pl_b = plen_slot(bi), cap_b = (int)S.bcap[S.sbuf[bi]] - offset;  // the packet's own slot
        const uint32_t pseq = R.x, pgso = R.z & 0xFFFFu, piph = (R.w >> 8) & 0xFFu;
        const bool ppsh = (R.w >> 16) & 1u, pvalid = (R.w >> 24) & 1u;
        // tcpPacketsCanCoalesce (gro.go:433-512), as tcp_can
        const uint16_t lhs = (uint16_t)(g + (uint16_t)(g * nm));
        const bool app = pseq == iseq + (uint32_t)lhs;
        const bool app_ok = !ipsh && (plen_s - (int)(piph + pth)) % (int)g == 0 && pgso <= g;
        const bool pre_ok = pseq + pgso == iseq && !ppsh && pgso >= g && !(pgso > g && nm > 0);
        can = (pth != l4h || R.y != tattr) ? CC_UNAV : app ? (app_ok ? CC_APPEND : CC_UNAV) : pre_ok ? CC_PREPEND : CC_UNAV;
        if (pth > 20 && can != CC_UNAV && !options_equal(bi, tgt, S.it_iph[it])) can = CC_UNAV;  // TCP options (gro.go:442-448)
        const int new_len = plen_s + pl_b - hdrs;
        const int cap = can == CC_PREPEND ? cap_b : cap_s;
        code = can == CC_UNAV                                       ? W_SKIP
               : (cap < new_len || (can == CC_PREPEND && ppsh))     ? W_SKIP   // coalesceInsufficientCap / PSHEnding
               : (nm == 0 && !vs)                                   ? W_DEL    // coalesceItemInvalidChecksum
               : !pvalid                                            ? W_STOP   // coalescePktInvalidChecksum
                                                                    : W_OK;
      }
      const uint64_t dec = __ballot(code >= W_STOP);
      const uint64_t del = __ballot(code == W_DEL) & (dec ? ((1ull << __builtin_ctzll(dec)) - 1ull) : ~0ull);
      if (del) {  // deleteAt: the surviving items close up, in order (every lane moves its own)
        if (k < nit && !((del >> lane) & 1ull)) {
          const int p = nit - 1 - k;  // position from the first item
          // deleted items below position p are those of higher lanes
          const int np = p - (int)__builtin_popcountll(lane < 63 ? del >> (lane + 1) : 0ull);
          S.fitem[base + np] = (int16_t)it;
        }
        if ((del >> lane) & 1ull) S.it_alive[it] = 0;
        wave_lds_sync();  // the compaction, before lane 0 reads fitem below
      }
      if (dec) {
        const int d = __builtin_ctzll(dec);
        const int cd = __shfl(code, d);
        mode = __shfl(can, d);
        it_ok = __shfl(it, d);
        result = cd == W_OK ? R_COALESCED : R_NOOP;
        // the items after it (lanes below d) are all deleted: it is the last one now
        tail_app = result == R_COALESCED && mode == CC_APPEND && d == (int)__builtin_popcountll(del);
      } else {
        tail_app = 0;
      }
      nit -= (int)__builtin_popcountll(del);
    }
    if (lane == 0) {
      if (result == R_COALESCED) {
        tcp_coalesce(mode, bi, it_ok);  // its checks pass: decided above from the same state
      } else if (result == R_INSERT) {
        init_item(bi, 0);
        S.fitem[base + nit] = (int16_t)bi;
        ++nit;
      }
      S.fnit[f] = (int16_t)nit;
      S.fl_tail[f] = nit ? S.fitem[base + nit - 1] : (int16_t)kNone;
    }
    wave_lds_sync();  // lane 0's coalesce / insert, before any lane reads the flow again
    return result;
  }

  // tcp_append_fast (udp: udp_gro's append) for a whole wave: the flow's
  // packets from bi on, 64 packet indices at a time (lane k: packet w + k, a
  // member of the flow when its flow id is f -- a flow's packets are in index
  // order).  Every member evaluates the append checks against the item as it
  // would be after each earlier member of the run had appended: numMerged
  // grows by one per member, and since a member only appends when the one
  // before it left a multiple of gsoSize (without PSH), every earlier
  // member's payload was gsoSize.  So the first member whose checks fail is
  // exactly the packet at which the one-lane walk stops appending, and every
  // member before it appends -- all at once, each lane linking its own piece.
  // Returns that packet (kNone: the flow's remaining packets all appended).
  // c is wave-uniform.  For UDP that packet then starts a new item, bad (in
  // ubad) when only its own checksum kept it from appending (gro.go:1062-1075).
  template <bool udp>
  __device__ int append_run(TailCache& c, int f, int bi, int n_eff, int lane, int& ubad) {
    ubad = 0;
    if (c.it == kNone) return bi;
    for (int w = bi; w < n_eff; w += 64) {  // wave-uniform
      const int q = w + lane;
      const bool mem = q < n_eff && S.cand[q] != C_NOT && !S.noop[q] && S.flow[q] == f;
      const uint64_t M = __ballot(mem);
      if (!M) continue;
      const uint64_t Mb = M & ((1ull << lane) - 1ull);
      const int rank = __builtin_popcountll(Mb);
      const int prev = Mb ? 63 - __builtin_clzll(Mb) : lane;  // the member before (lane: none in this window)
      uint4 R = make_uint4(0, 0, 0, 0);
      if (mem) R = S.rec[q];
      const uint32_t gso = R.z & 0xFFFFu, pshb = (R.w >> 16) & 1u, th = R.w & 0xFFu;
      const uint32_t gso_prev = (uint32_t)__shfl((int)gso, prev), psh_prev = (uint32_t)__shfl((int)pshb, prev);
      const bool first = Mb == 0;
      const uint32_t nm = c.nm + (uint32_t)rank;
      const uint32_t slen = c.slen + (uint32_t)rank * c.g;
      const uint16_t lhs = (uint16_t)(c.g + (uint16_t)(c.g * nm));
      const bool psh = first ? c.psh != 0 : psh_prev != 0;
      const bool mult = first ? c.mult : gso_prev == c.g;
      // TCP: tcpPacketsCanCoalesce's append branch + coalesceTCPPackets
      // (gro.go:433-512, :709-734); UDP: udpPacketsCanCoalesce +
      // coalesceUDPPackets (gro.go:519-544, :745-783).  Either way the
      // appended payload is the packet's gsoSize (same IP attributes, so the
      // same header lengths).
      const bool l4_ok = udp || (th == c.l4h && th <= 20 && R.x == c.seq + (uint32_t)lhs && !psh);
      const bool fits = l4_ok && R.y == c.ipattr && mult && gso <= c.g &&
                        (int)c.cap - offset >= ((int)slen - offset) + (int)gso && (nm != 0 || c.valid_s);
      const bool ok = fits && ((R.w >> 24) & 1u);
      const uint64_t fail = __ballot(mem && !ok);
      const uint64_t A = fail ? M & ((1ull << __builtin_ctzll(fail)) - 1ull) : M;
      if ((A >> lane) & 1ull) {
        S.pstart[q] = (uint16_t)(c.iphit + c.l4h);
        S.plen[q] = (uint16_t)gso;  // S.pnext[q] is kNone since step 1
        S.ndst[q] = (int16_t)c.buf;
        S.npos[q] = slen - (uint32_t)offset;
        S.pnext[first ? c.stail : w + prev] = (int16_t)q;
        S.res[q] = R_COALESCED;
      }
      wave_lds_sync();  // every member's piece links
      if (A) {  // the item after the run (only its last member may carry PSH or a short payload)
        const int L = 63 - __builtin_clzll(A);
        const int cnt = __builtin_popcountll(A);
        const uint32_t gl = (uint32_t)__builtin_amdgcn_readlane((int)gso, L), pl = (uint32_t)__builtin_amdgcn_readlane((int)pshb, L);
        c.stail = w + L;
        c.scount += cnt;
        c.slen += (uint32_t)(cnt - 1) * c.g + gl;
        c.nm += (uint32_t)cnt;
        c.mult = gl == c.g;
        c.dirty = true;
        if (pl) {  // pktHead[iphLen+13] |= PSH (gro.go:724-729)
          if (lane == 0) {
            S.it_psh[c.it] = 1;
            S.spsh[c.s] = 1;
          }
          c.psh = 1;
        }
      }
      if (fail) {
        const int F = __builtin_ctzll(fail);
        ubad = __builtin_amdgcn_readlane((int)fits, F);
        return w + F;
      }
    }
    return kNone;
  }

  // run_flow for a long flow, by a whole wave (f wave-uniform): runs of
  // in-order appends go through append_run; a packet that leaves it goes
  // through tcp_gro_wave (one lane per item) or, for UDP (which only ever
  // meets the flow's last item), udp_gro on lane 0.
  template <bool udp>
  __device__ void run_flow_wave(int f, int n_eff, int lane) {
    TailCache c;
    c.it = kNone;
    c.dirty = false;
    bool try_fast = true;
    int ubad = 0;
    for (int i = f; i != kNone;) {  // wave-uniform
      if (try_fast) {
        load_tail(c, f);
        i = append_run<udp>(c, f, i, n_eff, lane, ubad);
        if (lane == 0) flush_tail(c);  // the item loop below reads the item from LDS
        wave_lds_sync();
        c.dirty = false;
        if (i == kNone) break;
      }
      int res = R_INSERT;
      if constexpr (udp) {  // udpGRO's outcome for a packet that does not append: a new item (the flow's last)
        if (lane == 0) insert(i, f, (uint8_t)ubad);
        wave_lds_sync();
      } else {
        // in a reordered flow the in-order fast path is tried again only after
        // the item loop appended to the flow's last item
        int tail_app;
        res = tcp_gro_wave(i, f, lane, tail_app);
        try_fast = tail_app >= 0 ? tail_app != 0
                                 : res == R_COALESCED && S.fl_tail[f] != kNone && S.stail[S.it_slot[S.fl_tail[f]]] == i;
      }
      if (lane == 0) S.res[i] = (uint8_t)res;
      wave_lds_sync();
      i = S.fnext[i];
    }
  }

  // apply{TCP,UDP}Coalesce (gro.go:1364-1366) for item `it`, or -- after
  // "invalid offset" -- nothing: its buffer keeps what the coalescing wrote
  __device__ void finish_item(int it, bool raw) {
    const int s = S.it_slot[it];
    const int h = S.shead[s];
    const bool changed = S.scount[s] > 1 || S.spsh[s];
    if (raw ? !changed : S.it_nm[it] == 0) {
      if (!raw) S.szero[s] = 1;  // numMerged == 0: empty virtioNetHdr (:1168-1174, :1250-1256)
      return;
    }
    // the item's pieces go behind its head packet: one row each (step 4).
    // Every append placed its piece already (ndst / npos); only after a
    // prepend, which puts a new head before them all, are they placed again
    if (S.swalk[s]) {
      uint32_t pos = S.plen[h];
      for (int p = S.pnext[h]; p != kNone; p = S.pnext[p]) {
        S.ndst[p] = S.sbuf[s];
        S.npos[p] = pos;
        pos += S.plen[p];
      }
    }
    materialize(S.sbuf[s], kNone, 0, 0, S.spsh[s], raw ? kNone : it);
  }
};

// checksumValid (gro.go:554-612) of packet p on one 16-lane row (lane r):
// pkt[iphLen:] summed in aligned 16-byte chunks, plus the pseudo header.
__device__ bool row_checksum_valid(const uint8_t* pk, int pl, int iphl, bool v6, uint32_t proto, int r) {
  constexpr int U = 6;  // 16-byte chunks per lane in flight: a 1536-byte packet in one batch
  const uint8_t* lo = pk + iphl;
  const uint8_t* hi = pk + pl;
  const uint8_t* a0 = reinterpret_cast<const uint8_t*>((uintptr_t)lo & ~(uintptr_t)15);
  const int nch = (int)((hi - a0 + 15) >> 4);
  const int x00 = (int)(a0 - lo);  // position of chunk 0 relative to the L4 start
  uint64_t acc = 0;
  for (int c0 = 0; c0 < nch; c0 += 16 * U) {  // row-uniform
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int c = c0 + r + 16 * u;
      v[u] = c < nch ? ld16(a0 + 16 * c) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc += chunk_sum(v[u], x00 + 16 * (c0 + r + 16 * u), 0, pl - iphl);
  }
  uint32_t s = fold32_16(row16_sum_u32(fold64_16(acc)));
  if (((uintptr_t)lo & 1u) == 0) s = bswap16(s);  // LE pairs at even addresses -> BE words from lo
  // pseudo header: addresses (BE words), protocol, L4 length (gro.go:561-571)
  const int a_lo = v6 ? 8 : 12, nw = v6 ? 16 : 4;
  const uint32_t aw = r < nw ? be16g(pk + a_lo + 2 * r) : 0u;
  const uint32_t ad = row16_sum_u32(aw);
  const uint32_t t = fold32_16(s + fold32_16(ad) + proto + (uint32_t)((pl - iphl) & 0xFFFF));
  return t == 0xFFFFu;
}

// n bytes src -> dst on one 16-lane row (lane r), any alignments: destination
// chunk k (16-byte aligned) = bytes [sb, sb + 16) of the dword-aligned source
// window k and the first dword of window k + 1 (the next lane's, DPP row_ror);
// all windows of a 1536-byte piece in flight at once.
__device__ void row_copy(const uint8_t* src, int n, uint8_t* dst, int r) {
  constexpr int U = 6;
  const int dalign = (int)((uintptr_t)dst & 15u);
  uint8_t* dbase = dst - dalign;
  const int nk = (n + dalign + 15) >> 4;
  const uint8_t* w0 = src - dalign;  // source of destination chunk 0's first byte
  const int sb = (int)((uintptr_t)w0 & 3u);
  const uint8_t* abase = w0 - sb;
  const uint8_t* src_hi = src + n;
  const uint4 z = make_uint4(0, 0, 0, 0);
  for (int k0 = 0; k0 < nk; k0 += 16 * U) {  // row-uniform
    uint4 A[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint8_t* ca = abase + 16 * (k0 + r + 16 * u);
      A[u] = (ca < src_hi && ca + 16 > src) ? ld_window<false>(ca, src_hi) : z;
    }
    uint32_t E = 0;
    if (r == 15) {
      const uint8_t* ce = abase + 16 * (k0 + 16 * U);
      if (ce < src_hi) E = *reinterpret_cast<const uint32_t*>(__builtin_assume_aligned(ce, 4));
    }
    uint32_t Rc = row_next(A[0].x);
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
        store_chunk(dbase + 16 * k, v, 16 * k - dalign, n);
      }
    }
  }
}

// Header byte x of an applied item before the two computed checksums
// (applyTCPCoalesce / applyUDPCoalesce, gro.go:1099-1268).
__device__ __forceinline__ uint32_t patched(uint32_t b, int x, int iphl, int csum_at, uint32_t pkt_len, bool v6,
                                            bool udp, bool pshf) {
  if (!v6) {
    if (x == 2) b = (pkt_len >> 8) & 0xFF;  // total length, uint16(len(pkt)) (:1131 / :1214)
    if (x == 3) b = pkt_len & 0xFF;
    if (x == 10 || x == 11) b = 0;  // :1134 / :1217
  } else {
    const uint32_t pl = pkt_len - (uint32_t)iphl;  // payload length (:1124-1127 / :1207-1210)
    if (x == 4) b = (pl >> 8) & 0xFF;
    if (x == 5) b = pl & 0xFF;
  }
  if (udp) {
    const uint32_t ul = pkt_len - (uint32_t)iphl;  // UDP length (:1229-1232)
    if (x == iphl + 4) b = (ul >> 8) & 0xFF;
    if (x == iphl + 5) b = ul & 0xFF;
  } else if (pshf && x == iphl + 13) {
    b |= 0x08;  // PSH of an appended packet (gro.go:724-729)
  }
  if (x == csum_at || x == csum_at + 1) b = 0;
  return b;
}

}  // namespace

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(7, 8))) void gro_batch_kernel(uint8_t* __restrict__ arena, wgcs_gro_buf* __restrict__ bufs,
                                                        const wgcs_gro_call* __restrict__ calls,
                                                        int32_t* __restrict__ status, int32_t* __restrict__ n_write,
                                                        int32_t* __restrict__ to_write) {
  __shared__ GroSmem S;
#ifdef WGCS_GRO_STAMPS  // timing-only build (scripts/probe_gro_phases.py): s_memrealtime at each phase boundary
  uint64_t stp[6];
  stp[0] = __builtin_amdgcn_s_memrealtime();
#endif
  const int t = threadIdx.x;
  const int lane = t & 63, wv = t >> 6, r = lane & 15, row = t >> 4;
  const wgcs_gro_call call = calls[blockIdx.x];
  const int n = (int)call.n, offset = call.offset;
  const bool can_udp = (call.flags & WGCS_GRO_CAN_UDP) != 0;
  if (n > kMaxB || offset < 0) {  // block-uniform
    if (t == 0) {
      status[blockIdx.x] = WGCS_ERR_INVALID_ARG;
      n_write[blockIdx.x] = 0;
    }
    return;
  }
  wgcs_gro_buf* cb = bufs + call.first;

  // ---- 1. slice headers, handleGRO's offset check (gro.go:1335-1337)
  if (t == 0) {
    S.n_eff = n;
    S.n_mat = 0;
    S.n_coop = 0;
    S.fitem_top = 0;
  }
  __syncthreads();
  if (t < n) {
    const wgcs_gro_buf b = cb[t];
    S.boff[t] = b.off;
    S.blen[t] = b.len;
    S.bcap[t] = b.cap;
    if (offset < kVnet || (int64_t)offset > (int64_t)b.len - 1) atomicMin(&S.n_eff, t);
  }
  __syncthreads();
  const int n_eff = S.n_eff;
  if (t < n) {
    S.sbuf[t] = (int16_t)t;
    S.slen[t] = S.blen[t];
    S.shead[t] = S.stail[t] = (int16_t)t;
    S.scount[t] = 1;
    S.pnext[t] = kNone;
    S.pstart[t] = 0;
    S.plen[t] = (uint16_t)(t < n_eff ? S.blen[t] - offset : 0);
    S.spsh[t] = 0;
    S.swalk[t] = 0;
    S.szero[t] = 0;
    S.fl_head[t] = S.fl_tail[t] = kNone;
    S.cand[t] = C_NOT;
    S.noop[t] = 1;
    S.valid[t] = 0;
    S.res[t] = R_NOOP;
    S.it_alive[t] = 0;
    S.ndst[t] = kNone;
    S.fsize[t] = 0;
  }
  // groCandidate + the tcpGRO / udpGRO checks that return groResultNoop, and
  // checksumValid of every candidate, in one pass over each packet (round
  // 5): one 16-lane row per packet loads its aligned 16-byte chunks once (6
  // per lane in flight, 1,536 bytes); the header fields come from the first
  // five chunks (packet bytes 0..63, fetched across the row), the L4 checksum
  // (gro.go:554-612) from all of them.  Until round 4 a thread per packet read
  // the header with its own five loads and a row read the packet again after
  // the flow ids: the packet's first 128-byte line came from HBM twice.
  __syncthreads();  // the slot state above, before the rows write packet fields
  for (int p = row; p < n_eff; p += 16) {  // row-uniform
    constexpr int U = 6;
    const uint8_t* pk = arena + S.boff[p] + offset;
    const int pl = (int)(S.blen[p] - (uint32_t)offset);
    const uint8_t* a0 = reinterpret_cast<const uint8_t*>((uintptr_t)pk & ~(uintptr_t)15);
    const int sh = (int)((uintptr_t)pk & 15u);
    const int nch = (pl + sh + 15) >> 4;
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int c = r + 16 * u;
      v[u] = c < nch ? ld16(a0 + 16 * c) : make_uint4(0, 0, 0, 0);
    }
    // packet bytes 0..63: chunks 0..4 (the row's lanes 0..4) staged in the
    // row's LDS slot, read back byte by byte (broadcast reads; registers
    // holding them would spill at this kernel's 72-VGPR budget)
    wave_lds_sync();  // the row's reads of its previous packet's bytes come first
    if (r < 5) *reinterpret_cast<uint4*>(&S.hdr[row][16 * r]) = v[0];
    wave_lds_sync();
    const uint8_t* hb = &S.hdr[row][sh];
    // byte k (< 64) of the packet; every byte the checks below read lies
    // below len(pkt) (each read is behind its length check), and every such
    // byte is in a loaded chunk
    auto B = [&](int k) -> uint32_t { return hb[k]; };
    auto BE16 = [&](int k) -> uint32_t { return (B(k) << 8) | B(k + 1); };
    auto BE32 = [&](int k) -> uint32_t { return (BE16(k) << 16) | BE16(k + 2); };
    // checksumValid's sum first, so the chunks die before the header checks:
    // pkt[iphLen:] with iphLen from the version nibble (every candidate's; a
    // packet that is none never uses it), chunk c at L4 position 16 c - sh -
    // iphLen, more batches for a packet past 1,536 bytes
    const int ihv = (B(0) >> 4) == 6 ? 40 : 20;
    uint64_t acc = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) acc += chunk_sum(v[u], 16 * (r + 16 * u) - sh - ihv, 0, pl - ihv);
    uint8_t c = C_NOT;
    if (pl >= 28) {  // gro.go:1280-1317
      const uint32_t b0 = B(0), ver = b0 >> 4;
      if (ver == 4 && (b0 & 0x0F) == 5) {
        const uint32_t pr = B(9);
        if (pr == 6 && pl >= 40) c = C_TCP4;
        else if (pr == 17 && can_udp) c = C_UDP4;
      } else if (ver == 6) {
        const uint32_t nh = B(6);
        if (nh == 6 && pl >= 60) c = C_TCP6;
        else if (nh == 17 && pl >= 48 && can_udp) c = C_UDP6;
      }
    }
    if (r == 0) S.cand[p] = c;
    if (c != C_NOT) {  // row-uniform
      const bool v6 = c == C_TCP6 || c == C_UDP6, tcp = c <= C_TCP6;
      const int ih = v6 ? 40 : 20;  // IPv4 candidates have IHL 5
      bool nop = pl > 65535;
      if (v6) nop = nop || BE16(4) != (uint32_t)(pl - 40);
      else nop = nop || BE16(2) != (uint32_t)pl;
      int thl = 8;
      uint32_t fl = 0;
      if (tcp) {
        nop = nop || pl < ih;
        thl = (int)((v6 ? B(52) : B(32)) >> 4) * 4;
        nop = nop || thl < 20 || thl > 60 || pl < ih + thl;
      } else {
        nop = nop || pl < ih + 8;
      }
      if (!v6) nop = nop || (B(6) & 0x20) || (uint8_t)(B(6) << 3) || B(7);  // fragments
      if (!nop && tcp) {
        fl = v6 ? B(53) : B(33);
        nop = fl != 0x10 && fl != 0x18;  // ACK, or ACK|PSH
      }
      const int g = nop ? 0 : pl - ih - thl;
      nop = nop || g < 1;
      if (r == 0) {
        S.noop[p] = nop ? 1 : 0;
        S.iph[p] = (uint8_t)ih;
        S.th[p] = (uint8_t)thl;
        S.psh[p] = (fl & 0x08) ? 1 : 0;
        S.gso[p] = (uint16_t)g;
      }
      if (!nop) {  // row-uniform
        if (r == 0) {
          S.seq[p] = tcp ? (v6 ? BE32(44) : BE32(24)) : 0u;
          S.ipattr[p] = v6 ? B(0) | ((B(1) >> 4) << 8) | (B(7) << 16) | (6u << 24)
                           : B(1) | ((B(6) >> 5) << 8) | (B(8) << 16) | (4u << 24);
          // flow key words (addresses, ports, ack for TCP) into LDS + their hash
          uint32_t h = 2166136261u;
          if (v6) {
#pragma unroll
            for (int w = 0; w < 8; ++w) {
              const uint32_t x = BE32(8 + 4 * w);
              S.kw[p][w] = x;
              h = fnv(h, x);
            }
          } else {
#pragma unroll
            for (int w = 0; w < 2; ++w) {
              const uint32_t x = BE32(12 + 4 * w);
              S.kw[p][w] = x;
              h = fnv(h, x);
            }
          }
          const int nab = v6 ? 32 : 8;
          const uint32_t ports = v6 ? BE32(40) : BE32(20);
          const uint32_t ack = tcp ? (v6 ? BE32(48) : BE32(28)) : 0u;
          S.kw[p][nab / 4] = ports;
          S.kw[p][nab / 4 + 1] = ack;
          S.keyh[p] = fnv(fnv(fnv(h, ports), ack), c);
          uint32_t oh = 2166136261u;
          if (tcp)
            for (int k = 20; k < thl; ++k) oh = fnv(oh, pk[ih + k]);
          S.opth[p] = oh;
        }
        // checksumValid's fold (ih == ihv for every candidate)
        uint32_t sm = fold32_16(row16_sum_u32(fold64_16(acc)));
        if (((uintptr_t)(pk + ih) & 1u) == 0) sm = bswap16(sm);  // LE pairs at even addresses -> BE words from L4
        // pseudo header: addresses (BE words), protocol, L4 length (gro.go:561-571);
        // lane r's word at packet byte 8 + 2r (IPv6: 16 words from 8; IPv4: lanes 2..5, bytes 12..19)
        const int ka = 8 + 2 * r;
        const bool in_a = v6 ? r < 16 : (r >= 2 && r < 6);
        const uint32_t aw = in_a ? ((uint32_t)hb[ka] << 8) | hb[ka + 1] : 0u;
        const uint32_t ad = row16_sum_u32(aw);
        const uint32_t tt = fold32_16(sm + fold32_16(ad) + (tcp ? 6u : 17u) + (uint32_t)((pl - ih) & 0xFFFF));
        // a packet past 1,536 bytes (not an MTU-sized Write) is summed
        // whole after the flow ids (row_checksum_valid: a second batch in
        // this loop would cost the kernel ~40 spilled VGPRs); 2 = pending
        if (r == 0) S.valid[p] = nch > 16 * U ? 2 : (tt == 0xFFFFu ? 1 : 0);
      }
    }
  }
  __syncthreads();

#ifdef WGCS_GRO_STAMPS
  stp[1] = __builtin_amdgcn_s_memrealtime();
#endif
  // ---- 2. flow ids (first earlier packet with the same key in the same table)
  if (t < n_eff && S.cand[t] != C_NOT && !S.noop[t]) {
    const uint8_t c = S.cand[t];
    const bool v6 = c == C_TCP6 || c == C_UDP6;
    const int nkw = v6 ? 10 : 4;  // key words: the class fixes the layout (ack is 0 for UDP)
    const uint32_t kh = S.keyh[t];
    int f = t;
    for (int q = 0; q < t; ++q) {
      if (S.keyh[q] != kh || S.cand[q] != c || S.noop[q]) continue;
      bool eq = true;
      for (int w = 0; w < nkw; ++w) eq = eq && S.kw[q][w] == S.kw[t][w];
      if (eq) {
        f = q;
        break;
      }
    }
    S.flow[t] = (uint16_t)f;
    atomicAdd(&S.fsize[f], 1u);
    // and the next later packet of the same flow, so the flow's thread walks
    // only its own packets (each thread searches for its own link in parallel)
    int nx = kNone;
    for (int q = t + 1; q < n_eff; ++q) {
      if (S.keyh[q] != kh || S.cand[q] != c || S.noop[q]) continue;
      bool eq = true;
      for (int w = 0; w < nkw; ++w) eq = eq && S.kw[q][w] == S.kw[t][w];
      if (eq) {
        nx = q;
        break;
      }
    }
    S.fnext[t] = (int16_t)nx;
  }
  // checksumValid of the candidates past 1,536 bytes (step 1 left them pending)
  for (int p = row; p < n_eff; p += 16) {  // row-uniform
    if (S.valid[p] != 2) continue;
    const uint8_t c = S.cand[p];
    const bool v6 = c == C_TCP6 || c == C_UDP6;
    const bool ok = row_checksum_valid(arena + S.boff[p] + offset, (int)(S.blen[p] - offset), S.iph[p], v6,
                                       c <= C_TCP6 ? 6u : 17u, r);
    wave_lds_sync();  // every lane of the row has read S.valid[p]
    if (r == 0) S.valid[p] = ok ? 1 : 0;
  }
  __syncthreads();

#ifdef WGCS_GRO_STAMPS
  stp[2] = __builtin_amdgcn_s_memrealtime();
#endif
  // ---- 3. the handleGRO loop: one thread per flow.  First each packet's
  // PktRec -- {seq, ipattr, gsoSize | fnext << 16, th | iph << 8 | psh << 16 |
  // valid << 24} -- over the dead key words, so the walker fetches a packet
  // with one LDS read and prefetches the next one while it decides this one.
  uint4 rec = make_uint4(0, 0, 0, 0);
  const bool live = t < n_eff && S.cand[t] != C_NOT && !S.noop[t];
  if (live)
    rec = make_uint4(S.seq[t], S.ipattr[t], (uint32_t)S.gso[t] | ((uint32_t)(uint16_t)S.fnext[t] << 16),
                     (uint32_t)S.th[t] | ((uint32_t)S.iph[t] << 8) | ((uint32_t)S.psh[t] << 16) |
                         ((uint32_t)S.valid[t] << 24));
  if (live) S.rec[t] = rec;  // step 2's key-word reads ended at the barrier above
  // a flow of kCoopMin or more packets is walked by a whole wave (its
  // in-order runs 64 packets at a time, a TCP flow's item loop one lane per
  // item, run_flow_wave); the others by one thread
  const bool leader = live && S.flow[t] == t;
  const bool coop = leader && S.fsize[t] >= (uint32_t)kCoopMin;
  if (coop) {
    S.coop[atomicAdd(&S.n_coop, 1)] = (int16_t)t;
    S.fbase[t] = (int16_t)atomicAdd(&S.fitem_top, (int)S.fsize[t]);  // room for one item per packet
    S.fnit[t] = 0;
  }
  __syncthreads();
  const bool raw = n_eff < n;  // "invalid offset": coalescing happened, apply* did not
  Planner P{S, arena, offset};
  if (leader && !coop) P.run_flow(t);
  for (int k = wv; k < S.n_coop; k += 4) {  // wave-uniform
    const int f = S.coop[k];
    if (S.cand[f] >= C_UDP4) P.run_flow_wave<true>(f, n_eff, lane);
    else P.run_flow_wave<false>(f, n_eff, lane);
  }
  __syncthreads();
#ifdef WGCS_GRO_STAMPS
  stp[3] = __builtin_amdgcn_s_memrealtime();
#endif
  // toWrite in packet order (groResultNoop and groResultTableInsert,
  // gro.go:1349-1362); NOOP buffers get an empty virtioNetHdr (:1350-1358)
  if (wv == 0) {
    int base = 0;
    for (int c0 = 0; c0 < n_eff; c0 += 64) {  // wave-uniform
      const int p = c0 + lane;
      const bool w = p < n_eff && S.res[p] != R_COALESCED;
      const uint64_t m = __ballot(w);
      if (w) S.to_write[base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0))] = (int16_t)p;
      base += __popcll(m);
    }
    if (lane == 0) S.n_write = raw ? 0 : base;
  }
  if (t < n_eff && S.res[t] == R_NOOP) S.szero[t] = 1;
  if (t < n_eff && S.it_alive[t]) P.finish_item(t, raw);
  __syncthreads();

#ifdef WGCS_GRO_STAMPS
  stp[4] = __builtin_amdgcn_s_memrealtime();
#endif
  // ---- 4. apply in place
  // slice headers after the prepend swaps; toWrite; status
  if (t < n) {
    const int b = S.sbuf[t];
    wgcs_gro_buf o;
    o.off = S.boff[b];
    o.len = S.slen[t];
    o.cap = S.bcap[b];
    cb[t] = o;
  }
  const int nw = S.n_write;
  if (t < nw) to_write[call.first + t] = S.to_write[t];
  if (t == 0) {
    status[blockIdx.x] = raw ? WGCS_ERR_INVALID_OFFSET : 0;
    n_write[blockIdx.x] = nw;
  }
  // empty virtio headers (NOOP buffers; unapplied items unless "invalid offset")
  if (t < n && S.szero[t]) {
    uint8_t* vh = arena + S.boff[S.sbuf[t]] + offset - kVnet;
    for (int k = 0; k < kVnet; ++k) vh[k] = 0;
  }
  // materializations: one wave each -- the pieces appended behind the
  // buffer's own packet (coalesce*Packets' appends, from the original packet
  // bytes), then the item's apply* header rewrite + virtio header, or just the
  // PSH the appends set
  // final items' pieces: one 16-lane row per piece
  for (int p = row; p < n_eff; p += 16) {  // row-uniform
    const int d = S.ndst[p];
    if (d == kNone) continue;
    row_copy(arena + S.boff[p] + offset + S.pstart[p], (int)S.plen[p], arena + S.boff[d] + offset + S.npos[p], r);
  }
  const int nm = S.n_mat;
  for (int k = wv; k < nm; k += 4) {  // wave-uniform
    const int buf = S.m_buf[k];
    uint8_t* head = arena + S.boff[buf] + offset;
    uint32_t pos = S.m_pos[k];
    int p = S.m_first[k];
    for (int q = 0; q < S.m_count[k]; ++q) {  // a buffer a prepend moved out: its appends, in order
      copy_range(arena + S.boff[p] + offset + S.pstart[p], (int)S.plen[p], head + pos, lane);
      pos += S.plen[p];
      p = S.pnext[p];
    }
    const int it = S.m_item[k];
    if (it < 0) {  // never applied: only the PSH that appends OR'ed in (gro.go:724-729)
      if (lane == 0 && S.m_psh[k] && S.cand[buf] <= C_TCP6) head[S.iph[buf] + 13] |= 0x08;
      continue;
    }
    const int s = S.it_slot[it];
    const int ih = S.it_iph[it], hl = ih + S.it_l4h[it];
    const uint8_t c = S.it_cand[it];
    const bool v6 = c == C_TCP6 || c == C_UDP6, udp = c >= C_UDP4;
    const bool pshf = S.m_psh[k] != 0;
    const uint32_t pkt_len = S.slen[s] - (uint32_t)offset;
    const int csum_at = ih + (udp ? 6 : 16);
    const int x0 = 2 * lane;  // BE word x0 of the header, read before any write
    uint32_t b0 = 0, b1 = 0;
    if (x0 < hl) b0 = patched(head[x0], x0, ih, csum_at, pkt_len, v6, udp, pshf);
    if (x0 + 1 < hl) b1 = patched(head[x0 + 1], x0 + 1, ih, csum_at, pkt_len, v6, udp, pshf);
    const uint32_t w = (b0 << 8) | b1;
    const int a_lo = v6 ? 8 : 12, a_hi = v6 ? 40 : 20;
    const uint32_t ipc = (~fold32_16(wave_sum_u32(!v6 && x0 < ih ? w : 0u))) & 0xFFFFu;
    // checksum([]byte{}, pseudoHeaderChecksumNoFold(src, dst, proto, len-iph)), not complemented
    const uint32_t pcs = fold32_16(fold32_16(wave_sum_u32(x0 >= a_lo && x0 < a_hi ? w : 0u)) + (udp ? 17u : 6u) +
                                   ((pkt_len - (uint32_t)ih) & 0xFFFFu));
    if (!v6 && x0 == 10) {
      b0 = ipc >> 8;
      b1 = ipc & 0xFF;
    }
    if (x0 == csum_at) {
      b0 = pcs >> 8;
      b1 = pcs & 0xFF;
    }
    if (x0 < hl) head[x0] = (uint8_t)b0;
    if (x0 + 1 < hl) head[x0 + 1] = (uint8_t)b1;
    // virtio_net_hdr (gro.go:1107-1117 / :1191-1201), native byte order
    if (lane < kVnet) {
      const uint32_t gso_type = udp ? 5u : (v6 ? 4u : 1u);
      const uint32_t f[5] = {(uint32_t)hl, S.it_gso[it], (uint32_t)ih, udp ? 6u : 16u, 0u};
      uint32_t vb;
      if (lane == 0) vb = 1;  // VIRTIO_NET_HDR_F_NEEDS_CSUM
      else if (lane == 1) vb = gso_type;
      else vb = (f[(lane - 2) >> 1] >> (8 * (lane & 1))) & 0xFF;
      head[lane - kVnet] = (uint8_t)vb;
    }
  }
#ifdef WGCS_GRO_STAMPS  // to_write[first + 100 .. 106) of 128-buffer calls with < 100 writes (the bench's shapes)
  __syncthreads();
  stp[5] = __builtin_amdgcn_s_memrealtime();
  if (t == 0 && n == kMaxB && S.n_write < 100)
    for (int k = 0; k < 6; ++k) to_write[call.first + 100 + k] = (int32_t)(uint32_t)stp[k];
#endif
}

// ---- write stager (wstager.cpp): staged packets -> slices, toWrite images -> packed output
//
// One wave per staged packet: the aligned 16-byte chunks that hold its
// virtio header and packet, from the packed stage (or, for zero-copy pushes,
// straight from pinned host memory over PCIe) into its slice, which has the
// same phase mod 16.
__global__ __launch_bounds__(256) void ws_scatter_kernel(const uint8_t* __restrict__ stage,
                                                         uint8_t* __restrict__ arena, const WsMove* __restrict__ mv,
                                                         uint32_t n) {
  const uint32_t w = blockIdx.x * 4u + (threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63u;
  if (w >= n) return;  // wave-uniform
  const WsMove m = mv[w];
  const uint4* s = (m.flags & WS_MOVE_ABS) ? reinterpret_cast<const uint4*>((uintptr_t)m.src)
                                           : reinterpret_cast<const uint4*>(stage + m.src);
  uint4* d = reinterpret_cast<uint4*>(arena + m.dst);
  uint32_t k = lane;
  for (; k + 64 < m.n16; k += 128) {  // two chunks per lane in flight
    const uint4 a = s[k], b = s[k + 64];
    d[k] = a;
    d[k + 64] = b;
  }
  if (k < m.n16) d[k] = s[k];
}

// One block per call: Tun.Write's write(2) images, bufs[i][offset-10:len] for
// i in toWrite (tun.go:687-698), packed in toWrite order into the call's
// output region as the aligned 16-byte chunks that hold them (so source and
// destination share their phase mod 16); wlen / wpos[first + k] = the image's
// length and its first byte in the region.  An image set larger than the
// region (not possible: each packet's bytes end up in at most one written
// buffer, and the host reserves 32 + align16(len) bytes per packet) would be
// reported as WGCS_ERR_OUT_OF_RANGE, never written past it.
__global__ __launch_bounds__(256) void ws_gather_kernel(const uint8_t* __restrict__ arena,
                                                        const wgcs_gro_buf* __restrict__ bufs,
                                                        const wgcs_gro_call* __restrict__ calls,
                                                        const WsOut* __restrict__ outs, int32_t* __restrict__ status,
                                                        const int32_t* __restrict__ n_write,
                                                        const int32_t* __restrict__ to_write,
                                                        int32_t* __restrict__ wlen, int32_t* __restrict__ wpos,
                                                        uint8_t* __restrict__ out) {
  __shared__ uint32_t pos[kMaxB + 1];
  __shared__ uint32_t lead[kMaxB];
  __shared__ uint64_t src[kMaxB];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const wgcs_gro_call call = calls[blockIdx.x];
  const WsOut o = outs[blockIdx.x];
  const int st = status[blockIdx.x];
  int nw = st == 0 ? n_write[blockIdx.x] : 0;
  nw = nw < 0 ? 0 : (nw > kMaxB ? kMaxB : nw);
  if (t < nw) {
    const int i = to_write[call.first + t];
    const wgcs_gro_buf b = bufs[call.first + i];
    const uint64_t img = b.off + (uint64_t)call.offset - kVnet;  // bufs[i][offset-10]
    const uint64_t c0 = img & ~(uint64_t)15, c1 = (b.off + b.len + 15) & ~(uint64_t)15;
    wlen[call.first + t] = (int32_t)(b.len - (uint32_t)call.offset + kVnet);
    lead[t] = (uint32_t)(img - c0);
    pos[t + 1] = (uint32_t)(c1 - c0);
    src[t] = c0;
  }
  __syncthreads();
  if (t == 0) {
    pos[0] = 0;
    for (int k = 1; k <= nw; ++k) pos[k] += pos[k - 1];
    if (pos[nw] > o.room) status[blockIdx.x] = WGCS_ERR_OUT_OF_RANGE;
  }
  __syncthreads();
  if (pos[nw] > o.room) return;  // block-uniform
  if (t < nw) wpos[call.first + t] = (int32_t)(pos[t] + lead[t]);
  for (int k = wv; k < nw; k += 4) {  // wave-uniform: one image per wave
    const uint4* s = reinterpret_cast<const uint4*>(arena + src[k]);
    uint4* d = reinterpret_cast<uint4*>(out + o.base + pos[k]);
    const uint32_t n16 = (pos[k + 1] - pos[k]) >> 4;
    uint32_t c = (uint32_t)lane;
    for (; c + 64 < n16; c += 128) {
      const uint4 a = s[c], b = s[c + 64];
      d[c] = a;
      d[c + 64] = b;
    }
    if (c < n16) d[c] = s[c];
  }
}

hipError_t launch_ws_scatter(const uint8_t* stage, uint8_t* arena, const WsMove* mv, uint32_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(ws_scatter_kernel, dim3((n + 3) / 4), dim3(256), 0, s, stage, arena, mv, n);
  return hipGetLastError();
}

hipError_t launch_ws_gather(const uint8_t* arena, const wgcs_gro_buf* bufs, const wgcs_gro_call* calls,
                            const WsOut* outs, uint32_t n_calls, int32_t* status, const int32_t* n_write,
                            const int32_t* to_write, int32_t* wlen, int32_t* wpos, uint8_t* out, hipStream_t s) {
  if (n_calls == 0) return hipSuccess;
  hipLaunchKernelGGL(ws_gather_kernel, dim3(n_calls), dim3(256), 0, s, arena, bufs, calls, outs, status, n_write,
                     to_write, wlen, wpos, out);
  return hipGetLastError();
}

hipError_t launch_gro_batch(uint8_t* arena, wgcs_gro_buf* bufs, const wgcs_gro_call* calls, uint32_t n_calls,
                            int32_t* status, int32_t* n_write, int32_t* to_write, hipStream_t s) {
  if (n_calls == 0) return hipSuccess;
  hipLaunchKernelGGL(gro_batch_kernel, dim3(n_calls), dim3(256), 0, s, arena, bufs, calls, status, n_write, to_write);
  return hipGetLastError();
}

}  // namespace wgcs
