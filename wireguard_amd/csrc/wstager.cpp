// wstager.cpp -- Tun.Write batch staging.
//
// The reference handles one Write call at a time: handleGRO over <= 128
// packets (tun/tun.go:654-700 -> gro.go:1326-1367), then one write(2) per
// toWrite entry of bufs[i][offset-10:] (tun.go:687-698); it is called from
// every peer's RoutineSendToInternet (device/receive.go:483-498).  One such
// call is far too small for a GPU round trip (wgcs_handle_gro: ~70 us), so the
// write stager aggregates many Write batches into one pinned ring slot:
//
//   push      stage one Write call's packets (pinned), plan its flows on the
//             host assuming every checksum is valid (wgcs_gro_plan.h)
//   submit    slot stream: H2D of all staged packets + candidate descriptors
//             -> ONE VALIDATE launch over every candidate of every batch
//             -> ONE coalesce launch over every merged item of every batch
//             -> D2H of the validity bits and the super-packets
//   wait      settle each batch: a batch whose plan consulted a checksum that
//             is invalid is re-planned with the real bits and its items rebuilt
//             (one more small round trip, that batch only)
//   result    per batch, what Tun.Write hands to write(2): for each toWrite
//             index the bytes bufs[i][offset-10:len(bufs[i])] after handleGRO,
//             in pinned memory (a 10-byte virtio header + packet)
//
// `depth` slots rotate, each with its own stream: slot k's D2H overlaps slot
// k+1's kernels and slot k+2's H2D.  The caller's buffers are only read by
// push; handleGRO's in-place edits of bufs are not replayed into them (Write's
// callers recycle bufs after the call, device/receive.go:500-505).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/wgcsum.h"
#include "wgcs_ctx.h"
#include "wgcs_gro_plan.h"
#include "wgcs_kernels.h"

using namespace wgcs;
using namespace wgcs::gro;

namespace {

constexpr size_t kHead = 16;  // headroom before each staged packet: its virtio header bytes go there

inline size_t al16(size_t x) { return (x + 15) & ~(size_t)15; }

struct WBatch {  // one Tun.Write call
  int n = 0, offset = 0, can_udp = 0;
  int status = 0;                  // 0 or WGCS_ERR_INVALID_OFFSET (gro.go:1335-1337)
  int n_eff = 0;                   // packets the handleGRO loop reaches
  std::vector<uint64_t> stage;     // staged packet offsets (packet k's bytes at h_stage + stage[k])
  std::vector<size_t> lens0, caps0;
  std::vector<int> cand;
  std::vector<uint32_t> vidx;      // candidate k -> index into the slot's validity array
  std::vector<uint8_t> consulted;  // validity bits the plan depended on
  Plan plan;
  std::vector<int> order;          // order[i] = original buffer now at position i
  std::vector<size_t> lens;        // final len(bufs[i])
  bool fixup = false;              // items rebuilt by the settle pass (outputs in the fixup region)
};

struct WSlot {
  uint64_t id = 0;
  int state = 0;  // 0 free, 1 open, 2 submitted, 3 settled
  std::vector<WBatch> batches;
  size_t used = 0;       // staged bytes
  uint64_t out_used = 0; // coalesce output bytes
  uint32_t ncand = 0;
  std::vector<GroItem> items;
  std::vector<GroSeg> segs;
  // pinned host
  uint8_t* h_stage = nullptr;
  wgcs_pkt* h_pkts = nullptr;
  uint8_t* h_valid = nullptr;
  uint8_t* h_meta = nullptr;  // items | segs (H2D)
  uint8_t* h_out = nullptr;
  uint8_t* h_fix = nullptr;   // settle pass: rebuilt items' outputs
  size_t fix_cap = 0;
  // device
  uint8_t* d_stage = nullptr;
  wgcs_pkt* d_pkts = nullptr;
  uint8_t* d_valid = nullptr;
  uint8_t* d_meta = nullptr;
  uint8_t* d_out = nullptr;
  uint8_t* d_fix = nullptr;
  hipStream_t stream = nullptr;
  hipEvent_t done = nullptr;
};

}  // namespace

struct wgcs_wstager {
  wgcs_ctx* ctx = nullptr;
  uint32_t depth = 0, max_writes = 0, max_pkts = 0;
  size_t max_bytes = 0, max_out = 0, max_meta = 0;
  std::vector<WSlot> slots;
  uint32_t open = 0;
  uint64_t next_id = 1;
  std::mutex mu;
  WSlot* find(uint64_t id) {
    for (auto& s : slots)
      if (s.id == id && id != 0) return &s;
    return nullptr;
  }
};

namespace {

void free_wslot(WSlot& s) {
  for (void* p : {(void*)s.h_stage, (void*)s.h_pkts, (void*)s.h_valid, (void*)s.h_meta, (void*)s.h_out, (void*)s.h_fix})
    if (p) hipHostFree(p);
  for (void* p : {(void*)s.d_stage, (void*)s.d_pkts, (void*)s.d_valid, (void*)s.d_meta, (void*)s.d_out, (void*)s.d_fix})
    if (p) hipFree(p);
  if (s.done) hipEventDestroy(s.done);
  if (s.stream) hipStreamDestroy(s.stream);
  s = WSlot();
}

int open_wslot(wgcs_wstager* ws, uint32_t idx) {
  WSlot& s = ws->slots[idx];
  if (s.state == 2) {
    hipError_t e = hipEventSynchronize(s.done);
    if (e != hipSuccess) return hip_fail(ws->ctx, e, "wstager: wait for ring slot");
  }
  s.id = ws->next_id++;
  s.state = 1;
  s.batches.clear();
  s.used = 0;
  s.out_used = 0;
  s.ncand = 0;
  s.items.clear();
  s.segs.clear();
  ws->open = idx;
  return WGCS_OK;
}

// Plan batch b of slot s with the validity bits `valid` (per packet of the
// batch): handleGRO's loop + apply, as a gather plan whose items write into
// the output region at `out_base`.
void plan_batch(WSlot& s, WBatch& b, const std::vector<uint8_t>& valid, uint64_t out_base) {
  const int n = b.n;
  std::vector<uint8_t*> ptrs(n);  // tokens: follow the prepend swaps (gro.go:696-697)
  for (int i = 0; i < n; ++i) ptrs[i] = reinterpret_cast<uint8_t*>((uintptr_t)(i + 1));
  b.lens = b.lens0;
  std::vector<size_t> caps = b.caps0;
  std::vector<const uint8_t*> orig(n, nullptr);
  // orig[i] = the packet bytes (bufs[i][offset:]): staged at h_stage + stage[i]
  for (int i = 0; i < b.n_eff; ++i) orig[i] = s.h_stage + b.stage[i];
  Planner P;
  init_planner(P, ptrs.data(), b.lens.data(), caps.data(), b.n_eff, b.offset, orig, valid);
  b.plan = Plan();
  b.plan.out_bytes = out_base;
  make_plan(P, b.cand, b.stage, b.n_eff, b.status != 0, b.plan);
  b.consulted = P.consulted;
  b.order.resize(n);
  for (int i = 0; i < n; ++i) b.order[i] = (int)((uintptr_t)ptrs[i] - 1);
}

// GroItem/GroSeg offsets are relative to the staged packets (head_off /
// src_off are stage offsets; the packet's own bytes start at stage[k]).
void add_plan_items(WSlot& s, WBatch& b) {
  const uint32_t seg0 = (uint32_t)s.segs.size();
  for (GroItem it : b.plan.items) {
    it.seg_first += seg0;
    s.items.push_back(it);
  }
  s.segs.insert(s.segs.end(), b.plan.segs.begin(), b.plan.segs.end());
}

}  // namespace

extern "C" {

int wgcs_wstager_create(wgcs_ctx* ctx, uint32_t depth, uint32_t max_writes, uint32_t max_pkts, size_t max_bytes,
                        wgcs_wstager** out) {
  if (!ctx || !out || depth < 2 || depth > 64 || max_writes == 0 || max_pkts == 0 || max_bytes == 0)
    return WGCS_ERR_INVALID_ARG;
  if (max_bytes > 0xF0000000ull) return set_err(ctx, WGCS_ERR_INVALID_ARG, "wstager: max_bytes >= 4 GB");
  *out = nullptr;
  auto* ws = new (std::nothrow) wgcs_wstager();
  if (!ws) return WGCS_ERR_NOMEM;
  ws->ctx = ctx;
  ws->depth = depth;
  ws->max_writes = max_writes;
  ws->max_pkts = max_pkts;
  ws->max_bytes = al16(max_bytes + (size_t)max_pkts * (kHead + 16));
  // coalesced outputs never exceed the staged packets + one virtio header and alignment per packet
  ws->max_out = al16(max_bytes + (size_t)max_pkts * 32);
  ws->max_meta = (size_t)max_pkts * (sizeof(GroItem) + sizeof(GroSeg)) + 64;
  ws->slots.resize(depth);
  hipSetDevice(ctx->device);
  for (auto& s : ws->slots) {
    hipError_t e = hipSuccess;
    if (e == hipSuccess) e = hipHostMalloc((void**)&s.h_stage, ws->max_bytes + 64, hipHostMallocDefault);
    if (e == hipSuccess) e = hipHostMalloc((void**)&s.h_pkts, max_pkts * sizeof(wgcs_pkt), hipHostMallocDefault);
    if (e == hipSuccess) e = hipHostMalloc((void**)&s.h_valid, max_pkts + 64, hipHostMallocDefault);
    if (e == hipSuccess) e = hipHostMalloc((void**)&s.h_meta, ws->max_meta, hipHostMallocDefault);
    if (e == hipSuccess) e = hipHostMalloc((void**)&s.h_out, ws->max_out + 64, hipHostMallocDefault);
    if (e == hipSuccess) e = hipMalloc((void**)&s.d_stage, ws->max_bytes + 64);
    if (e == hipSuccess) e = hipMalloc((void**)&s.d_pkts, max_pkts * sizeof(wgcs_pkt));
    if (e == hipSuccess) e = hipMalloc((void**)&s.d_valid, max_pkts + 64);
    if (e == hipSuccess) e = hipMalloc((void**)&s.d_meta, ws->max_meta);
    if (e == hipSuccess) e = hipMalloc((void**)&s.d_out, ws->max_out + 64);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&s.done, hipEventDisableTiming);
    if (e != hipSuccess) {
      const int rc = hip_fail(ctx, e, "wstager allocation");
      for (auto& t : ws->slots) free_wslot(t);
      delete ws;
      return rc;
    }
  }
  const int rc = open_wslot(ws, 0);
  if (rc) {
    for (auto& t : ws->slots) free_wslot(t);
    delete ws;
    return rc;
  }
  *out = ws;
  return WGCS_OK;
}

int wgcs_wstager_destroy(wgcs_wstager* ws) {
  if (!ws) return WGCS_ERR_INVALID_ARG;
  hipSetDevice(ws->ctx->device);
  for (auto& s : ws->slots) {
    if (s.state == 2) hipEventSynchronize(s.done);
    free_wslot(s);
  }
  delete ws;
  return WGCS_OK;
}

// Stage one Tun.Write(bufs, offset) call: bufs[i] is a Go slice, its packet at
// bufs[i][offset:lens[i]], cap(bufs[i]) = caps[i] (device/receive.go:483).
int wgcs_wstager_push(wgcs_wstager* ws, const uint8_t* const* bufs, const size_t* lens, const size_t* caps, int n,
                      int offset, int can_udp_gro, int* write_idx) {
  if (!ws || !write_idx || n < 0 || (n > 0 && (!bufs || !lens || !caps))) return WGCS_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(ws->mu);
  WSlot& s = ws->slots[ws->open];
  // handleGRO's loop stops at the first buffer with an invalid offset (gro.go:1335-1337)
  int n_eff = n;
  for (int i = 0; i < n; ++i)
    if (offset < kVnetLen || (long)offset > (long)lens[i] - 1) {
      n_eff = i;
      break;
    }
  if (n_eff < n) {  // Tun.Write returns (0, err) and writes nothing (tun.go:667-676): no staging needed
    if (s.batches.size() >= ws->max_writes)
      return set_err(ws->ctx, WGCS_ERR_BATCH_FULL, "wstager: open batch is full");
    WBatch b;
    b.n = n;
    b.offset = offset;
    b.status = WGCS_ERR_INVALID_OFFSET;
    *write_idx = (int)s.batches.size();
    s.batches.push_back(std::move(b));
    return WGCS_OK;
  }
  size_t need = 0;
  uint32_t npk = 0;
  for (int i = 0; i < n_eff; ++i) {
    if (lens[i] - (size_t)offset > 65535 + 64) return set_err(ws->ctx, WGCS_ERR_INVALID_ARG, "wstager: packet > 64 KiB");
    need += kHead + al16(lens[i] - offset);
  }
  uint32_t npk_total = 0;
  for (const auto& b : s.batches) npk_total += (uint32_t)b.n_eff;
  npk = (uint32_t)n_eff;
  if (s.batches.size() >= ws->max_writes || npk_total + npk > ws->max_pkts || s.used + need > ws->max_bytes)
    return set_err(ws->ctx, WGCS_ERR_BATCH_FULL, "wstager: open batch is full");
  WBatch b;
  b.n = n;
  b.offset = offset;
  b.can_udp = can_udp_gro != 0;
  b.n_eff = n_eff;
  b.status = n_eff < n ? WGCS_ERR_INVALID_OFFSET : 0;
  b.stage.assign(n, 0);
  b.lens0.assign(lens, lens + n);
  b.caps0.assign(caps, caps + n);
  b.cand.assign(n, NOT_CAND);
  std::vector<uint8_t> assume(n, 0);
  for (int i = 0; i < n_eff; ++i) {
    const size_t pl = lens[i] - (size_t)offset;
    const uint64_t at = s.used + kHead;
    // headroom: the caller's bytes bufs[i][offset-10:offset].  A buffer whose
    // table item was dropped (tcpGRO's deleteAt after coalesceItemInvalidChecksum,
    // gro.go:942-945) is written with them, as no virtio header is ever encoded
    // into it; NOOP and unmerged items get a zero header at settle (wait).
    memset(s.h_stage + s.used, 0, kHead - kVnetLen);
    memcpy(s.h_stage + at - kVnetLen, bufs[i] + offset - kVnetLen, kVnetLen);
    memcpy(s.h_stage + at, bufs[i] + offset, pl);
    b.stage[i] = at;
    s.used = at + al16(pl);
    b.cand[i] = gro_candidate(s.h_stage + at, pl, b.can_udp);
    if (b.cand[i] != NOT_CAND) {
      const bool v6 = b.cand[i] == TCP6 || b.cand[i] == UDP6;
      const bool udp = b.cand[i] == UDP4 || b.cand[i] == UDP6;
      wgcs_pkt_set(&s.h_pkts[s.ncand], at, (uint32_t)pl, (uint16_t)(v6 ? 40 : 20), 0, (uint8_t)(udp ? 17 : 6),
                   (uint8_t)(v6 ? WGCS_PKT_V6 : 0));
      b.vidx.push_back(s.ncand++);
      assume[i] = 1;  // speculation: valid (checked at settle)
    } else {
      b.vidx.push_back(0xFFFFFFFFu);
    }
  }
  plan_batch(s, b, assume, s.out_used);
  s.out_used = b.plan.out_bytes;
  add_plan_items(s, b);
  *write_idx = (int)s.batches.size();
  s.batches.push_back(std::move(b));
  return WGCS_OK;
}

int wgcs_wstager_submit(wgcs_wstager* ws, uint64_t* batch) {
  if (!ws || !batch) return WGCS_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(ws->mu);
  hipSetDevice(ws->ctx->device);
  WSlot& s = ws->slots[ws->open];
  const hipStream_t q = s.stream;
  hipError_t e = hipSuccess;
  const size_t ib = s.items.size() * sizeof(GroItem), sb = s.segs.size() * sizeof(GroSeg);
  if (ib + sb > ws->max_meta || s.out_used > ws->max_out)
    return set_err(ws->ctx, WGCS_ERR_INVALID_ARG, "wstager: plan larger than the slot");
  if (s.used) e = hipMemcpyAsync(s.d_stage, s.h_stage, s.used, hipMemcpyHostToDevice, q);
  if (e == hipSuccess && s.ncand) {
    e = hipMemcpyAsync(s.d_pkts, s.h_pkts, s.ncand * sizeof(wgcs_pkt), hipMemcpyHostToDevice, q);
    if (e == hipSuccess)
      e = launch_checksum_batch(WGCS_MODE_VALIDATE, 0, s.d_stage, s.d_pkts, nullptr, s.ncand, s.d_valid, q,
                                ws->ctx->num_cu, ws->ctx->tune);
    if (e == hipSuccess) e = hipMemcpyAsync(s.h_valid, s.d_valid, s.ncand, hipMemcpyDeviceToHost, q);
  }
  if (e == hipSuccess && !s.items.empty()) {
    memcpy(s.h_meta, s.items.data(), ib);
    memcpy(s.h_meta + ib, s.segs.data(), sb);
    e = hipMemcpyAsync(s.d_meta, s.h_meta, ib + sb, hipMemcpyHostToDevice, q);
    if (e == hipSuccess)
      e = launch_gro_coalesce(s.d_stage, (const GroItem*)s.d_meta, (uint32_t)s.items.size(),
                              (const GroSeg*)(s.d_meta + ib), (uint32_t)s.segs.size(), s.d_out, q);
    if (e == hipSuccess) e = hipMemcpyAsync(s.h_out, s.d_out, s.out_used, hipMemcpyDeviceToHost, q);
  }
  if (e == hipSuccess) e = hipEventRecord(s.done, q);
  if (e != hipSuccess) return hip_fail(ws->ctx, e, "wstager submit");
  s.state = 2;
  *batch = s.id;
  return open_wslot(ws, (ws->open + 1) % ws->depth);
}

// Wait for a submitted slot and settle it: batches whose plan consulted a
// checksum that the VALIDATE kernel found invalid are re-planned with the real
// bits; their rebuilt items go through the coalesce kernel once more.
int wgcs_wstager_wait(wgcs_wstager* ws, uint64_t batch) {
  if (!ws) return WGCS_ERR_INVALID_ARG;
  hipEvent_t ev;
  {
    std::lock_guard<std::mutex> g(ws->mu);
    WSlot* s = ws->find(batch);
    if (!s || s->state == 1) return WGCS_ERR_NOT_READY;
    if (s->state == 3) return WGCS_OK;
    ev = s->done;
  }
  hipError_t e = hipEventSynchronize(ev);
  if (e != hipSuccess) return hip_fail(ws->ctx, e, "wstager wait");
  std::lock_guard<std::mutex> g(ws->mu);
  WSlot* s = ws->find(batch);
  if (!s) return WGCS_ERR_NOT_READY;
  if (s->state == 3) return WGCS_OK;
  std::vector<GroItem> fix_items;
  std::vector<GroSeg> fix_segs;
  uint64_t fix_out = 0;
  for (WBatch& b : s->batches) {
    if (b.status) continue;
    bool redo = false;
    std::vector<uint8_t> real(b.n, 0);
    for (int i = 0; i < b.n_eff; ++i) {
      if (b.vidx[i] == 0xFFFFFFFFu) continue;
      real[i] = s->h_valid[b.vidx[i]];
      redo = redo || (b.consulted[i] && !real[i]);
    }
    if (!redo) continue;
    plan_batch(*s, b, real, fix_out);
    fix_out = b.plan.out_bytes;
    const uint32_t seg0 = (uint32_t)fix_segs.size();
    for (GroItem it : b.plan.items) {
      it.seg_first += seg0;
      fix_items.push_back(it);
    }
    fix_segs.insert(fix_segs.end(), b.plan.segs.begin(), b.plan.segs.end());
    b.fixup = true;
  }
  if (!fix_items.empty()) {
    hipSetDevice(ws->ctx->device);
    const size_t ib = fix_items.size() * sizeof(GroItem), sb = fix_segs.size() * sizeof(GroSeg);
    if (ib + sb > ws->max_meta) return set_err(ws->ctx, WGCS_ERR_INVALID_ARG, "wstager: re-plan too large");
    if (fix_out + 16 > s->fix_cap) {
      if (s->h_fix) hipHostFree(s->h_fix);
      if (s->d_fix) hipFree(s->d_fix);
      s->h_fix = nullptr;
      s->d_fix = nullptr;
      s->fix_cap = 0;
      const size_t want = al16(fix_out + fix_out / 4 + 4096);
      e = hipHostMalloc((void**)&s->h_fix, want, hipHostMallocDefault);
      if (e == hipSuccess) e = hipMalloc((void**)&s->d_fix, want);
      if (e != hipSuccess) return hip_fail(ws->ctx, e, "wstager: fixup region");
      s->fix_cap = want;
    }
    memcpy(s->h_meta, fix_items.data(), ib);
    memcpy(s->h_meta + ib, fix_segs.data(), sb);
    e = hipMemcpyAsync(s->d_meta, s->h_meta, ib + sb, hipMemcpyHostToDevice, s->stream);
    if (e == hipSuccess)
      e = launch_gro_coalesce(s->d_stage, (const GroItem*)s->d_meta, (uint32_t)fix_items.size(),
                              (const GroSeg*)(s->d_meta + ib), (uint32_t)fix_segs.size(), s->d_fix, s->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(s->h_fix, s->d_fix, fix_out, hipMemcpyDeviceToHost, s->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
    if (e != hipSuccess) return hip_fail(ws->ctx, e, "wstager re-plan");
  }
  // the zero virtio header of NOOP buffers (gro.go:1350-1356) and of unmerged
  // items (applyTCPCoalesce / applyUDPCoalesce, gro.go:1168-1174), into the
  // staged headroom of the buffer now at that slot (H2D is long done)
  for (const WBatch& b : s->batches) {
    if (b.status) continue;
    for (int slot : b.plan.zero_hdr) memset(s->h_stage + b.stage[b.order[slot]] - kVnetLen, 0, kVnetLen);
  }
  s->state = 3;
  return WGCS_OK;
}

// What Tun.Write(bufs, offset) of batch `write_idx` hands to write(2)
// (tun.go:679-698): status (0 or INVALID_OFFSET -- then nothing is written),
// to_write[k] (handleGRO's toWrite), and for each k the bytes
// bufs[to_write[k]][offset-10:len] after handleGRO: pkts[k] (pinned, valid
// until the slot is recycled), pkt_lens[k].  Arrays hold at least n entries.
int wgcs_wstager_result(wgcs_wstager* ws, uint64_t batch, int write_idx, int* status, int* n_write, int* to_write,
                        const uint8_t** pkts, size_t* pkt_lens) {
  if (!ws || !status || !n_write) return WGCS_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(ws->mu);
  WSlot* s = ws->find(batch);
  if (!s || s->state != 3) return WGCS_ERR_NOT_READY;
  if (write_idx < 0 || (size_t)write_idx >= s->batches.size()) return WGCS_ERR_INVALID_ARG;
  const WBatch& b = s->batches[write_idx];
  *status = b.status;
  *n_write = 0;
  if (b.status) return WGCS_OK;  // Tun.Write returns (0, err) before writing (tun.go:674-676)
  if ((int)b.plan.to_write.size() > 0 && (!to_write || !pkts || !pkt_lens)) return WGCS_ERR_INVALID_ARG;
  const uint8_t* out = b.fixup ? s->h_fix : s->h_out;
  int k = 0;
  for (int i : b.plan.to_write) {
    to_write[k] = i;
    const size_t ln = b.lens[i] - (size_t)b.offset + kVnetLen;
    const uint8_t* p = nullptr;
    for (size_t t = 0; t < b.plan.items.size(); ++t)
      if (b.plan.item_slot[t] == i) p = out + b.plan.items[t].out_off;  // merged super-packet (apply*)
    if (!p) p = s->h_stage + b.stage[b.order[i]] - kVnetLen;         // zero virtio header + the packet as pushed
    pkts[k] = p;
    pkt_lens[k] = ln;
    ++k;
  }
  *n_write = k;
  return WGCS_OK;
}

}  // extern "C"
