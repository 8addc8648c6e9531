// wstager.cpp -- Tun.Write batch staging.
//
// The reference handles one Write call at a time: handleGRO over <= 128
// packets (tun/tun.go:654-700 -> gro.go:1326-1367), then one write(2) per
// toWrite entry of bufs[i][offset-10:] (tun.go:687-698); it is called from
// every peer's RoutineSendToInternet (device/receive.go:483-498).  One such
// call is far too small for a GPU round trip (wgcs_handle_gro: ~55 us), so the
// write stager aggregates many Write calls into one pinned ring slot and runs
// all of handleGRO on the GPU, one workgroup per call (gro_batch_kernels.hip):
//
//   push      copy one Write call's packets into the pinned slot, back to back
//             (16 B of headroom before each holds the caller's
//             bufs[i][offset-10:offset]); record each as a Go slice of the
//             caller's capacity in the slot's device arena.  No host planning.
//   submit    slot stream: H2D of the packets and descriptors -> scatter into
//             the slices -> ONE handleGRO launch over every call (flow table,
//             checksumValid, coalescing, apply*, all on the device) -> gather
//             every call's toWrite images into its output region -> one D2H
//   wait      the slot's event
//   result    per call, what Tun.Write hands to write(2): for each toWrite
//             index the bytes bufs[i][offset-10:len(bufs[i])] after handleGRO,
//             in pinned memory (a 10-byte virtio header + packet)
//
// wgcs_wstager_push_pinned is the zero-copy form: the caller's buffers live in
// pinned memory from wgcs_host_alloc, push only records descriptors, and the
// scatter kernel reads the packets straight from host memory over PCIe.
//
// `depth` slots rotate, each with its own stream: slot k's D2H overlaps slot
// k+1's kernels and slot k+2's H2D.  The caller's buffers are only read by
// push; handleGRO's in-place edits of bufs are not replayed into them (Write's
// callers recycle bufs after the call, device/receive.go:500-505).
//
// Device arena layout of one staged buffer (16-byte aligned region R): the
// packet at P = align128(R + 32 + align16(offset)) + phase, where phase is the packet's
// address mod 16 in its source (0 for the packed stage, the caller's for
// pinned pushes), so source and slice share their phase; the slice `off` =
// P - offset holds cap bytes; 16+ bytes of pad on both sides.  The scatter and
// the gather move whole aligned 16-byte chunks.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/wgcsum.h"
#include "wgcs_ctx.h"
#include "wgcs_kernels.h"

using namespace wgcs;
using wgcs::host_mapped;

namespace {

constexpr size_t kHead = 16;  // headroom before each staged packet: its virtio header bytes go there
constexpr int kVnet = 10;     // virtioNetHdrLen (tun/gro.go:67)

inline size_t al16(size_t x) { return (x + 15) & ~(size_t)15; }

struct WCall {  // one Tun.Write call
  int n = 0, offset = 0;
  int status = 0;   // 0 or WGCS_ERR_INVALID_OFFSET (gro.go:1335-1337) before the launch
  int dev = -1;     // index among the slot's device calls (-1: nothing staged)
  uint32_t first = 0;
  uint64_t out_base = 0;  // its output region in h_out
};

// Output bytes reserved per packet: its write(2) image as whole aligned chunks
// (align16(len + 10) + up to 15 bytes of phase) fits in 32 + align16(len).
inline size_t out_need(size_t pl) { return 32 + al16(pl); }
// Device arena bytes of one slice (+112: the packet moved up to the next
// 128-byte line, below)
inline uint64_t arena_need(size_t offset, size_t cap) { return 64 + 112 + al16(offset) + al16(cap - offset); }
inline uint64_t al128(uint64_t x) { return (x + 127) & ~(uint64_t)127; }

struct WSlot {
  uint64_t id = 0;
  int state = 0;  // 0 free, 1 open, 2 submitted, 3 done
  std::vector<WCall> calls;
  size_t used = 0;      // staged bytes (copying pushes)
  size_t out_used = 0;  // output region bytes
  uint64_t arena = 0;   // device arena bytes of the staged slices
  uint32_t npk = 0, ndev = 0;
  int copying = 0;      // pushes whose packet copies into h_stage are still running
  // pinned host
  uint8_t* h_stage = nullptr;
  wgcs_gro_buf* h_bufs = nullptr;
  WsMove* h_moves = nullptr;
  wgcs_gro_call* h_calls = nullptr;
  WsOut* h_outs = nullptr;
  int32_t* h_res = nullptr;  // status[ndev] | n_write[ndev] | to_write[npk] | wlen[npk] | wpos[npk]
  uint8_t* h_out = nullptr;
  // device
  uint8_t* d_stage = nullptr;
  wgcs_gro_buf* d_bufs = nullptr;
  WsMove* d_moves = nullptr;
  wgcs_gro_call* d_calls = nullptr;
  WsOut* d_outs = nullptr;
  int32_t* d_res = nullptr;
  uint8_t* d_out = nullptr;
  uint8_t* d_arena = nullptr;
  size_t arena_cap = 0;
  hipStream_t stream = nullptr;
  hipEvent_t done = nullptr;

  const int32_t* res_status() const { return h_res; }
  const int32_t* res_nwrite() const { return h_res + ndev; }
  const int32_t* res_towrite() const { return h_res + 2 * (size_t)ndev; }
  const int32_t* res_wlen() const { return h_res + 2 * (size_t)ndev + npk; }
  const int32_t* res_wpos() const { return h_res + 2 * (size_t)ndev + 2 * (size_t)npk; }
};

}  // namespace

struct wgcs_wstager {
  wgcs_ctx* ctx = nullptr;
  uint32_t depth = 0, max_writes = 0, max_pkts = 0;
  size_t max_bytes = 0, max_out = 0;
  std::vector<WSlot> slots;
  uint32_t open = 0;
  uint64_t next_id = 1;
  bool broken = false;  // a ring slot could not be opened (HIP error): every later call fails
  std::mutex mu;
  std::condition_variable copied;  // a push finished copying into its slot
  WSlot* find(uint64_t id) {
    for (auto& s : slots)
      if (s.id == id && id != 0) return &s;
    return nullptr;
  }
};

namespace {

void free_wslot(WSlot& s) {
  for (void* p : {(void*)s.h_stage, (void*)s.h_bufs, (void*)s.h_moves, (void*)s.h_calls, (void*)s.h_outs,
                  (void*)s.h_res, (void*)s.h_out})
    if (p) hipHostFree(p);
  for (void* p : {(void*)s.d_stage, (void*)s.d_bufs, (void*)s.d_moves, (void*)s.d_calls, (void*)s.d_outs,
                  (void*)s.d_res, (void*)s.d_out, (void*)s.d_arena})
    if (p) hipFree(p);
  if (s.done) hipEventDestroy(s.done);
  if (s.stream) hipStreamDestroy(s.stream);
  s = WSlot();
}

// Device arena bytes one slot may stage (the slices of its calls; each slice
// holds its capped capacity, arena_need): a push that would pass it is
// BATCH_FULL, or INVALID_ARG for a call that alone exceeds it.
constexpr uint64_t kMaxArena = 8ull << 30;

int open_wslot(wgcs_wstager* ws, uint32_t idx) {
  WSlot& s = ws->slots[idx];
  if (s.state == 2) {
    hipError_t e = hipEventSynchronize(s.done);
    if (e != hipSuccess) {
      ws->broken = true;  // ws->open still names the submitted slot: nothing may be pushed into it
      return hip_fail(ws->ctx, e, "wstager: wait for ring slot (stager unusable)");
    }
  }
  s.id = ws->next_id++;
  s.state = 1;
  s.calls.clear();
  s.used = 0;
  s.out_used = 0;
  s.arena = 0;
  s.npk = s.ndev = 0;
  s.copying = 0;
  ws->open = idx;
  return WGCS_OK;
}

}  // namespace

namespace wgcs {

bool wstager_references(wgcs_wstager* ws, uintptr_t a, uintptr_t b) {
  std::lock_guard<std::mutex> g(ws->mu);
  for (const WSlot& s : ws->slots) {
    if (s.state != 1 && !(s.state == 2 && hipEventQuery(s.done) == hipErrorNotReady)) continue;
    for (uint32_t k = 0; k < s.npk; ++k) {
      const WsMove& m = s.h_moves[k];
      if ((m.flags & WS_MOVE_ABS) && m.src < b && m.src + 16ull * m.n16 > a) return true;
    }
  }
  return false;
}

}  // namespace wgcs

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
  ws->max_out = al16(max_bytes + (size_t)max_pkts * 48);
  ws->slots.resize(depth);
  hipSetDevice(ctx->device);
  const size_t nres = (2 * (size_t)max_writes + 3 * (size_t)max_pkts) * sizeof(int32_t);
  for (auto& s : ws->slots) {
    hipError_t e = hipSuccess;
    if (e == hipSuccess) e = hipHostMalloc((void**)&s.h_stage, ws->max_bytes + 64, hipHostMallocDefault);
    if (e == hipSuccess) e = hipHostMalloc((void**)&s.h_bufs, max_pkts * sizeof(wgcs_gro_buf), hipHostMallocDefault);
    if (e == hipSuccess) e = hipHostMalloc((void**)&s.h_moves, max_pkts * sizeof(WsMove), hipHostMallocDefault);
    if (e == hipSuccess) e = hipHostMalloc((void**)&s.h_calls, max_writes * sizeof(wgcs_gro_call), hipHostMallocDefault);
    if (e == hipSuccess) e = hipHostMalloc((void**)&s.h_outs, max_writes * sizeof(WsOut), hipHostMallocDefault);
    if (e == hipSuccess) e = hipHostMalloc((void**)&s.h_res, nres, hipHostMallocDefault);
    if (e == hipSuccess) e = hipHostMalloc((void**)&s.h_out, ws->max_out + 64, hipHostMallocDefault);
    if (e == hipSuccess) e = hipMalloc((void**)&s.d_stage, ws->max_bytes + 64);
    if (e == hipSuccess) e = hipMalloc((void**)&s.d_bufs, max_pkts * sizeof(wgcs_gro_buf));
    if (e == hipSuccess) e = hipMalloc((void**)&s.d_moves, max_pkts * sizeof(WsMove));
    if (e == hipSuccess) e = hipMalloc((void**)&s.d_calls, max_writes * sizeof(wgcs_gro_call));
    if (e == hipSuccess) e = hipMalloc((void**)&s.d_outs, max_writes * sizeof(WsOut));
    if (e == hipSuccess) e = hipMalloc((void**)&s.d_res, nres);
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
  {
    std::lock_guard<std::mutex> g(ctx->host_mu);
    ctx->wstagers.push_back(ws);
  }
  *out = ws;
  return WGCS_OK;
}

int wgcs_wstager_destroy(wgcs_wstager* ws) {
  if (!ws) return WGCS_ERR_INVALID_ARG;
  {
    std::lock_guard<std::mutex> g(ws->ctx->host_mu);
    auto& v = ws->ctx->wstagers;
    v.erase(std::remove(v.begin(), v.end(), ws), v.end());
  }
  hipSetDevice(ws->ctx->device);
  for (auto& s : ws->slots) {
    if (s.state == 2) hipEventSynchronize(s.done);
    free_wslot(s);
  }
  delete ws;
  return WGCS_OK;
}

namespace {

// Stage one Tun.Write(bufs, offset) call: bufs[i] is a Go slice, its packet at
// bufs[i][offset:lens[i]], cap(bufs[i]) = caps[i] (device/receive.go:483).
// Room and descriptors are reserved under the stager's lock; a copying push
// copies the packet bytes after releasing it, so pushes from many threads (one
// per peer's RoutineSendToInternet) copy concurrently, and submit waits for
// the open slot's copies.  A pinned push copies nothing: its moves point at
// the caller's pinned buffers.
int push_call(wgcs_wstager* ws, const uint8_t* const* bufs, const size_t* lens, const size_t* caps, int n, int offset,
              int can_udp_gro, bool pinned, int* write_idx) {
  if (!ws || !write_idx || n < 0 || (n > 0 && (!bufs || !lens || !caps))) return WGCS_ERR_INVALID_ARG;
  if (n > WGCS_GRO_MAX_CALL)
    return set_err(ws->ctx, WGCS_ERR_INVALID_ARG, "wstager: %d buffers in one Write call (at most %d)", n,
                   WGCS_GRO_MAX_CALL);
  WCall c;
  c.n = n;
  c.offset = offset;
  // handleGRO's loop stops at the first buffer with an invalid offset
  // (gro.go:1335-1337) and Tun.Write then returns (0, err) without writing
  // anything (tun.go:667-676): nothing to stage
  for (int i = 0; i < n; ++i)
    if (offset < kVnet || (long)offset > (long)lens[i] - 1) {
      c.status = WGCS_ERR_INVALID_OFFSET;
      break;
    }
  size_t need = 0, need_out = 0, total = 0;
  uint64_t need_arena = 0;
  if (!c.status) {
    for (int i = 0; i < n; ++i) {
      if (caps[i] < lens[i]) return set_err(ws->ctx, WGCS_ERR_INVALID_ARG, "wstager: cap(bufs[%d]) < len", i);
      total += lens[i] - offset;
      if (!pinned) need += kHead + al16(lens[i] - offset);
      need_out += out_need(lens[i] - offset);
    }
    for (int i = 0; i < n; ++i) need_arena += arena_need((size_t)offset, std::min(caps[i], (size_t)offset + total));
    if (need_arena > kMaxArena)
      return set_err(ws->ctx, WGCS_ERR_INVALID_ARG, "wstager: one Write call needs %llu arena bytes (at most %llu)",
                     (unsigned long long)need_arena, (unsigned long long)kMaxArena);
  }
  uint8_t* stage;
  uint64_t at;
  WSlot* sp;
  // A zero-copy push holds host_mu from its check that every buffer lies in
  // wgcs_host_alloc memory until its moves are recorded (host_mu, then
  // ws->mu, the order wgcs_host_free takes them): a concurrent
  // wgcs_host_free either runs first (this push is refused) or finds the
  // recorded moves (it returns NOT_READY); the memory is never freed under a
  // slot that will read it.
  std::unique_lock<std::mutex> hg(ws->ctx->host_mu, std::defer_lock);
  if (pinned && !c.status) {
    hg.lock();
    for (int i = 0; i < n; ++i)
      if (!host_mapped_locked(ws->ctx, bufs[i] + offset - kVnet, lens[i] - offset + kVnet))
        return set_err(ws->ctx, WGCS_ERR_INVALID_ARG, "wstager: bufs[%d] is not in wgcs_host_alloc memory", i);
  }
  {
    std::lock_guard<std::mutex> g(ws->mu);
    if (ws->broken) return set_err(ws->ctx, WGCS_ERR_HIP, "wstager unusable after a HIP error");
    WSlot& s = ws->slots[ws->open];
    if (s.calls.size() >= ws->max_writes) return set_err(ws->ctx, WGCS_ERR_BATCH_FULL, "wstager: open batch is full");
    if (c.status || n == 0) {
      *write_idx = (int)s.calls.size();
      s.calls.push_back(c);
      return WGCS_OK;
    }
    if (s.npk + (uint32_t)n > ws->max_pkts || s.used + need > ws->max_bytes || s.out_used + need_out > ws->max_out ||
        s.arena + need_arena > kMaxArena) {
      if (s.npk == 0)  // would never fit, even in an empty slot: not a BATCH_FULL the caller can retry
        return set_err(ws->ctx, WGCS_ERR_INVALID_ARG, "wstager: one Write call exceeds max_pkts / max_bytes");
      return set_err(ws->ctx, WGCS_ERR_BATCH_FULL, "wstager: open batch is full");
    }
    c.dev = (int)s.ndev;
    c.first = s.npk;
    c.out_base = s.out_used;
    at = s.used;
    for (int i = 0; i < n; ++i) {
      const size_t pl = lens[i] - (size_t)offset;
      // The device slice's capacity: a coalesced buffer never holds more than
      // all of the call's packets, so capping cap there changes no capacity
      // check of handleGRO (gro.go:685-688, :730-733) and bounds the arena.
      const size_t cap = std::min(caps[i], (size_t)offset + total);
      const uintptr_t hp = (uintptr_t)(bufs[i] + offset);  // the packet in host memory
      const uint64_t phase = pinned ? (uint64_t)(hp & 15u) : 0u;
      // the packet in the arena: on a 128-byte line (+ its source phase mod 16
      // for a zero-copy push), so its reads and the appends behind it touch
      // no more lines than its bytes need (round 5)
      const uint64_t pkt = al128(s.arena + 32 + al16((size_t)offset)) + phase;
      wgcs_gro_buf& b = s.h_bufs[s.npk];
      b.off = pkt - (uint64_t)offset;
      b.len = (uint32_t)lens[i];
      b.cap = (uint32_t)cap;
      WsMove& m = s.h_moves[s.npk];
      if (pinned) {  // the aligned chunks holding bufs[i][offset-10:len], read over PCIe
        const uintptr_t c0 = (hp - kVnet) & ~(uintptr_t)15, c1 = (hp + pl + 15) & ~(uintptr_t)15;
        m.src = (uint64_t)c0;
        m.dst = pkt - (uint64_t)(hp - c0);
        m.n16 = (uint32_t)((c1 - c0) >> 4);
        m.flags = WS_MOVE_ABS;
      } else {  // headroom chunk, then the packet (16-byte aligned in the stage)
        m.src = s.used;
        m.dst = pkt - kHead;
        m.n16 = (uint32_t)((kHead + al16(pl)) >> 4);
        m.flags = 0;
        s.used += kHead + al16(pl);
      }
      s.arena += arena_need((size_t)offset, cap);
      ++s.npk;
    }
    s.out_used += need_out;
    wgcs_gro_call& dc = s.h_calls[s.ndev];
    dc.first = c.first;
    dc.n = (uint32_t)n;
    dc.offset = offset;
    dc.flags = can_udp_gro ? WGCS_GRO_CAN_UDP : 0u;
    WsOut& o = s.h_outs[s.ndev];
    o.base = c.out_base;
    o.room = (uint32_t)need_out;
    o.pad = 0;
    ++s.ndev;
    *write_idx = (int)s.calls.size();
    s.calls.push_back(c);
    if (pinned) return WGCS_OK;
    ++s.copying;
    stage = s.h_stage;
    sp = &s;
  }
  for (int i = 0; i < n; ++i) {  // headroom: 6 zero bytes + bufs[i][offset-10:offset], then the packet
    const size_t pl = lens[i] - (size_t)offset;
    memset(stage + at, 0, kHead - kVnet);
    memcpy(stage + at + kHead - kVnet, bufs[i] + offset - kVnet, kVnet);
    memcpy(stage + at + kHead, bufs[i] + offset, pl);
    at += kHead + al16(pl);
  }
  {
    std::lock_guard<std::mutex> g(ws->mu);
    --sp->copying;
  }
  ws->copied.notify_all();
  return WGCS_OK;
}

}  // namespace

int wgcs_wstager_push(wgcs_wstager* ws, const uint8_t* const* bufs, const size_t* lens, const size_t* caps, int n,
                      int offset, int can_udp_gro, int* write_idx) {
  return push_call(ws, bufs, lens, caps, n, offset, can_udp_gro, false, write_idx);
}

int wgcs_wstager_push_pinned(wgcs_wstager* ws, const uint8_t* const* bufs, const size_t* lens, const size_t* caps,
                             int n, int offset, int can_udp_gro, int* write_idx) {
  return push_call(ws, bufs, lens, caps, n, offset, can_udp_gro, true, write_idx);
}

int wgcs_wstager_submit(wgcs_wstager* ws, uint64_t* batch) {
  if (!ws || !batch) return WGCS_ERR_INVALID_ARG;
  std::unique_lock<std::mutex> g(ws->mu);
  hipSetDevice(ws->ctx->device);
  // Wait for the pushes still copying into the open slot.  The wait releases
  // the lock, so another submit may queue that slot meanwhile: re-read
  // ws->open after every wake-up and submit whatever slot is open then (each
  // submit queues a distinct slot; none is skipped or queued twice).
  ws->copied.wait(g, [&] { return ws->broken || ws->slots[ws->open].copying == 0; });
  if (ws->broken) return set_err(ws->ctx, WGCS_ERR_HIP, "wstager unusable after a HIP error");
  WSlot& s = ws->slots[ws->open];
  const hipStream_t q = s.stream;
  hipError_t e = hipSuccess;
  if (s.ndev) {
    if (s.arena + 64 > s.arena_cap) {  // the slot is idle (open_wslot waited for it)
      if (s.d_arena) hipFree(s.d_arena);
      s.d_arena = nullptr;
      s.arena_cap = 0;
      const size_t want = al16(s.arena + s.arena / 4 + 64);
      e = hipMalloc((void**)&s.d_arena, want);
      if (e != hipSuccess) return hip_fail(ws->ctx, e, "wstager: device arena");
      s.arena_cap = want;
    }
    const uint32_t nd = s.ndev, np = s.npk;
    int32_t* d_status = s.d_res;
    int32_t* d_nw = s.d_res + nd;
    int32_t* d_tw = s.d_res + 2 * (size_t)nd;
    int32_t* d_wlen = s.d_res + 2 * (size_t)nd + np;
    int32_t* d_wpos = s.d_res + 2 * (size_t)nd + 2 * (size_t)np;
    if (s.used) e = hipMemcpyAsync(s.d_stage, s.h_stage, s.used, hipMemcpyHostToDevice, q);
    if (e == hipSuccess) e = hipMemcpyAsync(s.d_bufs, s.h_bufs, np * sizeof(wgcs_gro_buf), hipMemcpyHostToDevice, q);
    if (e == hipSuccess) e = hipMemcpyAsync(s.d_moves, s.h_moves, np * sizeof(WsMove), hipMemcpyHostToDevice, q);
    if (e == hipSuccess) e = hipMemcpyAsync(s.d_calls, s.h_calls, nd * sizeof(wgcs_gro_call), hipMemcpyHostToDevice, q);
    if (e == hipSuccess) e = hipMemcpyAsync(s.d_outs, s.h_outs, nd * sizeof(WsOut), hipMemcpyHostToDevice, q);
    if (e == hipSuccess) e = launch_ws_scatter(s.d_stage, s.d_arena, s.d_moves, np, q);
    if (e == hipSuccess) e = launch_gro_batch(s.d_arena, s.d_bufs, s.d_calls, nd, d_status, d_nw, d_tw, q);
    if (e == hipSuccess)
      e = launch_ws_gather(s.d_arena, s.d_bufs, s.d_calls, s.d_outs, nd, d_status, d_nw, d_tw, d_wlen, d_wpos,
                           s.d_out, q);
    if (e == hipSuccess)
      e = hipMemcpyAsync(s.h_res, s.d_res, (2 * (size_t)nd + 3 * (size_t)np) * sizeof(int32_t), hipMemcpyDeviceToHost,
                         q);
    if (e == hipSuccess) e = hipMemcpyAsync(s.h_out, s.d_out, s.out_used, hipMemcpyDeviceToHost, q);
  }
  if (e == hipSuccess) e = hipEventRecord(s.done, q);
  if (e != hipSuccess) return hip_fail(ws->ctx, e, "wstager submit");
  s.state = 2;
  *batch = s.id;
  return open_wslot(ws, (ws->open + 1) % ws->depth);
}

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
  s->state = 3;
  return WGCS_OK;
}

// What Tun.Write(bufs, offset) of call `write_idx` hands to write(2)
// (tun.go:679-698): status (0 or INVALID_OFFSET -- then nothing is written),
// to_write[k] (handleGRO's toWrite), and for each k the bytes
// bufs[to_write[k]][offset-10:len] after handleGRO: pkts[k] (pinned, valid
// until the slot is recycled), pkt_lens[k].  Arrays hold at least n entries.
int wgcs_wstager_result(wgcs_wstager* ws, uint64_t batch, int write_idx, int* status, int* n_write, int* to_write,
                        const uint8_t** pkts, size_t* pkt_lens) {
  if (!ws || !status || !n_write) return WGCS_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(ws->mu);
  WSlot* s = ws->find(batch);
  if (!s || s->state == 1 || (s->state == 2 && hipEventQuery(s->done) != hipSuccess)) return WGCS_ERR_NOT_READY;
  if (write_idx < 0 || (size_t)write_idx >= s->calls.size()) return WGCS_ERR_INVALID_ARG;
  const WCall& c = s->calls[write_idx];
  *n_write = 0;
  *status = c.status;
  if (c.dev < 0) return WGCS_OK;  // Tun.Write returns (0, err) before writing (tun.go:674-676), or n == 0
  *status = s->res_status()[c.dev];
  if (*status) return WGCS_OK;
  const int nw = s->res_nwrite()[c.dev];
  if (nw > 0 && (!to_write || !pkts || !pkt_lens)) return WGCS_ERR_INVALID_ARG;
  const int32_t* tw = s->res_towrite() + c.first;
  const int32_t* wl = s->res_wlen() + c.first;
  const int32_t* wp = s->res_wpos() + c.first;
  for (int k = 0; k < nw; ++k) {
    to_write[k] = tw[k];
    pkts[k] = s->h_out + c.out_base + (uint32_t)wp[k];
    pkt_lens[k] = (size_t)wl[k];
  }
  *n_write = nw;
  return WGCS_OK;
}

}  // extern "C"
