// gro_host.cpp -- handleGRO (/root/reference/tun/gro.go:1326-1367) behind the
// C ABI, MI355X-first:
//   1. the candidate packets are gathered once into pinned staging, which
//      the kernels read over PCIe (no copy commands); checksumValid
//      (gro.go:554-612) for every candidate is computed by the batch VALIDATE
//      kernel.  Validation always
//      precedes mutation in the reference (gro.go:665-681, :709-723,
//      :767-775), so precomputed validity bits are exact.  The plan (2) is
//      made first assuming valid checksums and queued with the VALIDATE
//      launch (one round trip); it is redone if a bit it used is false.
//   2. the order-dependent flow-table decisions of tcpGRO / udpGRO
//      (gro.go:801-1095: Go maps keyed by flow, sequence adjacency, PSH,
//      capacity, prepend swaps) run here on the host, on headers and lengths
//      only -- no payload byte is touched; appends are recorded as a gather
//      plan per output buffer.
//   3. the GPU coalesce kernel (gro_kernels.hip) builds every merged
//      super-packet (payload gather + applyTCPCoalesce/applyUDPCoalesce
//      header rewrite + virtio header) into pinned staging, and the results
//      are copied into the caller's buffers.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "../../include/wgcsum.h"
#include "wgcs_ctx.h"
#include "wgcs_gro_plan.h"
#include "wgcs_kernels.h"

using namespace wgcs;

namespace {

using namespace wgcs::gro;

// Queue the coalesce plan on stream s, zero-copy: the kernel reads the staged
// packets, the items and the pieces from pinned host memory and writes the
// super-packets into pinned host memory (pinned staging is mapped into the
// device's address space at its host address, checked by ensure_pinned).
int queue_coalesce(wgcs_ctx* ctx, const Plan& pl, hipStream_t s) {
  if (pl.items.empty()) return WGCS_OK;
  const size_t ib = pl.items.size() * sizeof(GroItem), sb = std::max<size_t>(pl.segs.size(), 1) * sizeof(GroSeg);
  int rc;
  if ((rc = ensure_pinned(ctx, ctx->h_meta, ib + sb)) || (rc = ensure_pinned(ctx, ctx->h_out, pl.out_bytes + 16)))
    return rc;
  memcpy(ctx->h_meta.ptr, pl.items.data(), ib);
  memcpy((uint8_t*)ctx->h_meta.ptr + ib, pl.segs.data(), pl.segs.size() * sizeof(GroSeg));
  const hipError_t e =
      launch_gro_coalesce((const uint8_t*)ctx->h_stage.ptr, (const GroItem*)ctx->h_meta.ptr, (uint32_t)pl.items.size(),
                          (const GroSeg*)((uint8_t*)ctx->h_meta.ptr + ib), (uint32_t)pl.segs.size(),
                          (uint8_t*)ctx->h_out.ptr, s);
  return e == hipSuccess ? WGCS_OK : hip_fail(ctx, e, "GRO coalesce");
}

}  // namespace

// handleGRO with one GPU round trip in the common case: the flow plan is made
// assuming every candidate's checksum is valid and queued together with the
// VALIDATE kernel; if any validity bit the plan consulted turns out false,
// the slice headers are restored and the plan is redone with the real bits
// (a second round trip).  Results are therefore always those of the
// reference's order of checks (gro.go:665-681, :709-723, :767-775).
extern "C" int wgcs_handle_gro(wgcs_ctx* ctx, uint8_t** bufs, size_t* lens, size_t* caps, int n, int offset,
                               int can_udp_gro, int* to_write, int* n_to_write) {
  if (!ctx || !n_to_write || (n > 0 && (!bufs || !lens || !caps || !to_write))) return WGCS_ERR_INVALID_ARG;
  *n_to_write = 0;
  if (n <= 0) return WGCS_OK;
  // gro.go:1335-1337: the loop returns "invalid offset" at the first bad
  // buffer, after the earlier ones went through tcpGRO / udpGRO
  int n_eff = n;
  for (int i = 0; i < n; ++i)
    if (offset < kVnetLen || (long)offset > (long)lens[i] - 1) {
      n_eff = i;
      break;
    }
  const bool bad_offset = n_eff < n;

  std::vector<const uint8_t*> orig(n, nullptr);
  std::vector<int> cand(n, NOT_CAND);
  std::vector<uint64_t> stage_off(n, 0);
  std::vector<uint8_t> assume(n, 0);
  uint64_t stage_bytes = 0;
  uint32_t ncand = 0;
  for (int i = 0; i < n_eff; ++i) {
    orig[i] = bufs[i] + offset;
    cand[i] = gro_candidate(orig[i], lens[i] - offset, can_udp_gro != 0);
    if (cand[i] != NOT_CAND) {
      stage_off[i] = stage_bytes;
      stage_bytes += (lens[i] - offset + 15) & ~(size_t)15;
      assume[i] = 1;
      ++ncand;
    }
  }
  // slice headers as the caller passed them (restored if the plan is redone)
  const std::vector<uint8_t*> bufs0(bufs, bufs + n);
  const std::vector<size_t> lens0(lens, lens + n), caps0(caps, caps + n);

  Planner P;
  init_planner(P, bufs, lens, caps, n_eff, offset, orig, assume);
  Plan pl;
  make_plan(P, cand, stage_off, n_eff, bad_offset, pl);

  std::lock_guard<std::mutex> g(ctx->mu);
  hipSetDevice(ctx->device);
  hipStream_t s = ctx->stream;
  int rc;
  std::vector<uint8_t> real(n, 0);
  if (ncand) {
    // ---- one submission: stage candidates (pinned), VALIDATE, coalesce
    // (speculative plan); the kernels read and write pinned host memory
    // directly, so there is no copy command, one wait
    const size_t meta = (size_t)ncand * sizeof(wgcs_pkt);
    const size_t stage_al = (stage_bytes + 15) & ~(size_t)15;
    if ((rc = ensure_pinned(ctx, ctx->h_stage, stage_al + 16 + meta + ncand + 16))) return rc;
    uint8_t* hs = (uint8_t*)ctx->h_stage.ptr;
    wgcs_pkt* hp = (wgcs_pkt*)(hs + stage_al + 16);
    uint8_t* hv = (uint8_t*)(hp + ncand);
    std::vector<int> cidx;
    cidx.reserve(ncand);
    for (int i = 0; i < n_eff; ++i) {
      if (cand[i] == NOT_CAND) continue;
      memcpy(hs + stage_off[i], orig[i], lens0[i] - offset);
      const bool v6 = cand[i] == TCP6 || cand[i] == UDP6;
      const bool udp = cand[i] == UDP4 || cand[i] == UDP6;
      // checksumValid(pkt, item.iphLen (IHL 5 for IPv4 candidates), proto, isV6)
      wgcs_pkt_set(&hp[cidx.size()], stage_off[i], (uint32_t)(lens0[i] - offset), (uint16_t)(v6 ? 40 : 20), 0,
                   (uint8_t)(udp ? 17 : 6), (uint8_t)(v6 ? WGCS_PKT_V6 : 0));
      cidx.push_back(i);
    }
    hipError_t e = launch_checksum_batch(WGCS_MODE_VALIDATE, 0, hs, hp, nullptr, ncand, hv, s, ctx->num_cu, ctx->tune);
    if (e != hipSuccess) return hip_fail(ctx, e, "GRO validate");
    if ((rc = queue_coalesce(ctx, pl, s))) return rc;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return hip_fail(ctx, e, "GRO sync");
    for (uint32_t k = 0; k < ncand; ++k) real[cidx[k]] = hv[k];
    bool redo = false;
    for (int i = 0; i < n_eff && !redo; ++i) redo = P.consulted[i] && !real[i];
    if (redo) {  // mis-speculated: restore the slice headers, plan with the real bits
      std::copy(bufs0.begin(), bufs0.end(), bufs);
      std::copy(lens0.begin(), lens0.end(), lens);
      std::copy(caps0.begin(), caps0.end(), caps);
      Planner Q;
      init_planner(Q, bufs, lens, caps, n_eff, offset, orig, real);
      pl = Plan();
      make_plan(Q, cand, stage_off, n_eff, bad_offset, pl);
      if ((rc = queue_coalesce(ctx, pl, s))) return rc;
      if (!pl.items.empty() && (e = hipStreamSynchronize(s)) != hipSuccess) return hip_fail(ctx, e, "GRO sync");
    }
  }

  // ---- apply: empty virtio headers, coalesced super-packets (or, after an
  // invalid offset, the raw coalesced bytes), toWrite
  static const uint8_t zero_hdr[kVnetLen] = {0};
  for (int slot : pl.zero_hdr) memcpy(bufs[slot] + offset - kVnetLen, zero_hdr, kVnetLen);
  for (size_t k = 0; k < pl.items.size(); ++k) {
    const int slot = pl.item_slot[k];
    const GroItem& it = pl.items[k];
    if (it.kind & GRO_KIND_RAW)
      memcpy(bufs[slot] + offset, (uint8_t*)ctx->h_out.ptr + it.out_off + kVnetLen, it.pkt_len);  // RAW item
    else
      memcpy(bufs[slot] + offset - kVnetLen, (uint8_t*)ctx->h_out.ptr + it.out_off, kVnetLen + it.pkt_len);
  }
  for (int i : pl.to_write) to_write[(*n_to_write)++] = i;
  return bad_offset ? set_err(ctx, WGCS_ERR_INVALID_OFFSET, "invalid offset (packet %d)", n_eff) : WGCS_OK;
}

// Device-resident batch of Tun.Write calls: handleGRO per call, one workgroup
// per call, everything in HBM (gro_batch_kernels.hip).
extern "C" int wgcs_handle_gro_batch(wgcs_ctx* ctx, uint8_t* d_arena, wgcs_gro_buf* d_bufs,
                                     const wgcs_gro_call* d_calls, uint32_t n_calls, int32_t* d_status,
                                     int32_t* d_n_write, int32_t* d_to_write, void* stream) {
  if (!ctx) return WGCS_ERR_INVALID_ARG;
  if (n_calls == 0) return WGCS_OK;
  if (!d_arena || !d_bufs || !d_calls || !d_status || !d_n_write || !d_to_write)
    return set_err(ctx, WGCS_ERR_INVALID_ARG, "NULL pointer");
  std::lock_guard<std::mutex> g(ctx->mu);
  hipSetDevice(ctx->device);
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  const hipError_t e = launch_gro_batch(d_arena, d_bufs, d_calls, n_calls, d_status, d_n_write, d_to_write, s);
  return e == hipSuccess ? WGCS_OK : hip_fail(ctx, e, "handle_gro_batch launch");
}
