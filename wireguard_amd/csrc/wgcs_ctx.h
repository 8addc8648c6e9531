// wgcs_ctx.h -- the opaque wgcs_ctx of include/wgcsum.h.
#pragma once

#include <hip/hip_runtime.h>

#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "../../include/wgcsum.h"
#include "wgcs_kernels.h"

namespace wgcs {

struct DevBuf {
  void* ptr = nullptr;
  size_t cap = 0;
};
struct HostBuf {
  void* ptr = nullptr;
  size_t cap = 0;
};

int set_err(wgcs_ctx* ctx, int code, const char* fmt, ...);
int hip_fail(wgcs_ctx* ctx, hipError_t e, const char* what);
int ensure_dev(wgcs_ctx* ctx, DevBuf& b, size_t bytes);
int ensure_pinned(wgcs_ctx* ctx, HostBuf& b, size_t bytes);
// [p, p + n) lies inside one wgcs_host_alloc allocation of ctx (the _locked
// form: the caller holds ctx->host_mu)
bool host_mapped(wgcs_ctx* ctx, const void* p, size_t n);
bool host_mapped_locked(wgcs_ctx* ctx, const void* p, size_t n);
// A live write-stager slot (open, or submitted and not yet finished) still
// reads [a, b) through a zero-copy push (wstager.cpp); caller holds host_mu.
bool wstager_references(wgcs_wstager* ws, uintptr_t a, uintptr_t b);
// handleVirtioRead / gsoSplit of one job ([virtio header | packet], vlen
// bytes, not modified) into the caller's buffers through the per-call path
// (gso_api.cpp); takes ctx->mu.  Lock order: a read stager's mu before ctx->mu.
int gso_split_staged(wgcs_ctx* ctx, const uint8_t* vbuf, size_t vlen, uint32_t jflags, uint8_t* const* bufs,
                     const size_t* buf_lens, int nbufs, int* sizes, int offset, int* status, int* count);

// The resident per-call ring (ring.cpp): staging for one handleVirtioRead
// (segments at hs + i * pitch, int32 sizes[kbufs] | count | status at meta),
// its post-and-wait, the request bytes as the kernel may read them (caller
// memory from wgcs_host_alloc as it is, else a copy), the ring's lock and
// context.  Caller of ring_gso* / ring_input holds ring_mutex.
int ring_gso_prepare(wgcs_ring* rg, uint32_t kbufs, size_t region, uint8_t** hs, int32_t** meta);
int ring_gso(wgcs_ring* rg, const uint8_t* vbuf, uint32_t vlen, uint32_t jflags, uint32_t kbufs, uint32_t pitch,
             uint32_t room, uint32_t posflags, uint8_t* out, int32_t* meta);
// [p, p + n) lies in wgcs_host_alloc memory the ring reads and writes in place
bool ring_mapped(wgcs_ring* rg, const void* p, size_t n);
int ring_input(wgcs_ring* rg, const uint8_t* p, size_t n, const uint8_t** out);
std::mutex& ring_mutex(wgcs_ring* rg);
wgcs_ctx* ring_ctx(wgcs_ring* rg);

}  // namespace wgcs

struct wgcs_ctx {
  int device = 0;
  int num_cu = 256;
  hipStream_t stream = nullptr;
  std::mutex mu;
  wgcs::LaunchTuning tune;
  // device staging (grown on demand, never shrunk)
  wgcs::DevBuf d_arena, d_pkts, d_init, d_out, d_out2, d_aux;
  // pinned host staging
  wgcs::HostBuf h_stage, h_meta, h_out;
  // stream-join events of wgcs_checksum_batches (timing disabled; [1, 16) made by wgcs_init)
  hipEvent_t join_ev[WGCS_MAX_BATCH_STREAMS] = {};
  // wgcs_host_alloc allocations (device-readable pinned memory): [start, end),
  // the live write stagers, whose zero-copy pushes point into them, and the
  // live read stagers (wgcs_destroy refuses while any stager is alive).  Lock
  // order: host_mu before a write stager's mu; a read stager's mu before mu.
  std::mutex host_mu;
  std::vector<std::pair<uintptr_t, uintptr_t>> host_allocs;
  std::vector<wgcs_wstager*> wstagers;
  std::vector<wgcs_stager*> stagers;
};
