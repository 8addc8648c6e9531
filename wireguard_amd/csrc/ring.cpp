// ring.cpp -- the resident per-call ring (include/wgcsum.h, wgcs_ring_*).
//
// Round 6: the per-call entry points (wgcs_checksum_valid,
// wgcs_handle_virtio_read) pay one kernel launch plus one completion wait per
// Go call -- ~20 us on MI355X, more than the Go code of one Tun.Read
// (INTEGRATION.md §2.0).  A ring keeps ring_kernel
// (gso_kernels.hip) resident on a few CUs of its own stream; a call fills the
// request record in fine-grained pinned host memory, publishes it by storing
// the request number last, and spins on the completion word the workgroups
// bump after a system-scope release of their results.  Same arguments, bytes
// and errors as the per-call forms (tun/gro.go:554-612, tun/tun.go:514-632);
// only the transport differs.
//
// Liveness: the kernel leaves after `idle_us` without a request (and on
// wgcs_ring_destroy's stop word), so no launch outlives its use; a call that
// finds it gone (hipStreamQuery) launches it again, telling it the request
// number it last served.  One request is in flight at a time (ring->mu).
// Memory: the request bytes must be readable as they are at the call -- the
// ring's own staging and wgcs_host_alloc memory are fine-grained (coherent)
// allocations the GPU does not cache; other caller memory is copied into the
// ring's staging first, and results land in the ring's staging and are copied
// out (gso_api.cpp's post-processing), so every byte matches the per-call path.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>

#include "../../include/wgcsum.h"
#include "wgcs_ctx.h"
#include "wgcs_kernels.h"

using namespace wgcs;

struct wgcs_ring {
  wgcs_ctx* ctx = nullptr;
  hipStream_t stream = nullptr;
  RingCtl* ctl = nullptr;     // coherent pinned: the request and completion records
  uint8_t* in = nullptr;      // coherent pinned: copied request bytes
  size_t in_cap = 0;
  uint8_t* stage = nullptr;   // coherent pinned: segments / meta of a handleVirtioRead
  size_t stage_cap = 0;
  uint32_t nb = kRingBlocks;  // workgroups (segment groups of a 64-KiB read, kRingWaves x 4 rows each)
  uint64_t idle_ticks = 0;    // s_memrealtime ticks (100 MHz)
  uint32_t seq = 0;           // last request number posted
  uint64_t requests = 0, launches = 0;
  std::mutex mu;
};

namespace {

int grow_coherent(wgcs_ctx* ctx, uint8_t** p, size_t* cap, size_t want) {
  if (want <= *cap) return WGCS_OK;
  if (*p) hipHostFree(*p);
  *p = nullptr;
  *cap = 0;
  const size_t n = ((want < 65536 ? 65536 : want + want / 4) + 4095) & ~(size_t)4095;
  hipError_t e = hipHostMalloc((void**)p, n, hipHostMallocCoherent);
  if (e != hipSuccess) return hip_fail(ctx, e, "hipHostMalloc(coherent)");
  void* d = nullptr;
  e = hipHostGetDevicePointer(&d, *p, 0);
  if (e != hipSuccess || d != *p) {
    hipHostFree(*p);
    *p = nullptr;
    return e != hipSuccess ? hip_fail(ctx, e, "hipHostGetDevicePointer")
                           : set_err(ctx, WGCS_ERR_HIP, "pinned memory is not mapped at its host address");
  }
  *cap = n;
  return WGCS_OK;
}

uint32_t load_acq(const uint32_t* p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }

// WGCS_RING_INLINE=0: checksumValid requests pass a pointer to the packet
// instead of carrying its bytes (A/B measurements)
bool ring_inline_enabled() {
  static const bool on = [] {
    const char* e = getenv("WGCS_RING_INLINE");
    return !(e && e[0] == '0');
  }();
  return on;
}

int launch(wgcs_ring* rg, uint32_t last) {
  hipSetDevice(rg->ctx->device);
  const hipError_t e = launch_ring(rg->ctl, rg->nb, last, rg->idle_ticks, rg->stream);
  if (e != hipSuccess) return hip_fail(rg->ctx, e, "ring_kernel launch");
  ++rg->launches;
  return WGCS_OK;
}

// The request record's words (wgcs_host.h RingReq).
uint32_t* rq_word(RingReq* rq, uint32_t k) { return &rq->c[k >> 2][k & 3]; }
void rq_put(RingReq* rq, uint32_t k, uint32_t v) { __atomic_store_n(rq_word(rq, k), v, __ATOMIC_RELAXED); }
void rq_put64(RingReq* rq, uint32_t lo, uint32_t hi, const void* p) {
  rq_put(rq, lo, (uint32_t)(uintptr_t)p);
  rq_put(rq, hi, (uint32_t)((uint64_t)(uintptr_t)p >> 32));
}

// Inline bytes of the next request: chunk c = {seq, src[12c, 12c + 12)}
// (zeros past n), seq stored after the data, so a chunk read with the new
// seq holds them.
void ring_put_inline(wgcs_ring* rg, const uint8_t* src, uint32_t n) {
  const uint32_t q = rg->seq + 1;  // post_and_wait's number for this request
  for (uint32_t c = 0; c < (n + 11) / 12; ++c) {
    uint32_t w[3] = {0, 0, 0};
    memcpy(w, src + 12 * c, std::min<uint32_t>(12, n - 12 * c));
    uint32_t* ch = rg->ctl->inl[c];
    for (int k = 0; k < 3; ++k) __atomic_store_n(&ch[1 + k], w[k], __ATOMIC_RELAXED);
    __atomic_store_n(&ch[0], q, __ATOMIC_RELEASE);
  }
}

// workgroups [0, nb) have finished request q
bool served(wgcs_ring* rg, uint32_t q, uint32_t nb) {
  for (uint32_t b = 0; b < nb; ++b)
    if (load_acq(&rg->ctl->dn[b].seq) != q) return false;
  return true;
}

// Post the request record (filled by the caller) and wait for the
// completion of the workgroups that work on it: every one for a
// handleVirtioRead, workgroup 0 alone for a checksumValid (the others only
// note its number; a later record they read torn is read again).  Caller
// holds rg->mu.
int post_and_wait(wgcs_ring* rg, uint32_t need = 0) {
  if (need == 0 || need > rg->nb) need = rg->nb;
  RingReq* rq = &rg->ctl->req;
  const uint32_t q = ++rg->seq;
  if (q == 0xFFFFFFFFu) return set_err(rg->ctx, WGCS_ERR_INVALID_ARG, "ring: request numbers exhausted");
  for (int c = 0; c < 8; ++c) __atomic_store_n(&rq->c[c][0], q, __ATOMIC_RELEASE);  // after every field
  ++rg->requests;
  // the kernel may have left on its idle deadline: launch it again, telling
  // it the last request it has seen (it then serves q at once)
  if (hipStreamQuery(rg->stream) == hipSuccess) {
    const int rc = launch(rg, q - 1);
    if (rc) return rc;
  }
  const auto t0 = std::chrono::steady_clock::now();
  for (uint64_t spin = 1;; ++spin) {
    if (served(rg, q, need)) return WGCS_OK;
    if ((spin & 4095) == 0) {
      // the kernel left (idle deadline) between our query and the post: relaunch
      const hipError_t st = hipStreamQuery(rg->stream);
      if (st == hipSuccess) {
        if (served(rg, q, need)) return WGCS_OK;
        const int rc = launch(rg, q - 1);
        if (rc) return rc;
      } else if (st != hipErrorNotReady) {
        return hip_fail(rg->ctx, st, "ring_kernel");
      }
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(5))
        return set_err(rg->ctx, WGCS_ERR_HIP, "ring: request %u not served within 5 s", q);
    }
  }
}

}  // namespace

namespace wgcs {

// handleVirtioRead's device step through the ring: the job's bytes at vbuf
// (coherent memory), segments into the ring's staging at i * pitch, int32
// sizes[kbufs] | count | status after them.  Returns the staging pointers.
int ring_gso_prepare(wgcs_ring* rg, uint32_t kbufs, size_t region, uint8_t** hs, int32_t** meta) {
  const size_t mbytes = ((size_t)kbufs * 4 + 16 + 15) & ~(size_t)15;
  const size_t roff = (mbytes + 255) & ~(size_t)255;
  const int rc = grow_coherent(rg->ctx, &rg->stage, &rg->stage_cap, roff + region + 16);
  if (rc) return rc;
  *meta = (int32_t*)rg->stage;
  *hs = rg->stage + roff;
  return WGCS_OK;
}
// (out, meta from ring_gso_prepare; out may instead be the caller's own
// buffers -- bufs[0] + offset with segment i at + i * pitch -- when they are
// ring-readable memory on a fixed stride: gso_api.cpp)
int ring_gso(wgcs_ring* rg, const uint8_t* vbuf, uint32_t vlen, uint32_t jflags, uint32_t kbufs, uint32_t pitch,
             uint32_t room, uint32_t posflags, uint8_t* out, int32_t* meta) {
  RingReq* rq = &rg->ctl->req;
  uint32_t hin = 0;  // inline header bytes (with the phase padding)
  if (ring_inline_enabled()) {
    const uint32_t ph = (uint32_t)((uintptr_t)vbuf & 15u);
    const uint32_t n = vlen < kRingHdrBytes ? vlen : kRingHdrBytes;
    hin = ph + n;
    uint8_t tmp[16 + kRingHdrBytes] = {};
    memcpy(tmp + ph, vbuf, n);
    ring_put_inline(rg, tmp, hin);
  }
  rq_put(rq, kRqHdrInl, hin);
  rq_put(rq, kRqOp, kRingOpVirtioRead);
  rq_put64(rq, kRqVbufLo, kRqVbufHi, vbuf);
  rq_put(rq, kRqVlen, vlen);
  rq_put(rq, kRqJflags, jflags);
  rq_put(rq, kRqKbufs, kbufs);
  rq_put(rq, kRqPitch, pitch);
  rq_put(rq, kRqRoom, room);
  rq_put(rq, kRqPosFlags, posflags);
  rq_put64(rq, kRqOutLo, kRqOutHi, out);
  rq_put64(rq, kRqMetaLo, kRqMetaHi, meta);
  return post_and_wait(rg);
}

// The request bytes as the kernel may read them: caller memory from
// wgcs_host_alloc as it is, anything else copied into the ring's staging.
int ring_input(wgcs_ring* rg, const uint8_t* p, size_t n, const uint8_t** out) {
  if (n == 0 || host_mapped(rg->ctx, p, n)) {
    *out = p;
    return WGCS_OK;
  }
  const int rc = grow_coherent(rg->ctx, &rg->in, &rg->in_cap, n + 64);
  if (rc) return rc;
  memcpy(rg->in, p, n);
  *out = rg->in;
  return WGCS_OK;
}

bool ring_mapped(wgcs_ring* rg, const void* p, size_t n) { return host_mapped(rg->ctx, p, n); }
std::mutex& ring_mutex(wgcs_ring* rg) { return rg->mu; }
wgcs_ctx* ring_ctx(wgcs_ring* rg) { return rg->ctx; }

}  // namespace wgcs

extern "C" {

int wgcs_ring_create(wgcs_ctx* ctx, uint32_t idle_us, wgcs_ring** out) {
  if (!ctx || !out) return WGCS_ERR_INVALID_ARG;
  *out = nullptr;
  hipSetDevice(ctx->device);
  wgcs_ring* rg = new wgcs_ring;
  rg->ctx = ctx;
  rg->idle_ticks = (uint64_t)(idle_us ? idle_us : 100000) * 100;  // s_memrealtime: 100 MHz
  hipError_t e = hipStreamCreateWithFlags(&rg->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete rg;
    return hip_fail(ctx, e, "hipStreamCreate");
  }
  uint8_t* c = nullptr;
  size_t cc = 0;
  int rc = grow_coherent(ctx, &c, &cc, sizeof(RingCtl));
  if (rc) {
    hipStreamDestroy(rg->stream);
    delete rg;
    return rc;
  }
  rg->ctl = (RingCtl*)c;
  memset(rg->ctl, 0, sizeof(RingCtl));
  *out = rg;
  return WGCS_OK;
}

int wgcs_ring_destroy(wgcs_ring* rg) {
  if (!rg) return WGCS_ERR_INVALID_ARG;
  {
    std::lock_guard<std::mutex> g(rg->mu);
    hipSetDevice(rg->ctx->device);
    __atomic_store_n(rq_word(&rg->ctl->req, kRqStop), 1u, __ATOMIC_RELEASE);
    hipStreamSynchronize(rg->stream);  // every workgroup leaves on the stop word
    hipStreamDestroy(rg->stream);
    hipHostFree(rg->ctl);
    if (rg->in) hipHostFree(rg->in);
    if (rg->stage) hipHostFree(rg->stage);
  }
  delete rg;
  return WGCS_OK;
}

int wgcs_ring_info(wgcs_ring* rg, uint64_t* requests, uint64_t* launches, int* running) {
  if (!rg) return WGCS_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(rg->mu);
  if (requests) *requests = rg->requests;
  if (launches) *launches = rg->launches;
  if (running) *running = hipStreamQuery(rg->stream) == hipErrorNotReady ? 1 : 0;
  return WGCS_OK;
}

#ifdef WGCS_RING_STAMPS
// probe builds only (not in include/wgcsum.h): the last request's phase stamps
// of workgroup b, 4 words (ring_kernel, WGCS_RING_STAMPS)
int wgcs_ring_debug_stamps(wgcs_ring* rg, int b, uint32_t* out) {
  if (!rg || b < 0 || b >= (int)wgcs::kRingMaxBlocks || !out) return WGCS_ERR_INVALID_ARG;
  const volatile uint32_t* d = reinterpret_cast<const volatile uint32_t*>(&rg->ctl->dn[b]);
  for (int i = 0; i < 4; ++i) out[i] = d[4 + i];
  return WGCS_OK;
}
#endif

// checksumValid through the ring: wgcs_checksum_valid_cap's arguments and errors.
int wgcs_ring_checksum_valid_cap(wgcs_ring* rg, const uint8_t* pkt, size_t len, size_t cap, uint8_t iph_len,
                                 uint8_t proto, int is_v6, int* valid) {
  if (!rg || !valid || (!pkt && cap) || cap < len) return WGCS_ERR_INVALID_ARG;
  wgcs_ctx* ctx = rg->ctx;
  const size_t need = is_v6 ? 40 : 20;
  if (cap < need || len < iph_len)
    return set_err(ctx, WGCS_ERR_OUT_OF_RANGE, "pkt[%u:] or its addresses past the slice", (unsigned)iph_len);
  if (len >= 0x80000000u) return set_err(ctx, WGCS_ERR_INVALID_ARG, "packet too large");
  std::lock_guard<std::mutex> g(rg->mu);
  RingReq* rq = &rg->ctl->req;
  const size_t nbytes = std::max(len, need);  // what checksumValid reads
  int rc;
  if (nbytes <= kRingInlineMax && ring_inline_enabled()) {
    // the bytes travel with the request: chunk c = {seq, pkt[12c, 12c + 12)},
    // seq stored after the data, so a chunk read with the new seq holds them
    ring_put_inline(rg, pkt, (uint32_t)nbytes);
    rq_put(rq, kRqOp, kRingOpChecksumInline);
    rq_put(rq, kRqInl, (uint32_t)nbytes);
  } else {
    const uint8_t* p = nullptr;
    if ((rc = ring_input(rg, pkt, nbytes, &p))) return rc;
    rq_put(rq, kRqOp, kRingOpChecksumValid);
    rq_put64(rq, kRqPktLo, kRqPktHi, p);
  }
  rq_put(rq, kRqLen, (uint32_t)len);
  rq_put(rq, kRqCs, iph_len);
  rq_put(rq, kRqProto, proto);
  rq_put(rq, kRqFlags, is_v6 ? WGCS_PKT_V6 : 0u);
  if ((rc = post_and_wait(rg, 1))) return rc;
  *valid = (int)__atomic_load_n(&rg->ctl->dn[0].valid, __ATOMIC_ACQUIRE);

  return WGCS_OK;
}

int wgcs_ring_checksum_valid(wgcs_ring* rg, const uint8_t* pkt, size_t len, uint8_t iph_len, uint8_t proto,
                             int is_v6, int* valid) {
  return wgcs_ring_checksum_valid_cap(rg, pkt, len, len, iph_len, proto, is_v6, valid);
}

}  // extern "C"
