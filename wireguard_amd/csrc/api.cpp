// api.cpp -- C ABI (include/wgcsum.h): context, staging and the
// reference-shaped host entry points.  All per-byte work is done by the
// gfx950 kernels in checksum_kernels.hip / gso_kernels.hip; there is no CPU
// fallback: if HIP or the device is unavailable every call fails loudly.
#include <hip/hip_runtime.h>

#include <algorithm>

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>

#include "../../include/wgcsum.h"
#include "wgcs_ctx.h"
#include "wgcs_kernels.h"

using namespace wgcs;

namespace wgcs {

// The last error message is per calling thread (like errno): concurrent
// callers of one context (Tun.Write runs on many goroutines, tun.go:654-700)
// never write one shared string, and the pointer wgcs_last_error returns stays
// valid until the same thread's next failing call.
namespace {
thread_local const wgcs_ctx* tls_err_ctx = nullptr;
thread_local char tls_err[512];
}  // namespace

int set_err(wgcs_ctx* ctx, int code, const char* fmt, ...) {
  if (ctx) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(tls_err, sizeof tls_err, fmt, ap);
    va_end(ap);
    tls_err_ctx = ctx;
  }
  return code;
}

int hip_fail(wgcs_ctx* ctx, hipError_t e, const char* what) {
  return set_err(ctx, WGCS_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
}

int ensure_dev(wgcs_ctx* ctx, DevBuf& b, size_t bytes) {
  if (bytes <= b.cap) return WGCS_OK;
  if (b.ptr) hipFree(b.ptr);
  b.ptr = nullptr;
  b.cap = 0;
  size_t want = bytes < 4096 ? 4096 : bytes + bytes / 4;
  hipError_t e = hipMalloc(&b.ptr, want);
  if (e != hipSuccess) return hip_fail(ctx, e, "hipMalloc");
  b.cap = want;
  return WGCS_OK;
}

int ensure_pinned(wgcs_ctx* ctx, HostBuf& b, size_t bytes) {
  if (bytes <= b.cap) return WGCS_OK;
  if (b.ptr) hipHostFree(b.ptr);
  b.ptr = nullptr;
  b.cap = 0;
  size_t want = bytes < 4096 ? 4096 : bytes + bytes / 4;
  hipError_t e = hipHostMalloc(&b.ptr, want, hipHostMallocDefault);
  if (e != hipSuccess) return hip_fail(ctx, e, "hipHostMalloc");
  // kernels take pinned staging pointers as they are (zero-copy per-call paths)
  void* d = nullptr;
  e = hipHostGetDevicePointer(&d, b.ptr, 0);
  if (e != hipSuccess || d != b.ptr) {
    hipHostFree(b.ptr);
    b.ptr = nullptr;
    return e != hipSuccess ? hip_fail(ctx, e, "hipHostGetDevicePointer")
                           : set_err(ctx, WGCS_ERR_HIP, "pinned memory is not mapped at its host address");
  }
  b.cap = want;
  return WGCS_OK;
}

bool host_mapped_locked(wgcs_ctx* ctx, const void* p, size_t n) {
  const uintptr_t a = (uintptr_t)p, b = a + n;
  for (const auto& r : ctx->host_allocs)
    if (a >= r.first && b <= r.second && b >= a) return true;
  return false;
}

bool host_mapped(wgcs_ctx* ctx, const void* p, size_t n) {
  std::lock_guard<std::mutex> g(ctx->host_mu);
  return host_mapped_locked(ctx, p, n);
}

}  // namespace wgcs

extern "C" {

int wgcs_abi_version(void) { return WGCS_ABI_VERSION; }

int wgcs_device_count(int* count) {
  if (!count) return WGCS_ERR_INVALID_ARG;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) {
    *count = 0;
    return WGCS_ERR_NO_DEVICE;
  }
  *count = n;
  return WGCS_OK;
}

int wgcs_init(int device, wgcs_ctx** out) {
  if (!out) return WGCS_ERR_INVALID_ARG;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return WGCS_ERR_NO_DEVICE;
  if (device < 0 || device >= n) return WGCS_ERR_INVALID_ARG;
  wgcs_ctx* ctx = new (std::nothrow) wgcs_ctx();
  if (!ctx) return WGCS_ERR_NOMEM;
  ctx->device = device;
  hipError_t e = hipSetDevice(device);
  // A blocking stream: work a caller queued on the HIP null stream (torch's
  // default stream) before a NULL-stream call is ordered before it, and after
  // it is ordered after it.
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&ctx->stream, hipStreamDefault);
  hipDeviceProp_t prop;
  if (e == hipSuccess) e = hipGetDeviceProperties(&prop, device);
  // stream-join events of wgcs_checksum_batches, made here so that no event is
  // created inside a caller's timed enqueue
  for (int j = 1; j < WGCS_MAX_BATCH_STREAMS && e == hipSuccess; ++j)
    e = hipEventCreateWithFlags(&ctx->join_ev[j], hipEventDisableTiming);
  if (e != hipSuccess) {
    for (hipEvent_t ev : ctx->join_ev)
      if (ev) hipEventDestroy(ev);
    if (ctx->stream) hipStreamDestroy(ctx->stream);
    delete ctx;
    return WGCS_ERR_HIP;
  }
  ctx->num_cu = prop.multiProcessorCount;
  const char* bpc = getenv("WGCS_BLOCKS_PER_CU");
  if (bpc && atoi(bpc) > 0) ctx->tune.blocks_per_cu = atoi(bpc);
  const char* unr = getenv("WGCS_UNROLL");
  if (unr && atoi(unr) > 0) ctx->tune.unroll = atoi(unr);
  const char* lpp = getenv("WGCS_LANES_PER_PKT");
  if (lpp && (atoi(lpp) == 64 || atoi(lpp) == 32 || atoi(lpp) == 16)) ctx->tune.lanes_per_pkt = atoi(lpp);
  const char* nt = getenv("WGCS_NT");
  if (nt) ctx->tune.nt = atoi(nt) ? 1 : 0;
  const char* xc = getenv("WGCS_XCD");
  if (xc) ctx->tune.xcd = atoi(xc) ? 1 : 0;
  const char* al = getenv("WGCS_ALIGN");
  if (al && (atoi(al) == 16 || atoi(al) == 32 || atoi(al) == 64 || atoi(al) == 128)) ctx->tune.align = atoi(al);
  *out = ctx;
  return WGCS_OK;
}

// Pinned host memory the device reads directly (zero-copy Write staging,
// wgcs_wstager_push_pinned).  HIP maps hipHostMalloc memory into the device's
// address space at the same address; that is checked once here, so kernels
// can take the host pointers as they are.
int wgcs_host_alloc(wgcs_ctx* ctx, size_t bytes, void** p) {
  if (!ctx || !p || bytes == 0) return WGCS_ERR_INVALID_ARG;
  *p = nullptr;
  hipSetDevice(ctx->device);
  const size_t n = (bytes + 15) & ~(size_t)15;
  void* h = nullptr;
  // fine-grained (coherent): the resident ring (ring.cpp) reads request bytes
  // here in place, and a buffer reused at one address between requests must
  // not be served from a stale GPU cache line
  hipError_t e = hipHostMalloc(&h, n, hipHostMallocCoherent);
  if (e != hipSuccess) return hip_fail(ctx, e, "wgcs_host_alloc");
  void* d = nullptr;
  e = hipHostGetDevicePointer(&d, h, 0);
  if (e != hipSuccess || d != h) {
    hipHostFree(h);
    return e != hipSuccess ? hip_fail(ctx, e, "hipHostGetDevicePointer")
                           : set_err(ctx, WGCS_ERR_HIP, "pinned memory is not mapped at its host address");
  }
  std::lock_guard<std::mutex> g(ctx->host_mu);
  ctx->host_allocs.emplace_back((uintptr_t)h, (uintptr_t)h + n);
  *p = h;
  return WGCS_OK;
}

int wgcs_host_free(wgcs_ctx* ctx, void* p) {
  if (!ctx || !p) return WGCS_ERR_INVALID_ARG;
  {
    std::lock_guard<std::mutex> g(ctx->host_mu);
    auto& v = ctx->host_allocs;
    auto it = std::find_if(v.begin(), v.end(), [&](const std::pair<uintptr_t, uintptr_t>& r) {
      return r.first == (uintptr_t)p;
    });
    if (it == v.end()) return set_err(ctx, WGCS_ERR_INVALID_ARG, "wgcs_host_free: not a wgcs_host_alloc pointer");
    for (wgcs_wstager* ws : ctx->wstagers)
      if (wstager_references(ws, it->first, it->second))
        return set_err(ctx, WGCS_ERR_NOT_READY, "wgcs_host_free: a write-stager slot still reads this memory");
    v.erase(it);
  }
  const hipError_t e = hipHostFree(p);
  return e == hipSuccess ? WGCS_OK : hip_fail(ctx, e, "hipHostFree");
}

int wgcs_destroy(wgcs_ctx* ctx) {
  if (!ctx) return WGCS_ERR_INVALID_ARG;
  {
    std::lock_guard<std::mutex> g(ctx->host_mu);
    // stagers keep the context (its device, staging and error state) and
    // write stagers' slots may read its host allocations
    if (!ctx->wstagers.empty() || !ctx->stagers.empty())
      return set_err(ctx, WGCS_ERR_INVALID_ARG,
                     "wgcs_destroy: %zu read stager(s) and %zu write stager(s) still alive: destroy them first",
                     ctx->stagers.size(), ctx->wstagers.size());
  }
  hipSetDevice(ctx->device);
  if (ctx->stream) hipStreamSynchronize(ctx->stream);
  for (const auto& r : ctx->host_allocs) hipHostFree((void*)r.first);
  for (DevBuf* b : {&ctx->d_arena, &ctx->d_pkts, &ctx->d_init, &ctx->d_out, &ctx->d_out2, &ctx->d_aux})
    if (b->ptr) hipFree(b->ptr);
  for (HostBuf* b : {&ctx->h_stage, &ctx->h_meta, &ctx->h_out})
    if (b->ptr) hipHostFree(b->ptr);
  if (ctx->stream) hipStreamDestroy(ctx->stream);
  for (hipEvent_t ev : ctx->join_ev)
    if (ev) hipEventDestroy(ev);
  delete ctx;
  return WGCS_OK;
}

const char* wgcs_strerror(int status) {
  switch (status) {
    case WGCS_OK: return "ok";
    case WGCS_ERR_INVALID_ARG: return "invalid argument";
    case WGCS_ERR_SHORT_BUFFER: return "short buffer";
    case WGCS_ERR_TOO_MANY_SEGMENTS: return "too many segments";
    case WGCS_ERR_INVALID_OFFSET: return "invalid offset";
    case WGCS_ERR_UNSUPPORTED_GSO: return "unsupported virtio GSO type";
    case WGCS_ERR_IP_GSO_MISMATCH: return "IP header version / GSO type mismatch";
    case WGCS_ERR_BAD_IP_VERSION: return "invalid IP header version";
    case WGCS_ERR_PACKET_TOO_SHORT: return "packet is too short";
    case WGCS_ERR_TCP_HDR_LEN: return "TCP header length is invalid";
    case WGCS_ERR_HDR_LEN: return "length of packet < virtioNetHdr.hdrLen";
    case WGCS_ERR_CSUM_OFFSET: return "end of checksum offset exceeds packet length";
    case WGCS_ERR_READ_OVERFLOW: return "read length overflows bufs element length";
    case WGCS_ERR_OUT_OF_RANGE: return "slice bounds out of range";
    case WGCS_ERR_BATCH_FULL: return "staging batch full";
    case WGCS_ERR_NOT_READY: return "batch not submitted or already recycled";
    case WGCS_ERR_CMSG: return "error parsing socket control message";
    case WGCS_ERR_SPLIT_OVERFLOW: return "splitting coalesced packet resulted in overflow";
    case WGCS_ERR_HIP: return "HIP runtime error";
    case WGCS_ERR_NOMEM: return "out of memory";
    case WGCS_ERR_NO_DEVICE: return "no HIP device";
    default: return "unknown status";
  }
}

const char* wgcs_last_error(wgcs_ctx* ctx) { return ctx && tls_err_ctx == ctx ? tls_err : ""; }

int wgcs_num_cu(wgcs_ctx* ctx) { return ctx ? ctx->num_cu : WGCS_ERR_INVALID_ARG; }

int wgcs_sync(wgcs_ctx* ctx) {
  if (!ctx) return WGCS_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(ctx->mu);
  hipSetDevice(ctx->device);
  hipError_t e = hipStreamSynchronize(ctx->stream);
  return e == hipSuccess ? WGCS_OK : hip_fail(ctx, e, "hipStreamSynchronize");
}

int wgcs_checksum_batch(wgcs_ctx* ctx, int mode, unsigned flags, uint8_t* d_arena, const wgcs_pkt* d_pkts,
                        const uint64_t* d_initial, uint32_t n, void* d_out, void* stream) {
  if (!ctx) return WGCS_ERR_INVALID_ARG;
  if (mode < WGCS_MODE_FOLD || mode > WGCS_MODE_IP4HDR) return set_err(ctx, WGCS_ERR_INVALID_ARG, "bad mode %d", mode);
  if (n == 0) return WGCS_OK;
  if (!d_arena || !d_pkts || !d_out) return set_err(ctx, WGCS_ERR_INVALID_ARG, "NULL pointer");
  std::lock_guard<std::mutex> g(ctx->mu);
  hipSetDevice(ctx->device);
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  hipError_t e = launch_checksum_batch(mode, flags, d_arena, d_pkts, d_initial, n, d_out, s, ctx->num_cu, ctx->tune);
  return e == hipSuccess ? WGCS_OK : hip_fail(ctx, e, "checksum_batch launch");
}

int wgcs_checksum_batches(wgcs_ctx* ctx, int mode, unsigned flags, const wgcs_batch* batches, uint32_t n_batches,
                          void* const* streams, uint32_t n_streams, void* ev_begin, void* ev_end) {
  if (!ctx) return WGCS_ERR_INVALID_ARG;
  if (mode < WGCS_MODE_FOLD || mode > WGCS_MODE_IP4HDR) return set_err(ctx, WGCS_ERR_INVALID_ARG, "bad mode %d", mode);
  if (n_streams > WGCS_MAX_BATCH_STREAMS || (n_streams && !streams) || (n_batches && !batches))
    return set_err(ctx, WGCS_ERR_INVALID_ARG, "bad stream list (%u streams)", n_streams);
  for (uint32_t k = 0; k < n_batches; ++k)
    if (batches[k].n && (!batches[k].arena || !batches[k].pkts || !batches[k].out))
      return set_err(ctx, WGCS_ERR_INVALID_ARG, "batch %u: NULL pointer", k);
  std::lock_guard<std::mutex> g(ctx->mu);
  hipSetDevice(ctx->device);
  const uint32_t ns = n_streams ? n_streams : 1;
  hipStream_t st[WGCS_MAX_BATCH_STREAMS];
  for (uint32_t j = 0; j < ns; ++j) st[j] = n_streams && streams[j] ? (hipStream_t)streams[j] : ctx->stream;
  hipError_t e = hipSuccess;
  // ev_begin, then batch 0 at once (the first launch is the latency-critical
  // one); each other stream waits on ev_begin just before its first launch
  if (ev_begin && (e = hipEventRecord((hipEvent_t)ev_begin, st[0])) != hipSuccess) return hip_fail(ctx, e, "ev_begin");
  for (uint32_t k = 0; k < n_batches; ++k) {
    const uint32_t j = k % ns;
    if (ev_begin && j != 0 && k < ns && st[j] != st[0] &&
        (e = hipStreamWaitEvent(st[j], (hipEvent_t)ev_begin, 0)) != hipSuccess)
      return hip_fail(ctx, e, "stream wait");
    const wgcs_batch& b = batches[k];
    e = launch_checksum_batch(mode, flags, b.arena, b.pkts, b.initial, b.n, b.out, st[j], ctx->num_cu, ctx->tune);
    if (e != hipSuccess) return hip_fail(ctx, e, "checksum_batches launch");
  }
  if (ev_end) {
    // join only the streams that received a batch: a stream without one may
    // hold unrelated work that must not land inside the bracket
    const uint32_t used = n_batches < ns ? n_batches : ns;
    for (uint32_t j = 1; j < used; ++j) {
      if (st[j] == st[0]) continue;
      if ((e = hipEventRecord(ctx->join_ev[j], st[j])) != hipSuccess ||
          (e = hipStreamWaitEvent(st[0], ctx->join_ev[j], 0)) != hipSuccess)
        return hip_fail(ctx, e, "stream join");
    }
    if ((e = hipEventRecord((hipEvent_t)ev_end, st[0])) != hipSuccess) return hip_fail(ctx, e, "ev_end");
  }
  return WGCS_OK;
}

int wgcs_stream_wait_flag(wgcs_ctx* ctx, void* stream, const uint32_t* flag, uint32_t value) {
  if (!ctx || !flag || ((uintptr_t)flag & 3u)) return WGCS_ERR_INVALID_ARG;
  if (!host_mapped(ctx, flag, sizeof(uint32_t)))
    return set_err(ctx, WGCS_ERR_INVALID_ARG, "wgcs_stream_wait_flag: flag is not wgcs_host_alloc memory");
  std::lock_guard<std::mutex> g(ctx->mu);
  hipSetDevice(ctx->device);
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  const hipError_t e = hipStreamWaitValue32(s, const_cast<uint32_t*>(flag), value, hipStreamWaitValueEq, 0xFFFFFFFFu);
  return e == hipSuccess ? WGCS_OK : hip_fail(ctx, e, "hipStreamWaitValue32");
}

// Host batches up to this size run zero-copy (the kernel reads pinned staging
// over PCIe); larger ones go through copy-engine H2D / D2H.
constexpr size_t kZeroCopyMax = 1u << 20;

int wgcs_checksum_batch_host(wgcs_ctx* ctx, int mode, unsigned flags, uint8_t* h_arena, size_t arena_len,
                             const wgcs_pkt* h_pkts, const uint64_t* h_initial, uint32_t n, void* h_out) {
  if (!ctx) return WGCS_ERR_INVALID_ARG;
  if (mode < WGCS_MODE_FOLD || mode > WGCS_MODE_IP4HDR) return set_err(ctx, WGCS_ERR_INVALID_ARG, "bad mode %d", mode);
  if (n == 0) return WGCS_OK;
  if (!h_pkts || !h_out || (!h_arena && arena_len)) return set_err(ctx, WGCS_ERR_INVALID_ARG, "NULL pointer");
  for (uint32_t i = 0; i < n; ++i) {
    const uint64_t off = (uint64_t)h_pkts[i].off_lo | ((uint64_t)h_pkts[i].off_hi << 32);
    if (h_pkts[i].len >= 0x80000000u || off + h_pkts[i].len > arena_len)
      return set_err(ctx, WGCS_ERR_INVALID_ARG, "packet %u outside the arena", i);
    // VALIDATE / L4_FILL read the pseudo-header addresses whatever len is (a
    // short packet's spare capacity, include/wgcsum.h): the arena is the cap
    const size_t addr_end = (h_pkts[i].flags & WGCS_PKT_V6) ? 40 : 20;
    if ((mode == WGCS_MODE_VALIDATE || mode == WGCS_MODE_L4_FILL) && off + addr_end > arena_len)
      return set_err(ctx, WGCS_ERR_OUT_OF_RANGE, "packet %u: pseudo-header addresses past the arena", i);
  }
  std::lock_guard<std::mutex> g(ctx->mu);
  hipSetDevice(ctx->device);
  const size_t out_bytes = (size_t)n * (mode == WGCS_MODE_VALIDATE ? 1 : 2);
  int rc;
  const bool fold_init = h_initial && mode == WGCS_MODE_FOLD;
  if (arena_len <= kZeroCopyMax) {
    // Small batches (the per-call entry points: one packet or one read):
    // zero-copy through pinned staging -- the kernel reads the packets and
    // descriptors and writes its results over PCIe; one launch, one wait, no
    // copy commands (their fixed costs dominate at this size).
    auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
    const size_t o_pk = al(arena_len) + 16, o_in = o_pk + al(n * sizeof(wgcs_pkt)),
                 o_out = o_in + (fold_init ? al(n * sizeof(uint64_t)) : 0);
    if ((rc = ensure_pinned(ctx, ctx->h_stage, o_out + al(out_bytes) + 16))) return rc;
    uint8_t* hs = (uint8_t*)ctx->h_stage.ptr;
    if (arena_len) memcpy(hs, h_arena, arena_len);
    memcpy(hs + o_pk, h_pkts, n * sizeof(wgcs_pkt));
    if (fold_init) memcpy(hs + o_in, h_initial, n * sizeof(uint64_t));
    hipError_t e = launch_checksum_batch(mode, flags, hs, (const wgcs_pkt*)(hs + o_pk),
                                         fold_init ? (const uint64_t*)(hs + o_in) : nullptr, n, hs + o_out,
                                         ctx->stream, ctx->num_cu, ctx->tune);
    if (e != hipSuccess) return hip_fail(ctx, e, "checksum_batch launch");
    if ((e = hipStreamSynchronize(ctx->stream)) != hipSuccess) return hip_fail(ctx, e, "checksum_batch wait");
    memcpy(h_out, hs + o_out, out_bytes);
    if ((flags & WGCS_F_INPLACE) && arena_len) memcpy(h_arena, hs, arena_len);
    return WGCS_OK;
  }
  if ((rc = ensure_dev(ctx, ctx->d_arena, arena_len + 16)) || (rc = ensure_dev(ctx, ctx->d_pkts, n * sizeof(wgcs_pkt))) ||
      (rc = ensure_dev(ctx, ctx->d_out, out_bytes)))
    return rc;
  if (fold_init && (rc = ensure_dev(ctx, ctx->d_init, n * sizeof(uint64_t)))) return rc;
  hipStream_t s = ctx->stream;
  hipError_t e = hipMemcpyAsync(ctx->d_arena.ptr, h_arena, arena_len, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipMemcpyAsync(ctx->d_pkts.ptr, h_pkts, n * sizeof(wgcs_pkt), hipMemcpyHostToDevice, s);
  const uint64_t* dinit = nullptr;
  if (e == hipSuccess && h_initial && mode == WGCS_MODE_FOLD) {
    e = hipMemcpyAsync(ctx->d_init.ptr, h_initial, n * sizeof(uint64_t), hipMemcpyHostToDevice, s);
    dinit = (const uint64_t*)ctx->d_init.ptr;
  }
  if (e != hipSuccess) return hip_fail(ctx, e, "H2D");
  e = launch_checksum_batch(mode, flags, (uint8_t*)ctx->d_arena.ptr, (const wgcs_pkt*)ctx->d_pkts.ptr, dinit, n,
                            ctx->d_out.ptr, s, ctx->num_cu, ctx->tune);
  if (e != hipSuccess) return hip_fail(ctx, e, "checksum_batch launch");
  e = hipMemcpyAsync(h_out, ctx->d_out.ptr, out_bytes, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess && (flags & WGCS_F_INPLACE) && arena_len)
    e = hipMemcpyAsync(h_arena, ctx->d_arena.ptr, arena_len, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  return e == hipSuccess ? WGCS_OK : hip_fail(ctx, e, "D2H");
}

// checksum(b, initial), tun/checksum.go:152-167
int wgcs_checksum(wgcs_ctx* ctx, const uint8_t* b, size_t n, uint64_t initial, uint16_t* out) {
  if (!ctx || !out || (!b && n)) return WGCS_ERR_INVALID_ARG;
  if (n >= 0x80000000u) return set_err(ctx, WGCS_ERR_INVALID_ARG, "buffer too large");
  wgcs_pkt p;
  wgcs_pkt_set(&p, 0, (uint32_t)n, 0, 0, 0, 0);
  return wgcs_checksum_batch_host(ctx, WGCS_MODE_FOLD, 0, const_cast<uint8_t*>(b), n, &p, &initial, 1, out);
}

// checksumValid(pkt, iphLen, proto, isV6), tun/gro.go:554-612
// checksumValid(pkt, iphLen, protocol, isV6), tun/gro.go:554-612; pkt[len, cap)
// is the slice's spare capacity, which the address slices (:558-563) reach
// for a packet shorter than its addresses.
int wgcs_checksum_valid_cap(wgcs_ctx* ctx, const uint8_t* pkt, size_t len, size_t cap, uint8_t iph_len, uint8_t proto,
                            int is_v6, int* valid) {
  if (!ctx || !valid || (!pkt && cap) || cap < len) return WGCS_ERR_INVALID_ARG;
  // pkt[srcAddrAt:...+2*addrSize] up to cap, pkt[iphLen:] up to len (gro.go:561-562, :611)
  const size_t need = is_v6 ? 40 : 20;
  if (cap < need || len < iph_len)
    return set_err(ctx, WGCS_ERR_OUT_OF_RANGE, "pkt[%u:] or its addresses past the slice", (unsigned)iph_len);
  if (len >= 0x80000000u) return set_err(ctx, WGCS_ERR_INVALID_ARG, "packet too large");
  wgcs_pkt p;
  wgcs_pkt_set(&p, 0, (uint32_t)len, iph_len, 0, proto, (uint8_t)(is_v6 ? WGCS_PKT_V6 : 0));
  uint8_t v = 0;
  int rc = wgcs_checksum_batch_host(ctx, WGCS_MODE_VALIDATE, 0, const_cast<uint8_t*>(pkt), std::max(len, need), &p,
                                    nullptr, 1, &v);
  *valid = v;
  return rc;
}

int wgcs_checksum_valid(wgcs_ctx* ctx, const uint8_t* pkt, size_t len, uint8_t iph_len, uint8_t proto, int is_v6,
                        int* valid) {
  return wgcs_checksum_valid_cap(ctx, pkt, len, len, iph_len, proto, is_v6, valid);
}

// gsoNoneChecksum(readBuf, csumStart, csumOffset), tun/gro.go:1497-1517
int wgcs_gso_none_checksum(wgcs_ctx* ctx, uint8_t* read_buf, size_t len, uint16_t csum_start, uint16_t csum_offset) {
  if (!ctx || (!read_buf && len)) return WGCS_ERR_INVALID_ARG;
  const uint16_t at = (uint16_t)(csum_start + csum_offset);
  if ((size_t)at + 2 > len || csum_start > len)
    return set_err(ctx, WGCS_ERR_OUT_OF_RANGE, "checksum field %u outside packet of %zu bytes", at, len);
  if (len >= 0x80000000u) return set_err(ctx, WGCS_ERR_INVALID_ARG, "packet too large");
  wgcs_pkt p;
  wgcs_pkt_set(&p, 0, (uint32_t)len, csum_start, csum_offset, 0, 0);
  uint16_t out = 0;
  return wgcs_checksum_batch_host(ctx, WGCS_MODE_PARTIAL, WGCS_F_INPLACE, read_buf, len, &p, nullptr, 1, &out);
}

}  // extern "C"
