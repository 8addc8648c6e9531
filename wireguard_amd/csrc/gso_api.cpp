// gso_api.cpp -- C ABI for the GSO split path (include/wgcsum.h).
//   wgcs_gso_split_batch     device-resident batch (one job per Tun.Read)
//   wgcs_gso_split           gsoSplit()          /root/reference/tun/gro.go:1373-1493
//   wgcs_handle_virtio_read  handleVirtioRead()  /root/reference/tun/tun.go:514-632
// The host-buffer entry points stage the super-packet into HBM, run
// gso_rows_kernel (all validation, header rewriting, payload copies and
// checksums happen there), and copy the produced segments back into the
// caller's buffers.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <mutex>

#include "../../include/wgcsum.h"
#include "wgcs_ctx.h"
#include "wgcs_kernels.h"

using namespace wgcs;

namespace {

struct GsoResult {
  int status = 0;
  int count = 0;
};

// Runs one job through the kernel and copies its segments into bufs.
// vbuf = [10-byte virtio header | packet bytes] in the context's pinned
// staging.  Zero-copy round trip: the kernel reads the job, its descriptor and
// the super-packet straight from pinned host memory over PCIe and writes the
// segments (into a packed region whose size the host bounds from the virtio
// header, gso_out_layout), their sizes, the count and the status straight
// back into pinned host memory -- one launch and one wait, no copy commands.
// The room checks use bufs[0]'s room, as the reference does (tun/tun.go:546,
// gro.go:1406-1410); other buffers are checked when copying, where the Go
// code would panic on the slice.  Caller holds ctx->mu.
// With `ring` the device step goes through the resident ring instead of a
// launch + wait (its own coherent staging; the caller holds the ring's lock).
int run_gso_host(wgcs_ctx* ctx, const uint8_t* vbuf, size_t vlen, uint32_t jflags, uint8_t* const* bufs,
                 const size_t* buf_lens, int nbufs, int* sizes, int offset, GsoResult* res,
                 wgcs_ring* ring = nullptr) {
  if (nbufs < 0 || (nbufs > 0 && (!bufs || !buf_lens || !sizes)) || offset < 0)
    return set_err(ctx, WGCS_ERR_INVALID_ARG, "bufs/sizes/offset");
  if (vlen > 0x7FFFFFF0u) return set_err(ctx, WGCS_ERR_INVALID_ARG, "super-packet too large");
  // len(bufs) == 0: the reference validates and prepares readBuf exactly as
  // usual, then fails at the first bufs access -- gsoSplit's loop returns
  // (i-1 = -1, ErrTooManySegments) before touching bufs[0] (gro.go:1408-1410),
  // handleVirtioRead's GSO_NONE path indexes bufs[0] (a panic: OUT_OF_RANGE),
  // and a split that yields no segment returns (0, nil).  The kernel runs the
  // job against one scratch slot of unbounded room to get that verdict.
  const bool nobuf = nbufs == 0;
  const int kbufs = nobuf ? 1 : nbufs;
  if (!nobuf && buf_lens[0] < (size_t)offset) return set_err(ctx, WGCS_ERR_OUT_OF_RANGE, "offset beyond bufs[0]");
  const size_t room = nobuf ? 0xFFFFFFFFu : std::min<size_t>(buf_lens[0] - (size_t)offset, 0xFFFFFFFFu);
  uint32_t pitch, nseg_bound;
  gso_out_layout(vbuf, vlen, jflags, (uint32_t)kbufs, &pitch, &nseg_bound);
  if (pitch == 0) pitch = 16;
  const bool raw = (jflags & WGCS_GSO_JOB_RAW) != 0;
  const uint8_t gtype = vlen >= 10 ? vbuf[1] : 0;
  // A header geometry whose result involves the caller's bytes beyond the
  // packets (a field past a segment's end, or the IPv4 id update reading
  // bufs[i][4:6], gro.go:1426-1431): the region mirrors each buffer's window
  // -- staged in, written by the kernel with its past-the-end header writes
  // (kOutPosTails), copied back over each segment's whole reach.
  const bool mirror = !nobuf && gso_touches_caller_bytes(vbuf, vlen, jflags);
  if (mirror) pitch = std::max<uint32_t>(pitch, (uint32_t)((gso_field_reach(vbuf, vlen, jflags) + 15) & ~(size_t)15));
  const size_t region = (size_t)pitch * nseg_bound;
  hipSetDevice(ctx->device);
  int rc;
  int32_t* h;
  uint8_t* hs;
  auto stage_mirror = [&]() {
    if (mirror && region) {
      memset(hs, 0, region);
      for (uint32_t i = 0; i < nseg_bound && i < (uint32_t)nbufs; ++i)
        if (buf_lens[i] > (size_t)offset)
          memcpy(hs + (size_t)i * pitch, bufs[i] + offset, std::min<size_t>(pitch, buf_lens[i] - offset));
    }
  };
  bool direct = false;  // ring: segments straight into the caller's buffers
  if (ring) {
    uint8_t* rs = nullptr;
    int32_t* rm = nullptr;
    // ring-readable caller buffers on a fixed stride (one slab of
    // wgcs_host_alloc memory, e.g. a pool of Read buffers), each with room for
    // any segment: the kernel writes segment i at bufs[0] + offset + i * stride
    // itself, byte for byte what the copy below would leave (no header write
    // past a packet: !mirror; no slice too short: room >= pitch)
    const uint32_t nw = std::min<uint32_t>(nseg_bound, (uint32_t)nbufs);
    if (!mirror && !nobuf && nw > 0) {
      const ptrdiff_t stride = nw > 1 ? bufs[1] - bufs[0] : (ptrdiff_t)pitch;
      direct = stride >= (ptrdiff_t)pitch && stride <= 0x7FFFFFFF && (stride & 15) == 0;
      for (uint32_t i = 0; direct && i < nw; ++i)
        direct = bufs[i] == bufs[0] + (ptrdiff_t)i * stride && buf_lens[i] >= (size_t)offset + pitch;
      direct = direct && ring_mapped(ring, bufs[0], (size_t)(nw - 1) * (size_t)stride + (size_t)offset + pitch);
      if (direct) pitch = (uint32_t)stride;
    }
    if ((rc = ring_gso_prepare(ring, (uint32_t)kbufs, direct ? 0 : region, &rs, &rm))) return rc;
    hs = rs;
    h = rm;
    if (!direct) stage_mirror();
    if ((rc = ring_gso(ring, vbuf, (uint32_t)vlen, jflags, (uint32_t)kbufs, pitch, (uint32_t)room,
                       mirror ? kOutPosTails : 0u, direct ? bufs[0] + offset : hs, h)))
      return rc;
  } else {
    const size_t meta = ((size_t)kbufs * 4 + 16 + 15) & ~(size_t)15;  // sizes[kbufs] | count | status
    const size_t aux = sizeof(wgcs_gso_job) + sizeof(GsoOutPos);
    if ((rc = ensure_pinned(ctx, ctx->h_meta, meta + aux)) || (rc = ensure_pinned(ctx, ctx->h_stage, region + 16)))
      return rc;
    hipStream_t s = ctx->stream;
    uint8_t* hm = (uint8_t*)ctx->h_meta.ptr;
    wgcs_gso_job* hjob = (wgcs_gso_job*)(hm + meta);
    GsoOutPos* hpos = (GsoOutPos*)(hjob + 1);
    hjob->off = 0;
    hjob->len = (uint32_t)vlen;
    hjob->flags = jflags;
    hpos->base = 0;
    hpos->pitch = pitch;
    hpos->flags = mirror ? kOutPosTails : 0u;
    h = (int32_t*)hm;
    hs = (uint8_t*)ctx->h_stage.ptr;
    stage_mirror();
    // pinned staging is mapped into the device's address space at its host
    // address (checked by ensure_pinned's hipHostMalloc contract, see api.cpp)
    hipError_t e = launch_gso_split_batch(vbuf, hjob, 1, hs, 0, 0, (uint32_t)kbufs, h, h + kbufs, h + kbufs + 1, s,
                                          hpos, (uint32_t)room);
    if (e != hipSuccess) return hip_fail(ctx, e, "gso_split launch");
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return hip_fail(ctx, e, "gso_split wait");
  }
  res->count = h[kbufs];
  res->status = h[kbufs + 1];
  if (nobuf) {
    const bool none = !raw && gtype == 0;  // handleVirtioRead's GSO_NONE path
    if (res->status == 0 && none) {
      res->status = WGCS_ERR_OUT_OF_RANGE;  // bufs[0] of an empty bufs
      res->count = 0;
    } else if ((res->status == 0 && res->count > 0) || res->status == WGCS_ERR_TOO_MANY_SEGMENTS) {
      res->status = WGCS_ERR_TOO_MANY_SEGMENTS;
      res->count = -1;
    } else if (res->status != 0) {
      res->count = 0;
    }
    return WGCS_OK;
  }
  if (res->status != 0 && res->status != WGCS_ERR_TOO_MANY_SEGMENTS) {
    res->count = 0;
    return WGCS_OK;
  }
  const int written = res->status == WGCS_ERR_TOO_MANY_SEGMENTS ? nbufs : res->count;
  for (int i = 0; i < written; ++i) {
    sizes[i] = h[i];
    const bool last = res->status == 0 && i == written - 1;
    const size_t need = gso_split_need(vbuf, vlen, jflags, (size_t)h[i], last);
    if (buf_lens[i] < (size_t)offset + need) {  // the Go code would panic on this slice
      res->status = WGCS_ERR_OUT_OF_RANGE;
      res->count = i;
      return WGCS_OK;
    }
    if (!direct) memcpy(bufs[i] + offset, hs + (size_t)i * pitch, mirror ? need : (size_t)h[i]);
  }
  return WGCS_OK;
}

// handleVirtioRead's edits of the caller's readBuf after a split (the GPU
// worked on a copy or read it in place without writing it).
void finish_virtio_read(uint8_t* read_buf, size_t n, uint8_t* const* bufs, int offset, const GsoResult& r) {
  if (n >= 10 && (r.status == 0 || r.status == WGCS_ERR_TOO_MANY_SEGMENTS)) {
    uint8_t* rb = read_buf + 10;
    uint16_t cs, co;
    memcpy(&cs, read_buf + 6, 2);
    memcpy(&co, read_buf + 8, 2);
    const size_t at = (uint16_t)(cs + co);
    if (read_buf[1] == 0) {
      // GSO_NONE: gsoNoneChecksum wrote the checksum into readBuf (gro.go:1512-1515)
      if (read_buf[0] & 1) {
        rb[at] = bufs[0][offset + at];
        rb[at + 1] = bufs[0][offset + at + 1];
      }
    } else {
      if ((rb[0] >> 4) == 4) rb[10] = rb[11] = 0;  // gro.go:1388
      rb[at] = rb[at + 1] = 0;                     // gro.go:1393
    }
  }
}

}  // namespace

namespace wgcs {

// The per-call path for one job whose bytes the caller owns (the read stager's
// copy_out for a geometry that touches the caller's buffers).  Takes ctx->mu.
int gso_split_staged(wgcs_ctx* ctx, const uint8_t* vbuf, size_t vlen, uint32_t jflags, uint8_t* const* bufs,
                     const size_t* buf_lens, int nbufs, int* sizes, int offset, int* status, int* count) {
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc;
  if ((rc = ensure_pinned(ctx, ctx->h_out, vlen + 16))) return rc;
  if (vlen) memcpy(ctx->h_out.ptr, vbuf, vlen);
  GsoResult r;
  if ((rc = run_gso_host(ctx, (const uint8_t*)ctx->h_out.ptr, vlen, jflags, bufs, buf_lens, nbufs, sizes, offset, &r)))
    return rc;
  *status = r.status;
  *count = r.count;
  return WGCS_OK;
}

}  // namespace wgcs

extern "C" {

int wgcs_gso_kernel_shape(int* lds_waves, int* parts, int* u, int* rows) {
  wgcs::gso_kernel_shape(lds_waves, parts, u, rows);
  return WGCS_OK;
}

int wgcs_gso_split_batch(wgcs_ctx* ctx, const uint8_t* d_arena, const wgcs_gso_job* d_jobs, uint32_t n_jobs,
                         uint8_t* d_out, uint32_t out_stride, uint32_t offset, uint32_t max_segs, int32_t* d_sizes,
                         int32_t* d_count, int32_t* d_status, void* stream) {
  if (!ctx) return WGCS_ERR_INVALID_ARG;
  if (n_jobs == 0) return WGCS_OK;
  if (!d_arena || !d_jobs || !d_out || !d_sizes || !d_count || !d_status || max_segs == 0)
    return set_err(ctx, WGCS_ERR_INVALID_ARG, "NULL pointer or max_segs == 0");
  std::lock_guard<std::mutex> g(ctx->mu);
  hipSetDevice(ctx->device);
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  if ((uint64_t)n_jobs * max_segs > 0xFFFFFFFFull) return set_err(ctx, WGCS_ERR_INVALID_ARG, "n_jobs*max_segs >= 2^32");
  if (max_segs > 0x7FFFFFFFu) return set_err(ctx, WGCS_ERR_INVALID_ARG, "max_segs >= 2^31 (len(bufs) is a Go int)");
  hipError_t e = launch_gso_split_batch(d_arena, d_jobs, n_jobs, d_out, out_stride, offset, max_segs, d_sizes, d_count,
                                        d_status, s);
  return e == hipSuccess ? WGCS_OK : hip_fail(ctx, e, "gso_split_batch launch");
}

// gsoSplit(readBuf, hdr, bufs, sizes, offset, isV6) (int, error) -- gro.go:1373;
// read_buf[len, cap) is readBuf's spare capacity.
int wgcs_gso_split_cap(wgcs_ctx* ctx, uint8_t* read_buf, size_t len, size_t cap, const wgcs_virtio_hdr* hdr,
                       uint8_t* const* bufs, const size_t* buf_lens, int nbufs, int* sizes, int offset, int is_v6,
                       int* n_out) {
  if (!ctx || !hdr || !n_out || (!read_buf && cap) || cap < len) return WGCS_ERR_INVALID_ARG;
  *n_out = 0;
  const size_t spare = std::min<size_t>(cap - len, 255);
  int rc;
  std::lock_guard<std::mutex> g(ctx->mu);
  if ((rc = ensure_pinned(ctx, ctx->h_out, len + spare + 10))) return rc;
  uint8_t* v = (uint8_t*)ctx->h_out.ptr;
  v[0] = hdr->flags;
  v[1] = hdr->gso_type;
  memcpy(v + 2, &hdr->hdr_len, 2);
  memcpy(v + 4, &hdr->gso_size, 2);
  memcpy(v + 6, &hdr->csum_start, 2);
  memcpy(v + 8, &hdr->csum_offset, 2);
  if (len + spare) memcpy(v + 10, read_buf, len + spare);
  GsoResult r;
  rc = run_gso_host(ctx, v, len + 10,
                    WGCS_GSO_JOB_RAW | (is_v6 ? WGCS_GSO_JOB_V6 : 0u) | WGCS_GSO_JOB_SPARE(spare), bufs, buf_lens,
                    nbufs, sizes, offset, &r);
  if (rc) return rc;
  if (r.status == 0 || r.status == WGCS_ERR_TOO_MANY_SEGMENTS) {
    // the reference zeroes these fields of readBuf before splitting (gro.go:1388,:1393)
    if (!is_v6) read_buf[10] = read_buf[11] = 0;
    const size_t at = (uint16_t)(hdr->csum_start + hdr->csum_offset);
    read_buf[at] = read_buf[at + 1] = 0;
  }
  *n_out = r.count;
  return r.status;
}

int wgcs_gso_split(wgcs_ctx* ctx, uint8_t* read_buf, size_t len, const wgcs_virtio_hdr* hdr, uint8_t* const* bufs,
                   const size_t* buf_lens, int nbufs, int* sizes, int offset, int is_v6, int* n_out) {
  return wgcs_gso_split_cap(ctx, read_buf, len, len, hdr, bufs, buf_lens, nbufs, sizes, offset, is_v6, n_out);
}

// handleVirtioRead(readBuf, bufs, sizes, offset) (int, error) -- tun/tun.go:514;
// read_buf[n, cap) is readBuf's spare capacity (Tun.Read passes tun.readBuf[:n]).
int wgcs_handle_virtio_read_cap(wgcs_ctx* ctx, uint8_t* read_buf, size_t n, size_t cap, uint8_t* const* bufs,
                                const size_t* buf_lens, int nbufs, int* sizes, int offset, int* n_out) {
  if (!ctx || !n_out || (!read_buf && cap) || cap < n) return WGCS_ERR_INVALID_ARG;
  *n_out = 0;
  const size_t spare = std::min<size_t>(cap - n, 255);
  GsoResult r;
  std::lock_guard<std::mutex> g(ctx->mu);
  int rc;
  if ((rc = ensure_pinned(ctx, ctx->h_out, n + spare + 16))) return rc;
  if (n + spare) memcpy(ctx->h_out.ptr, read_buf, n + spare);  // the kernel reads it from pinned memory
  rc = run_gso_host(ctx, (const uint8_t*)ctx->h_out.ptr, n, WGCS_GSO_JOB_SPARE(spare), bufs, buf_lens, nbufs, sizes,
                    offset, &r);
  if (rc) return rc;
  finish_virtio_read(read_buf, n, bufs, offset, r);
  *n_out = r.count;
  return r.status;
}

int wgcs_handle_virtio_read(wgcs_ctx* ctx, uint8_t* read_buf, size_t n, uint8_t* const* bufs, const size_t* buf_lens,
                            int nbufs, int* sizes, int offset, int* n_out) {
  return wgcs_handle_virtio_read_cap(ctx, read_buf, n, n, bufs, buf_lens, nbufs, sizes, offset, n_out);
}

// handleVirtioRead through the resident ring (ring.cpp): the same arguments,
// bytes and errors as wgcs_handle_virtio_read_cap.
int wgcs_ring_handle_virtio_read_cap(wgcs_ring* ring, uint8_t* read_buf, size_t n, size_t cap, uint8_t* const* bufs,
                                     const size_t* buf_lens, int nbufs, int* sizes, int offset, int* n_out) {
  if (!ring || !n_out || (!read_buf && cap) || cap < n) return WGCS_ERR_INVALID_ARG;
  *n_out = 0;
  wgcs_ctx* ctx = ring_ctx(ring);
  const size_t spare = std::min<size_t>(cap - n, 255);
  GsoResult r;
  std::lock_guard<std::mutex> g(ring_mutex(ring));
  const uint8_t* vbuf = nullptr;
  int rc = ring_input(ring, read_buf, n + spare, &vbuf);
  if (rc) return rc;
  rc = run_gso_host(ctx, vbuf, n, WGCS_GSO_JOB_SPARE(spare), bufs, buf_lens, nbufs, sizes, offset, &r, ring);
  if (rc) return rc;
  finish_virtio_read(read_buf, n, bufs, offset, r);
  *n_out = r.count;
  return r.status;
}

int wgcs_ring_handle_virtio_read(wgcs_ring* ring, uint8_t* read_buf, size_t n, uint8_t* const* bufs,
                                 const size_t* buf_lens, int nbufs, int* sizes, int offset, int* n_out) {
  return wgcs_ring_handle_virtio_read_cap(ring, read_buf, n, n, bufs, buf_lens, nbufs, sizes, offset, n_out);
}

}  // extern "C"
