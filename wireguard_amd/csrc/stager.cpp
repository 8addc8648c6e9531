// stager.cpp -- Tun.Read batch staging.
//
// The reference reads one super-packet per Tun.Read call and splits it on the
// CPU (tun/tun.go:477-508 -> handleVirtioRead :514-632).  A GPU only pays off
// on large batches, so the stager collects many reads into a pinned ring slot
// and runs them as one gso_rows_kernel launch:
//
//   push / reserve+commit   read bytes -> pinned slot (read(2) can target it)
//   submit                  slot stream: H2D in+jobs+layout -> split kernel
//                           -> D2H of sizes/counts/statuses + the packed output
//   wait / result / copy_out
//
// `depth` slots rotate, each with its own stream, so batch k's D2H, batch
// k+1's kernel and batch k+2's H2D overlap.  The output of a batch is packed:
// read r's segments sit at base_r + i*pitch_r, where the host derives a pitch
// that holds any segment the kernel may produce from the 10-byte virtio header
// (min(read, header bound + gsoSize), or the whole packet for GSO_NONE), so
// the D2H moves about the produced bytes instead of
// max_segs fixed-size slots per read.  The handleVirtioRead room checks use
// the caller's buffer room (seg_room), exactly as with bufs[i][offset:].
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/wgcsum.h"
#include "wgcs_ctx.h"
#include "wgcs_kernels.h"

using namespace wgcs;

namespace {

size_t align16(size_t x) { return (x + 15) & ~size_t(15); }

struct Slot {
  uint64_t id = 0;
  int state = 0;  // 0 free (results of `id` readable once done), 1 open, 2 submitted
  uint32_t n_reads = 0;
  size_t used_in = 0, used_out = 0;
  int reserved = -1;
  size_t reserved_max = 0;
  size_t carry = 0;  // committed read (bytes at h_in + used_in) whose output region did not fit: moved by submit
  // pinned host
  uint8_t* h_in = nullptr;
  wgcs_gso_job* h_jobs = nullptr;
  GsoOutPos* h_pos = nullptr;
  uint8_t* h_out = nullptr;
  int32_t* h_meta = nullptr;  // sizes[max_reads*max_segs] | count[max_reads] | status[max_reads]
  // device
  uint8_t* d_in = nullptr;
  wgcs_gso_job* d_jobs = nullptr;
  GsoOutPos* d_pos = nullptr;
  uint8_t* d_out = nullptr;
  int32_t* d_meta = nullptr;
  hipStream_t stream = nullptr;
  hipEvent_t done = nullptr;
};

}  // namespace

struct wgcs_stager {
  wgcs_ctx* ctx = nullptr;
  uint32_t depth = 0, max_reads = 0, max_segs = 0, seg_room = 0;
  size_t max_in = 0, max_out = 0;
  std::vector<Slot> slots;
  uint32_t open = 0;
  uint64_t next_id = 1;
  bool broken = false;  // a ring slot could not be opened (HIP error): every later call fails
  std::mutex mu;

  size_t meta_words() const { return (size_t)max_reads * max_segs + 2 * (size_t)max_reads; }
  Slot* find(uint64_t id) {
    for (auto& s : slots)
      if (s.id == id && id != 0) return &s;
    return nullptr;
  }
};

namespace {

void free_slot(Slot& s) {
  if (s.h_in) hipHostFree(s.h_in);
  if (s.h_jobs) hipHostFree(s.h_jobs);
  if (s.h_pos) hipHostFree(s.h_pos);
  if (s.h_out) hipHostFree(s.h_out);
  if (s.h_meta) hipHostFree(s.h_meta);
  if (s.d_in) hipFree(s.d_in);
  if (s.d_jobs) hipFree(s.d_jobs);
  if (s.d_pos) hipFree(s.d_pos);
  if (s.d_out) hipFree(s.d_out);
  if (s.d_meta) hipFree(s.d_meta);
  if (s.done) hipEventDestroy(s.done);
  if (s.stream) hipStreamDestroy(s.stream);
  s = Slot();
}

// Open slot `idx` for a new batch, waiting for its previous batch if needed.
int open_slot(wgcs_stager* st, uint32_t idx) {
  Slot& s = st->slots[idx];
  if (s.state == 2) {
    hipError_t e = hipEventSynchronize(s.done);
    if (e != hipSuccess) {
      st->broken = true;  // st->open still names the submitted slot: nothing may be staged into it
      return hip_fail(st->ctx, e, "stager: wait for ring slot (stager unusable)");
    }
  }
  s.id = st->next_id++;
  s.state = 1;
  s.n_reads = 0;
  s.used_in = s.used_out = 0;
  s.reserved = -1;
  s.carry = 0;
  st->open = idx;
  return WGCS_OK;
}

int stage(wgcs_stager* st, size_t max_n, uint8_t** dst, int* read_idx) {
  if (st->broken) return set_err(st->ctx, WGCS_ERR_HIP, "stager unusable after a HIP error");
  Slot& s = st->slots[st->open];
  if (s.reserved >= 0) return set_err(st->ctx, WGCS_ERR_INVALID_ARG, "stager: commit the open reservation first");
  if (s.carry) return set_err(st->ctx, WGCS_ERR_BATCH_FULL, "stager: a committed read waits for submit");
  if (max_n > 0x7FFFFFF0u) return set_err(st->ctx, WGCS_ERR_INVALID_ARG, "read too large");
  if (s.n_reads >= st->max_reads || s.used_in + align16(max_n) > st->max_in)
    return set_err(st->ctx, WGCS_ERR_BATCH_FULL, "stager: open batch is full");
  *dst = s.h_in + s.used_in;
  *read_idx = (int)s.n_reads;
  return WGCS_OK;
}

int finish(wgcs_stager* st, size_t n) {
  Slot& s = st->slots[st->open];
  uint32_t pitch, segs;
  gso_out_layout(s.h_in + s.used_in, n, 0, st->max_segs, &pitch, &segs);
  const size_t region = (size_t)pitch * segs;
  if (s.used_out + region > st->max_out)
    return set_err(st->ctx, WGCS_ERR_BATCH_FULL, "stager: output region of the open batch is full");
  const uint32_t r = s.n_reads;
  s.h_jobs[r].off = s.used_in;
  s.h_jobs[r].len = (uint32_t)n;
  s.h_jobs[r].flags = 0;
  s.h_pos[r].base = s.used_out;
  s.h_pos[r].pitch = pitch ? pitch : 16;
  s.h_pos[r].flags = 0;  // packets only: copy_out applies the rest
  s.used_in += align16(n);
  s.used_out += region;
  s.n_reads++;
  return WGCS_OK;
}

}  // namespace

extern "C" {

int wgcs_stager_create(wgcs_ctx* ctx, uint32_t depth, uint32_t max_reads, size_t max_bytes, uint32_t max_segs,
                       uint32_t seg_room, wgcs_stager** out) {
  if (!ctx || !out || depth < 2 || depth > 64 || max_reads == 0 || max_segs == 0 || max_bytes == 0 ||
      seg_room == 0)
    return WGCS_ERR_INVALID_ARG;
  if ((uint64_t)max_reads * max_segs > 0x7FFFFFFFull) return set_err(ctx, WGCS_ERR_INVALID_ARG, "max_reads*max_segs");
  *out = nullptr;
  auto* st = new (std::nothrow) wgcs_stager();
  if (!st) return WGCS_ERR_NOMEM;
  st->ctx = ctx;
  st->depth = depth;
  st->max_reads = max_reads;
  st->max_segs = max_segs;
  st->seg_room = seg_room;
  st->max_in = align16(max_bytes);
  // a read's region is its segment bound x (gsoSize + 240): about 1.2x the
  // read at MSS 1460, more for small MSS; a full region returns BATCH_FULL
  st->max_out = align16(2 * max_bytes + (size_t)max_reads * 16384);
  st->slots.resize(depth);
  hipSetDevice(ctx->device);
  for (auto& s : st->slots) {
    hipError_t e = hipSuccess;
    const size_t meta = st->meta_words() * sizeof(int32_t);
    if (e == hipSuccess) e = hipHostMalloc((void**)&s.h_in, st->max_in + 64, hipHostMallocDefault);
    if (e == hipSuccess) e = hipHostMalloc((void**)&s.h_jobs, max_reads * sizeof(wgcs_gso_job), hipHostMallocDefault);
    if (e == hipSuccess) e = hipHostMalloc((void**)&s.h_pos, max_reads * sizeof(GsoOutPos), hipHostMallocDefault);
    if (e == hipSuccess) e = hipHostMalloc((void**)&s.h_out, st->max_out + 64, hipHostMallocDefault);
    if (e == hipSuccess) e = hipHostMalloc((void**)&s.h_meta, meta, hipHostMallocDefault);
    if (e == hipSuccess) e = hipMalloc((void**)&s.d_in, st->max_in + 64);
    if (e == hipSuccess) e = hipMalloc((void**)&s.d_jobs, max_reads * sizeof(wgcs_gso_job));
    if (e == hipSuccess) e = hipMalloc((void**)&s.d_pos, max_reads * sizeof(GsoOutPos));
    if (e == hipSuccess) e = hipMalloc((void**)&s.d_out, st->max_out + 64);
    if (e == hipSuccess) e = hipMalloc((void**)&s.d_meta, meta);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&s.done, hipEventDisableTiming);
    if (e != hipSuccess) {
      const int rc = hip_fail(ctx, e, "stager allocation");
      for (auto& t : st->slots) free_slot(t);
      delete st;
      return rc;
    }
  }
  const int rc = open_slot(st, 0);
  if (rc) {
    wgcs_stager_destroy(st);
    return rc;
  }
  {
    std::lock_guard<std::mutex> g(ctx->host_mu);
    ctx->stagers.push_back(st);
  }
  *out = st;
  return WGCS_OK;
}

int wgcs_stager_destroy(wgcs_stager* st) {
  if (!st) return WGCS_ERR_INVALID_ARG;
  {
    std::lock_guard<std::mutex> g(st->ctx->host_mu);
    auto& v = st->ctx->stagers;
    v.erase(std::remove(v.begin(), v.end(), st), v.end());
  }
  hipSetDevice(st->ctx->device);
  for (auto& s : st->slots) {
    if (s.state == 2) hipEventSynchronize(s.done);
    free_slot(s);
  }
  delete st;
  return WGCS_OK;
}

int wgcs_stager_push(wgcs_stager* st, const uint8_t* read_buf, size_t n, int* read_idx) {
  if (!st || !read_idx || (!read_buf && n)) return WGCS_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(st->mu);
  uint8_t* dst;
  int rc = stage(st, n, &dst, read_idx);
  if (rc) return rc;
  if (n) memcpy(dst, read_buf, n);
  return finish(st, n);
}

int wgcs_stager_push_many(wgcs_stager* st, const uint8_t* const* read_bufs, const size_t* ns, int count,
                          int* first_idx, int* pushed) {
  if (!st || !read_bufs || !ns || !first_idx || !pushed || count < 0) return WGCS_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(st->mu);
  *pushed = 0;
  *first_idx = (int)st->slots[st->open].n_reads;
  for (int k = 0; k < count; ++k) {
    if (!read_bufs[k] && ns[k]) return WGCS_ERR_INVALID_ARG;
    uint8_t* dst;
    int idx;
    int rc = stage(st, ns[k], &dst, &idx);
    if (rc) return rc;
    if (ns[k]) memcpy(dst, read_bufs[k], ns[k]);
    if ((rc = finish(st, ns[k]))) return rc;
    ++*pushed;
  }
  return WGCS_OK;
}

int wgcs_stager_reserve(wgcs_stager* st, size_t max_n, uint8_t** dst, int* read_idx) {
  if (!st || !dst || !read_idx) return WGCS_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(st->mu);
  int rc = stage(st, max_n, dst, read_idx);
  if (rc) return rc;
  Slot& s = st->slots[st->open];
  s.reserved = *read_idx;
  s.reserved_max = max_n;
  return WGCS_OK;
}

int wgcs_stager_commit(wgcs_stager* st, int read_idx, size_t n) {
  if (!st) return WGCS_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(st->mu);
  Slot& s = st->slots[st->open];
  if (s.reserved < 0 || read_idx != s.reserved || n > s.reserved_max)
    return set_err(st->ctx, WGCS_ERR_INVALID_ARG, "stager: commit without a matching reservation");
  s.reserved = -1;
  if (n == 0) return WGCS_OK;  // nothing read: the reservation is dropped
  const int rc = finish(st, n);
  if (rc == WGCS_ERR_BATCH_FULL) {
    if (s.n_reads == 0) return set_err(st->ctx, WGCS_ERR_INVALID_ARG, "stager: one read's output exceeds max_out");
    // the bytes read(2) put into the slot stay: submit() queues this batch
    // without them and carries them into the next one (no read is lost)
    s.carry = n;
  }
  return rc;
}

int wgcs_stager_submit(wgcs_stager* st, uint64_t* batch) {
  if (!st || !batch) return WGCS_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(st->mu);
  if (st->broken) return set_err(st->ctx, WGCS_ERR_HIP, "stager unusable after a HIP error");
  hipSetDevice(st->ctx->device);
  Slot& s = st->slots[st->open];
  if (s.reserved >= 0) return set_err(st->ctx, WGCS_ERR_INVALID_ARG, "stager: open reservation");
  const hipStream_t q = s.stream;
  const size_t nm = st->meta_words() * sizeof(int32_t);
  hipError_t e = hipSuccess;
  if (s.n_reads > 0) {
    e = hipMemcpyAsync(s.d_in, s.h_in, s.used_in, hipMemcpyHostToDevice, q);
    if (e == hipSuccess)
      e = hipMemcpyAsync(s.d_jobs, s.h_jobs, s.n_reads * sizeof(wgcs_gso_job), hipMemcpyHostToDevice, q);
    if (e == hipSuccess)
      e = hipMemcpyAsync(s.d_pos, s.h_pos, s.n_reads * sizeof(GsoOutPos), hipMemcpyHostToDevice, q);
    if (e == hipSuccess)
      e = launch_gso_split_batch(s.d_in, s.d_jobs, s.n_reads, s.d_out, 0, 0, st->max_segs, s.d_meta,
                                 s.d_meta + (size_t)st->max_reads * st->max_segs,
                                 s.d_meta + (size_t)st->max_reads * st->max_segs + st->max_reads, q, s.d_pos,
                                 st->seg_room);
    if (e == hipSuccess) e = hipMemcpyAsync(s.h_meta, s.d_meta, nm, hipMemcpyDeviceToHost, q);
    if (e == hipSuccess && s.used_out)
      e = hipMemcpyAsync(s.h_out, s.d_out, s.used_out, hipMemcpyDeviceToHost, q);
  }
  if (e == hipSuccess) e = hipEventRecord(s.done, q);
  if (e != hipSuccess) return hip_fail(st->ctx, e, "stager submit");
  s.state = 2;
  *batch = s.id;
  const size_t carry = s.carry;
  const uint8_t* carry_src = s.h_in + s.used_in;  // not part of this batch's H2D
  int rc = open_slot(st, (st->open + 1) % st->depth);
  if (rc && carry)  // the batch went out without the carried read, and no slot is open to take it
    return set_err(st->ctx, rc, "stager: ring slot not reopened (HIP error): the read committed with "
                                "BATCH_FULL (%zu bytes) was NOT staged; the stager is unusable", carry);
  if (rc || !carry) return rc;
  Slot& t = st->slots[st->open];
  memcpy(t.h_in, carry_src, carry);
  rc = finish(st, carry);  // read 0 of the new batch
  return rc == WGCS_ERR_BATCH_FULL ? set_err(st->ctx, WGCS_ERR_INVALID_ARG, "stager: one read's output exceeds max_out")
                                   : rc;
}

int wgcs_stager_wait(wgcs_stager* st, uint64_t batch) {
  if (!st) return WGCS_ERR_INVALID_ARG;
  Slot* s;
  hipEvent_t ev;
  {
    std::lock_guard<std::mutex> g(st->mu);
    s = st->find(batch);
    if (!s || s->state == 1) return WGCS_ERR_NOT_READY;
    ev = s->done;
  }
  hipError_t e = hipEventSynchronize(ev);
  return e == hipSuccess ? WGCS_OK : hip_fail(st->ctx, e, "stager wait");
}

int wgcs_stager_result(wgcs_stager* st, uint64_t batch, int read_idx, int* status, int* n, const int32_t** sizes,
                       const uint8_t** segs) {
  if (!st || !status || !n) return WGCS_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(st->mu);
  Slot* s = st->find(batch);
  if (!s || s->state == 1 || hipEventQuery(s->done) != hipSuccess) return WGCS_ERR_NOT_READY;
  if (read_idx < 0 || (uint32_t)read_idx >= s->n_reads) return WGCS_ERR_INVALID_ARG;
  const int32_t* cnt = s->h_meta + (size_t)st->max_reads * st->max_segs;
  *n = cnt[read_idx];
  *status = cnt[st->max_reads + read_idx];
  if (sizes) *sizes = s->h_meta + (size_t)read_idx * st->max_segs;
  if (segs) *segs = s->h_out + s->h_pos[read_idx].base;
  return WGCS_OK;
}

int wgcs_stager_copy_out(wgcs_stager* st, uint64_t batch, int read_idx, uint8_t* const* bufs,
                         const size_t* buf_lens, int nbufs, int* sizes, int offset, int* n_out) {
  if (!st || !bufs || !buf_lens || !sizes || !n_out || offset < 0) return WGCS_ERR_INVALID_ARG;
  if ((uint32_t)nbufs != st->max_segs)
    return set_err(st->ctx, WGCS_ERR_INVALID_ARG, "copy_out: nbufs must equal the stager's max_segs");
  *n_out = 0;
  std::unique_lock<std::mutex> g(st->mu);  // the slot cannot be recycled while its results are copied
  Slot* s = st->find(batch);
  if (!s || s->state == 1 || hipEventQuery(s->done) != hipSuccess) return WGCS_ERR_NOT_READY;
  if (read_idx < 0 || (uint32_t)read_idx >= s->n_reads) return WGCS_ERR_INVALID_ARG;
  const int32_t* cnt = s->h_meta + (size_t)st->max_reads * st->max_segs;
  const int n = cnt[read_idx];
  const int status = cnt[st->max_reads + read_idx];
  if (status != 0 && status != WGCS_ERR_TOO_MANY_SEGMENTS) return status;
  const int32_t* sz = s->h_meta + (size_t)read_idx * st->max_segs;
  const uint8_t* seg = s->h_out + s->h_pos[read_idx].base;
  const uint32_t pitch = s->h_pos[read_idx].pitch;
  const uint8_t* vb = s->h_in + s->h_jobs[read_idx].off;
  const size_t vlen = s->h_jobs[read_idx].len;
  if (gso_touches_caller_bytes(vb, vlen, 0)) {
    // A header geometry whose result involves the caller's buffers beyond the
    // packets (a field past a segment's end, or the IPv4 id update reading
    // bufs[i][4:6]): the batch kernel wrote the packets only; the read runs
    // again on the GPU through the per-call path, with these buffers staged.
    // That is a synchronous round trip: it runs on a copy of the read, with
    // the stager unlocked, so submit / wait / result calls are not held up
    // behind it.
    std::vector<uint8_t> read(vb, vb + vlen);
    g.unlock();
    int st2 = 0, n2 = 0;
    const int rc = gso_split_staged(st->ctx, read.data(), vlen, 0, bufs, buf_lens, nbufs, sizes, offset, &st2, &n2);
    if (rc) return rc;
    *n_out = n2;
    return st2;
  }
  const int written = status == WGCS_ERR_TOO_MANY_SEGMENTS ? nbufs : n;
  for (int i = 0; i < written; ++i) {
    sizes[i] = sz[i];
    const bool last = status == 0 && i == written - 1;
    if (buf_lens[i] < (size_t)offset + gso_split_need(vb, vlen, 0, (size_t)sz[i], last)) {
      *n_out = i;  // the Go code would panic on this slice
      return WGCS_ERR_OUT_OF_RANGE;
    }
    memcpy(bufs[i] + offset, seg + (size_t)i * pitch, (size_t)sz[i]);
  }
  *n_out = n;
  return status;
}

}  // extern "C"
