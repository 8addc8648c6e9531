// udp_msgs_api.cpp -- C ABI of the outer-UDP message batching path
// (include/wgcsum.h):
//   wgcs_get_gso_size / wgcs_set_gso_size   getGSOSize / setGSOSize   conn/gso.go:35-100
//   wgcs_split_messages_batch               splitMessages, device-resident batches  conn/bind.go:542-597
//   wgcs_coalesce_messages_batch            coalesceMessages, device-resident       conn/bind.go:599-662
//   wgcs_split_messages / wgcs_coalesce_messages   the same at Go-call granularity (host buffers)
// The cmsg helpers only parse / build the few-byte control messages (host
// data the GPU never sees); every payload byte moves in udp_msgs_kernels.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <vector>

#include "../../include/wgcsum.h"
#include "wgcs_ctx.h"
#include "wgcs_kernels.h"

using namespace wgcs;

namespace {

// golang.org/x/sys/unix (linux/amd64): SizeofCmsghdr 16, 8-byte cmsg alignment.
constexpr size_t kCmsgHdr = 16;
inline size_t cmsg_align(size_t n) { return (n + 7) & ~size_t(7); }
constexpr int kSolUdp = 17, kUdpSegment = 103, kUdpGro = 104;  // linux/udp.h:35-36
constexpr size_t kSlot = 65536;                                 // staging slot >= MaxMessageSize

inline size_t align16(size_t n) { return (n + 15) & ~size_t(15); }

int parse_gso(const uint8_t* control, size_t len, int* gso) {
  *gso = 0;
  size_t off = 0, rlen = len;
  while (rlen > kCmsgHdr) {  // conn/gso.go:42 (strictly greater)
    uint64_t hlen;
    int32_t level, type;
    memcpy(&hlen, control + off, 8);
    memcpy(&level, control + off + 8, 4);
    memcpy(&type, control + off + 12, 4);
    if (hlen < kCmsgHdr || hlen > rlen) return WGCS_ERR_CMSG;  // ParseOneSocketControlMessage EINVAL
    if (level == kSolUdp && type == kUdpGro && hlen - kCmsgHdr >= 2) {  // :55-64
      uint16_t g;
      memcpy(&g, control + off + kCmsgHdr, 2);
      *gso = g;
      return WGCS_OK;
    }
    const size_t adv = cmsg_align((size_t)hlen);
    if (adv < rlen) {
      off += adv;
      rlen -= adv;
    } else {
      rlen = 0;
    }
  }
  return WGCS_OK;
}

void put_gso(uint8_t* control, size_t* len, size_t cap, uint16_t gso) {
  const size_t space = kCmsgHdr + cmsg_align(2);  // CmsgSpace(2)
  if (*len > cap || space > cap - *len) return;    // conn/gso.go:78-81
  uint8_t* c = control + *len;
  *len += space;
  const uint64_t hl = kCmsgHdr + 2;  // CmsgLen(2)
  const int32_t level = kSolUdp, type = kUdpSegment;
  memcpy(c, &hl, 8);
  memcpy(c + 8, &level, 4);
  memcpy(c + 12, &type, 4);
  memcpy(c + kCmsgHdr, &gso, 2);
}

}  // namespace

extern "C" {

int wgcs_get_gso_size(const uint8_t* control, size_t len, int* gso_size) {
  if (!gso_size || (!control && len)) return WGCS_ERR_INVALID_ARG;
  return parse_gso(control, len, gso_size);
}

int wgcs_set_gso_size(uint8_t* control, size_t* len, size_t cap, uint16_t gso_size) {
  if (!len || (!control && cap)) return WGCS_ERR_INVALID_ARG;
  put_gso(control, len, cap, gso_size);
  return WGCS_OK;
}

int wgcs_split_messages_batch(wgcs_ctx* ctx, const uint8_t* d_in, uint64_t in_stride, uint32_t buf_len,
                              const int32_t* d_n_in, const int32_t* d_gso, uint32_t n_msgs, uint32_t first_msg_at,
                              uint32_t n_batches, uint8_t* d_out, uint64_t out_stride, int32_t* d_n_out,
                              int32_t* d_src, int32_t* d_count, int32_t* d_status, void* stream) {
  if (!ctx) return WGCS_ERR_INVALID_ARG;
  if (n_batches == 0 || n_msgs == 0) return WGCS_OK;
  if (!d_in || !d_n_in || !d_gso || !d_out || !d_n_out || !d_src || !d_count || !d_status)
    return set_err(ctx, WGCS_ERR_INVALID_ARG, "NULL pointer");
  if (first_msg_at > n_msgs || n_msgs - first_msg_at > 128 || buf_len > 0x7FFFFFFFu || (out_stride & 15) ||
      ((uintptr_t)d_out & 15))
    return set_err(ctx, WGCS_ERR_INVALID_ARG, "first_msg_at (<= 128 sources) / buf_len / 16-byte aligned output slots");
  std::lock_guard<std::mutex> g(ctx->mu);
  hipSetDevice(ctx->device);
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  hipError_t e = launch_udp_split(d_in, in_stride, buf_len, d_n_in, d_gso, n_msgs, first_msg_at, n_batches, d_out,
                                  out_stride, d_n_out, d_src, d_count, d_status, s);
  return e == hipSuccess ? WGCS_OK : hip_fail(ctx, e, "split_messages launch");
}

int wgcs_coalesce_messages_batch(wgcs_ctx* ctx, uint8_t* d_bufs, uint64_t buf_stride, uint32_t buf_cap,
                                 const int32_t* d_caps, const int32_t* d_lens, const int32_t* d_nbufs,
                                 uint32_t max_bufs, uint32_t n_batches, int dst_is_v6, int32_t* d_n_msgs,
                                 int32_t* d_msg_first, int32_t* d_msg_len, int32_t* d_msg_gso, void* stream) {
  if (!ctx) return WGCS_ERR_INVALID_ARG;
  if (n_batches == 0 || max_bufs == 0) return WGCS_OK;
  if (!d_bufs || !d_lens || !d_nbufs || !d_n_msgs || !d_msg_first || !d_msg_len || !d_msg_gso)
    return set_err(ctx, WGCS_ERR_INVALID_ARG, "NULL pointer");
  if ((buf_stride & 15) || ((uintptr_t)d_bufs & 15) || buf_cap > buf_stride || buf_cap > 0x7FFFFFFFu)
    return set_err(ctx, WGCS_ERR_INVALID_ARG, "16-byte aligned slots with buf_cap <= buf_stride required");
  std::lock_guard<std::mutex> g(ctx->mu);
  hipSetDevice(ctx->device);
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  hipError_t e = launch_udp_coalesce(d_bufs, buf_stride, buf_cap, d_caps, d_lens, d_nbufs, max_bufs, n_batches,
                                     dst_is_v6, d_n_msgs, d_msg_first, d_msg_len, d_msg_gso, s);
  return e == hipSuccess ? WGCS_OK : hip_fail(ctx, e, "coalesce_messages launch");
}

// splitMessages(msgs, firstMsgAt) (nPackets, err) -- conn/bind.go:542-597.
// One round trip: the source messages are staged in pinned memory, the packets
// land in a packed pinned region whose pitch (the largest packet) the host
// knows from the (N, gsoSize) pairs; the kernel reads and writes both over PCIe.
int wgcs_split_messages(wgcs_ctx* ctx, uint8_t* const* bufs, size_t buf_len, int* ns, const uint8_t* const* oobs,
                        const size_t* nns, int n_msgs, int first_msg_at, int* addr_src, int* n_packets) {
  if (!ctx || !n_packets) return WGCS_ERR_INVALID_ARG;
  *n_packets = 0;
  // every message keeps its own Addr unless the split moves one (bind.go:570):
  // set before any early return, so an error never leaves addr_src unwritten
  if (addr_src)
    for (int k = 0; k < n_msgs; ++k) addr_src[k] = k;
  if (n_msgs <= 0 || !bufs || !ns || !addr_src || first_msg_at < 0 || first_msg_at > n_msgs ||
      n_msgs - first_msg_at > 128 ||
      buf_len > 0x7FFFFFFFu || (!oobs && first_msg_at < n_msgs) || (!nns && first_msg_at < n_msgs))
    return set_err(ctx, WGCS_ERR_INVALID_ARG, "bufs/ns/oobs/first_msg_at");
  const int nsrc = n_msgs - first_msg_at;
  std::vector<int32_t> gso(n_msgs, 0);
  size_t ext = 16, seg = 16;
  uint64_t total_pk = 0;
  for (int t = 0; t < nsrc; ++t) {
    const int i = first_msg_at + t;
    // N outside [0, buf_len] is reported by the kernel (WGCS_ERR_INVALID_ARG) only if the loop reaches it
    int gs = 0;
    const int rc = parse_gso(oobs[i], nns[i], &gs);
    gso[i] = rc ? rc : gs;
    const size_t g = rc ? 0 : (size_t)gs;
    const size_t n = (size_t)std::max(ns[i], 0);
    ext = std::max(ext, std::min(std::max(n, g), buf_len));  // packet 0 reads [0, gsoSize) even past N
    seg = std::max(seg, std::min(g ? g : n, buf_len));
    total_pk += g ? (n + g - 1) / g : 1;
  }
  const size_t in_stride = align16(ext), out_stride = align16(seg);
  const size_t n_out_slots = (size_t)std::min<uint64_t>((uint64_t)n_msgs, total_pk);
  const size_t in_bytes = (size_t)nsrc * in_stride, out_bytes = n_out_slots * out_stride;
  const size_t meta = (size_t)n_msgs * 4 * 4 + 16;  // n_in | gso | n_out | src | count | status
  std::lock_guard<std::mutex> g(ctx->mu);
  hipSetDevice(ctx->device);
  int rc;
  // zero-copy: the kernel reads the messages and writes the packets through
  // pinned staging over PCIe (one launch, one wait, no copy commands)
  if ((rc = ensure_pinned(ctx, ctx->h_stage, in_bytes + 16)) || (rc = ensure_pinned(ctx, ctx->h_out, out_bytes + 16)) ||
      (rc = ensure_pinned(ctx, ctx->h_meta, meta)))
    return rc;
  uint8_t* hs = (uint8_t*)ctx->h_stage.ptr;
  uint8_t* ho = (uint8_t*)ctx->h_out.ptr;
  for (int t = 0; t < nsrc; ++t) {
    const int i = first_msg_at + t;
    const size_t n = (size_t)std::max(ns[i], 0), gs = gso[i] > 0 ? (size_t)gso[i] : 0;
    const size_t want = std::min(std::max(n, gs), buf_len);
    if (want) memcpy(hs + (size_t)t * in_stride, bufs[i], want);
  }
  int32_t* hm = (int32_t*)ctx->h_meta.ptr;
  for (int i = 0; i < n_msgs; ++i) {
    hm[i] = ns[i];
    hm[n_msgs + i] = gso[i];
  }
  hipStream_t s = ctx->stream;
  int32_t* h_nout = hm + 2 * n_msgs;
  int32_t* h_src = hm + 3 * n_msgs;
  int32_t* h_cs = hm + 4 * n_msgs;  // count, status
  hipError_t e = launch_udp_split(hs, in_stride, (uint32_t)buf_len, hm, hm + n_msgs, (uint32_t)n_msgs,
                                  (uint32_t)first_msg_at, 1, ho, out_stride, h_nout, h_src, h_cs, h_cs + 1, s);
  if (e != hipSuccess) return hip_fail(ctx, e, "split_messages launch");
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return hip_fail(ctx, e, "split_messages wait");
  const int count = hm[4 * n_msgs], status = hm[4 * n_msgs + 1];
  for (int k = 0; k < n_msgs; ++k) {
    const int nk = hm[2 * n_msgs + k];
    if (k < count) {
      memcpy(bufs[k], ho + (size_t)k * out_stride, (size_t)nk);
      addr_src[k] = hm[3 * n_msgs + k];
    } else {
      addr_src[k] = k;
    }
    ns[k] = nk;
  }
  *n_packets = count;
  return status;
}

// coalesceMessages(msgs, bufs, endpoint, addr) nMsgs -- conn/bind.go:599-662.
// The buffers are staged into 64 KiB slots of pinned memory, the kernel plans
// and appends in place there (over PCIe), and each message's appended bytes
// are copied into its first buffer's spare capacity.
int wgcs_coalesce_messages(wgcs_ctx* ctx, uint8_t* const* bufs, const size_t* lens, const size_t* caps, int nbufs,
                           int dst_is_v6, const uint8_t* src_ctl, size_t src_len, uint8_t* const* oobs,
                           size_t* oob_lens, const size_t* oob_caps, int* msg_first, size_t* msg_len, int* n_msgs) {
  if (!ctx || !n_msgs) return WGCS_ERR_INVALID_ARG;
  *n_msgs = 0;
  if (nbufs <= 0) return WGCS_OK;  // for-range over no bufs: nMsgs = 0
  if (!bufs || !lens || !caps || !msg_first || !msg_len || (oobs && (!oob_lens || !oob_caps)) ||
      (src_len && !src_ctl))
    return set_err(ctx, WGCS_ERR_INVALID_ARG, "bufs/lens/caps/msg arrays");
  for (int j = 0; j < nbufs; ++j) {
    if (lens[j] > caps[j] || lens[j] > 0x7FFFFFFFu) return set_err(ctx, WGCS_ERR_INVALID_ARG, "len(bufs[%d]) > cap", j);
    if (lens[j] > kSlot) return set_err(ctx, WGCS_ERR_INVALID_ARG, "bufs[%d] longer than 64 KiB", j);
  }
  const size_t data = (size_t)nbufs * kSlot;
  const size_t meta = (size_t)nbufs * 4 * 5 + 16;  // lens | caps | first | len | gso | nbufs | n_msgs
  std::lock_guard<std::mutex> g(ctx->mu);
  hipSetDevice(ctx->device);
  int rc;
  // zero-copy: the kernel plans and appends in place in 64 KiB slots of
  // pinned staging, over PCIe (one launch, one wait, no copy commands)
  if ((rc = ensure_pinned(ctx, ctx->h_stage, data)) || (rc = ensure_pinned(ctx, ctx->h_meta, meta))) return rc;
  uint8_t* hs = (uint8_t*)ctx->h_stage.ptr;
  int32_t* hm = (int32_t*)ctx->h_meta.ptr;
  for (int j = 0; j < nbufs; ++j) {
    if (lens[j]) memcpy(hs + (size_t)j * kSlot, bufs[j], lens[j]);
    hm[j] = (int32_t)lens[j];
    hm[nbufs + j] = (int32_t)std::min(caps[j], kSlot);  // exact: appends stop at maxPayloadLen < 64 KiB
  }
  hm[5 * nbufs] = nbufs;
  hipStream_t s = ctx->stream;
  hipError_t e = launch_udp_coalesce(hs, kSlot, (uint32_t)kSlot, hm + nbufs, hm, hm + 5 * nbufs, (uint32_t)nbufs, 1,
                                     dst_is_v6, hm + 5 * nbufs + 1, hm + 2 * nbufs, hm + 3 * nbufs, hm + 4 * nbufs, s);
  if (e != hipSuccess) return hip_fail(ctx, e, "coalesce_messages launch");
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return hip_fail(ctx, e, "coalesce_messages wait");
  const int nm = hm[5 * nbufs + 1];
  if (nm < 0 || nm > nbufs) return set_err(ctx, WGCS_ERR_HIP, "coalesce kernel returned %d messages", nm);
  for (int m = 0; m < nm; ++m) {
    const int f = hm[2 * nbufs + m];
    const size_t l0 = lens[f], l = (size_t)hm[3 * nbufs + m];
    if (l > l0) memcpy(bufs[f] + l0, hs + (size_t)f * kSlot + l0, l - l0);
    msg_first[m] = f;
    msg_len[m] = l;
    if (oobs) {  // setSrcControl at the run start (:657), setGSOSize when it holds > 1 packet (:634, :647)
      if (oob_caps[m] >= src_len) {
        if (src_len) memcpy(oobs[m], src_ctl, src_len);
        oob_lens[m] = src_len;
      }
      const int gs = hm[4 * nbufs + m];
      if (gs >= 0) put_gso(oobs[m], &oob_lens[m], oob_caps[m], (uint16_t)gs);
    }
  }
  *n_msgs = nm;
  return WGCS_OK;
}

}  // extern "C"
