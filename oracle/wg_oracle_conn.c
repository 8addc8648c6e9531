/*
 * wg_oracle_conn.c -- TEST INFRASTRUCTURE ONLY (see wg_oracle.h).
 *
 * CPU restatement of the outer-UDP message batching of muhtutorials/wireguard
 * (SURVEY.md §8f row 3): splitMessages / coalesceMessages
 * (conn/bind.go:542-662), getGSOSize / setGSOSize (conn/gso.go:35-100) and
 * setSrcControl (conn/sticky.go:101-107).  Statement order follows the Go
 * source; each function cites the lines it restates.
 *
 * Third-party pieces restated from their published algorithm (not present in
 * /root/reference): golang.org/x/sys/unix v0.41.0 (go.mod:5) for linux/amd64 --
 *   SizeofCmsghdr = 16 ({Len uint64; Level int32; Type int32}),
 *   cmsgAlignOf(n) = (n + 7) &^ 7, CmsgLen(d) = 16 + d, CmsgSpace(d) = 16 + cmsgAlignOf(d),
 *   ParseOneSocketControlMessage(b): h = b[0:16]; EINVAL unless 16 <= h.Len <= len(b);
 *     data = b[16:h.Len]; remainder = b[cmsgAlignOf(h.Len):] if that is < len(b), else empty;
 *   SOL_UDP = 17, UDP_SEGMENT = 103, UDP_GRO = 104 (/usr/include/linux/udp.h:35-36).
 * Go panics (slice bounds) become OR_ERR_OUT_OF_RANGE.
 */
#include "wg_oracle.h"

#include <string.h>

#define CMSG_HDR 16
static size_t cmsg_align(size_t n) { return (n + 7) & ~(size_t)7; }

/* conn/gso.go:35-67 */
int or_get_gso_size(const uint8_t *control, size_t len, int *gso) {
  *gso = 0;
  const uint8_t *rem = control;
  size_t rlen = len;
  while (rlen > CMSG_HDR) { /* :42 strictly greater */
    uint64_t hlen;
    int32_t level, type;
    memcpy(&hlen, rem, 8);
    memcpy(&level, rem + 8, 4);
    memcpy(&type, rem + 12, 4);
    if (hlen < CMSG_HDR || hlen > rlen) return OR_ERR_CMSG; /* :43-49 */
    const uint8_t *data = rem + CMSG_HDR;
    size_t dlen = (size_t)hlen - CMSG_HDR;
    size_t adv = cmsg_align((size_t)hlen);
    if (level == 17 && type == 104 && dlen >= 2) { /* :55-64, native byte order */
      uint16_t g;
      memcpy(&g, data, 2);
      *gso = g;
      return OR_OK;
    }
    if (adv < rlen) {
      rem += adv;
      rlen -= adv;
    } else {
      rlen = 0;
    }
  }
  return OR_OK;
}

/* conn/gso.go:71-100 (bytes [len+18, len+24) of the new cmsg keep their old contents) */
void or_set_gso_size(uint8_t *control, size_t *len, size_t cap, uint16_t gso) {
  const size_t space = CMSG_HDR + cmsg_align(2);
  if (space > cap - *len) return; /* :78-81 */
  uint8_t *c = control + *len;
  *len += space;                  /* :82 */
  const uint64_t hl = CMSG_HDR + 2; /* :93 SetLen(CmsgLen(2)) */
  const int32_t level = 17, type = 103;
  memcpy(c + 8, &level, 4);       /* :85 */
  memcpy(c + 12, &type, 4);       /* :86 */
  memcpy(c, &hl, 8);
  memcpy(c + CMSG_HDR, &gso, 2);  /* :95-99 */
}

/* conn/sticky.go:101-107 */
void or_set_src_control(uint8_t *control, size_t *len, size_t cap, const uint8_t *src, size_t src_len) {
  if (cap < src_len) return;
  memcpy(control, src, src_len);
  *len = src_len;
}

/* conn/bind.go:542-597 */
int or_split_messages(or_msg *msgs, int n_msgs, int first_msg_at, int *n_packets) {
  int np = 0;
  for (int i = first_msg_at; i < n_msgs; i++) {
    or_msg *msg = &msgs[i];
    if (msg->n == 0) { *n_packets = np; return OR_OK; } /* :545-547 */
    int gso, num = 1, start = 0, end = msg->n;
    int rc = or_get_gso_size(msg->oob, (size_t)msg->nn, &gso); /* :554 */
    if (rc) { *n_packets = np; return rc; }
    if (gso > 0) { /* :558-562 */
      num = (msg->n + gso - 1) / gso;
      end = gso;
    }
    for (int j = 0; j < num; j++) {
      if (np > i) { *n_packets = np; return OR_ERR_SPLIT_OVERFLOW; } /* :564-567 */
      /* msg.Buffers[0][start:end]: Go requires start <= end <= cap */
      if (end < start || (size_t)end > msg->buf_cap) { *n_packets = np; return OR_ERR_OUT_OF_RANGE; }
      or_msg *d = &msgs[np];
      size_t nb = (size_t)(end - start);
      if (nb > d->buf_len) nb = d->buf_len;         /* copy() length */
      memmove(d->buf, msg->buf + start, nb);        /* :568 (overlap-safe like Go's copy) */
      d->n = (int)nb;                               /* :569 */
      d->addr = msg->addr;                          /* :570 */
      start = end;                                  /* :571 */
      end += gso;                                   /* :572 */
      if (end > msg->n) end = msg->n;               /* :574 */
      np++;
    }
    if (i != np - 1) msg->n = 0; /* :589-594 */
  }
  *n_packets = np;
  return OR_OK;
}

/* conn/bind.go:599-662.  msgs[i].buf aliases the first buffer of run i (its
 * buf_len grows by the appends, which land in that buffer's own spare capacity). */
int or_coalesce_messages(or_msg *msgs, int n_msgs_cap, uint8_t *const *bufs, const size_t *lens,
                         const size_t *caps, int nbufs, int dst_is_v6, const uint8_t *src_ctl,
                         size_t src_len, int addr, int *n_msgs) {
  int i = -1, npk = 0, gso = 0, end_batch = 0; /* :605-614 */
  const size_t max_payload = dst_is_v6 ? OR_MAX_IPV6_PAYLOAD : OR_MAX_IPV4_PAYLOAD; /* :615-618 */
  for (int j = 0; j < nbufs; j++) {
    if (j > 0) { /* :620-644 */
      const size_t buf_len = lens[j];
      const size_t msg_len = msgs[i].buf_len;
      const size_t available = msgs[i].buf_cap - msg_len;
      if (buf_len + msg_len <= max_payload && buf_len <= (size_t)gso && buf_len <= available &&
          npk < OR_MAX_UDP_SEGMENTS && !end_batch) {
        memcpy(msgs[i].buf + msg_len, bufs[j], buf_len); /* :629 append within cap */
        msgs[i].buf_len = msg_len + buf_len;
        if (j == nbufs - 1) or_set_gso_size(msgs[i].oob, &msgs[i].oob_len, msgs[i].oob_cap, (uint16_t)gso);
        npk++;
        if (buf_len < (size_t)gso) end_batch = 1; /* :637-641 */
        continue;
      }
    }
    if (npk > 1) or_set_gso_size(msgs[i].oob, &msgs[i].oob_len, msgs[i].oob_cap, (uint16_t)gso); /* :647-649 */
    i++;
    if (i >= n_msgs_cap) { *n_msgs = i; return OR_ERR_OUT_OF_RANGE; } /* msgs[i] index panic */
    npk = 1;                                                      /* :651 */
    gso = (int)lens[j];                                           /* :652 */
    end_batch = 0;                                                /* :655 */
    or_set_src_control(msgs[i].oob, &msgs[i].oob_len, msgs[i].oob_cap, src_ctl, src_len); /* :657 */
    msgs[i].buf = bufs[j];                                        /* :658 */
    msgs[i].buf_len = lens[j];
    msgs[i].buf_cap = caps[j];
    msgs[i].addr = addr;                                          /* :659 */
  }
  *n_msgs = i + 1;
  return OR_OK;
}

/* Batch drivers for tests and bench.py's cpu_baseline leg: n_batches
 * independent calls on a flat host layout (slot q = b*n + s at base + q*stride). */
void or_split_batch(uint8_t *bufs, size_t stride, size_t buf_len, int *ns, uint8_t *oobs, size_t oob_stride,
                    const int *nns, int n_msgs, int first, int n_batches, int *counts, int *statuses) {
  or_msg msgs[1024];
  if (n_msgs > 1024) return;
  for (int b = 0; b < n_batches; b++) {
    for (int s = 0; s < n_msgs; s++) {
      const size_t q = (size_t)b * n_msgs + s;
      msgs[s].buf = bufs + q * stride;
      msgs[s].buf_len = msgs[s].buf_cap = buf_len;
      msgs[s].n = ns[q];
      msgs[s].oob = oobs + q * oob_stride;
      msgs[s].oob_len = msgs[s].oob_cap = oob_stride;
      msgs[s].nn = nns[q];
      msgs[s].addr = s;
    }
    statuses[b] = or_split_messages(msgs, n_msgs, first, &counts[b]);
    for (int s = 0; s < n_msgs; s++) ns[(size_t)b * n_msgs + s] = msgs[s].n;
  }
}

void or_coalesce_batch(uint8_t *bufs, size_t stride, const size_t *lens, const size_t *caps, const int *nbufs,
                       int max_bufs, int n_batches, int dst_is_v6, int *n_msgs_out) {
  or_msg msgs[1024];
  uint8_t *ptrs[1024];
  uint8_t oob[1024][64];
  if (max_bufs > 1024) return;
  for (int b = 0; b < n_batches; b++) {
    const size_t q0 = (size_t)b * max_bufs;
    for (int j = 0; j < nbufs[b]; j++) {
      ptrs[j] = bufs + (q0 + j) * stride;
      msgs[j].oob = oob[j];
      msgs[j].oob_len = 0;
      msgs[j].oob_cap = 64;
    }
    or_coalesce_messages(msgs, max_bufs, ptrs, lens + q0, caps + q0, nbufs[b], dst_is_v6, NULL, 0, 0,
                         &n_msgs_out[b]);
  }
}
