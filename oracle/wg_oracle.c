/*
 * wg_oracle.c -- TEST INFRASTRUCTURE ONLY (see wg_oracle.h header comment).
 *
 * Line-by-line CPU restatement of the reference's hot path:
 *   /root/reference/tun/checksum.go   (checksumNoFold, pseudoHeaderChecksumNoFold,
 *                                      checksum)
 *   /root/reference/tun/gro.go        (checksumValid, gsoSplit, gsoNoneChecksum,
 *                                      handleGRO and its helpers)
 *   /root/reference/tun/tun.go:514-632 (handleVirtioRead)
 * Every function cites the reference lines it follows.  Where the reference
 * would panic (slice out of range) this restatement returns
 * OR_ERR_OUT_OF_RANGE instead; tests never feed such inputs to both sides.
 */
#include "wg_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ---- little helpers: Go's encoding/binary on a little-endian host ---- */
static inline uint64_t ne64(const uint8_t *p) { uint64_t v; memcpy(&v, p, 8); return v; }
static inline uint32_t ne32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static inline uint16_t ne16(const uint8_t *p) { uint16_t v; memcpy(&v, p, 2); return v; }
static inline uint16_t be16(const uint8_t *p) { return (uint16_t)((p[0] << 8) | p[1]); }
static inline uint32_t be32(const uint8_t *p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
static inline void put_be16(uint8_t *p, uint16_t v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }
static inline void put_be32(uint8_t *p, uint32_t v) {
  p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16); p[2] = (uint8_t)(v >> 8); p[3] = (uint8_t)v;
}
/* binary.NativeEndian.PutUint64 then binary.BigEndian.Uint64 == bswap64 on LE */
static inline uint64_t ne_to_be64(uint64_t v) { return __builtin_bswap64(v); }

/* bits.Add64(x, y, carry) */
static inline uint64_t add64(uint64_t x, uint64_t y, uint64_t c, uint64_t *co) {
  uint64_t s, t;
  int c1 = __builtin_add_overflow(x, y, &s);
  int c2 = __builtin_add_overflow(s, c, &t);
  *co = (uint64_t)(c1 | c2);
  return t;
}

/* checksum.go:8-120 */
uint64_t or_checksum_nofold(const uint8_t *b, size_t n, uint64_t initial) {
  uint64_t ac = ne_to_be64(initial); /* :39-41 */
  uint64_t carry;
  while (n >= 128) { /* :44-63 */
    ac = add64(ac, ne64(b + 0), 0, &carry);
    for (int k = 8; k < 128; k += 8) ac = add64(ac, ne64(b + k), carry, &carry);
    ac += carry;
    b += 128; n -= 128;
  }
  if (n >= 64) { /* :64-75 */
    ac = add64(ac, ne64(b + 0), 0, &carry);
    for (int k = 8; k < 64; k += 8) ac = add64(ac, ne64(b + k), carry, &carry);
    ac += carry;
    b += 64; n -= 64;
  }
  if (n >= 32) { /* :76-83 */
    ac = add64(ac, ne64(b + 0), 0, &carry);
    for (int k = 8; k < 32; k += 8) ac = add64(ac, ne64(b + k), carry, &carry);
    ac += carry;
    b += 32; n -= 32;
  }
  if (n >= 16) { /* :84-89 */
    ac = add64(ac, ne64(b + 0), 0, &carry);
    ac = add64(ac, ne64(b + 8), carry, &carry);
    ac += carry;
    b += 16; n -= 16;
  }
  if (n >= 8) { /* :90-94 */
    ac = add64(ac, ne64(b), 0, &carry);
    ac += carry;
    b += 8; n -= 8;
  }
  if (n >= 4) { /* :95-99 */
    ac = add64(ac, (uint64_t)ne32(b), 0, &carry);
    ac += carry;
    b += 4; n -= 4;
  }
  if (n >= 2) { /* :100-104 */
    ac = add64(ac, (uint64_t)ne16(b), 0, &carry);
    ac += carry;
    b += 2; n -= 2;
  }
  if (n == 1) { /* :105-117: NativeEndian.Uint16([]byte{b[0], 0}) */
    uint8_t tmp[2] = {b[0], 0};
    ac = add64(ac, (uint64_t)ne16(tmp), 0, &carry);
    ac += carry;
  }
  return ne_to_be64(ac); /* :118-119 */
}

/* checksum.go:152-167 -- four folds, NOT complemented */
uint16_t or_checksum(const uint8_t *b, size_t n, uint64_t initial) {
  uint64_t ac = or_checksum_nofold(b, n, initial);
  ac = (ac >> 16) + (ac & 0xffff);
  ac = (ac >> 16) + (ac & 0xffff);
  ac = (ac >> 16) + (ac & 0xffff);
  ac = (ac >> 16) + (ac & 0xffff);
  return (uint16_t)ac;
}

/* checksum.go:127-150 */
uint64_t or_pseudo_header_nofold(const uint8_t *src, const uint8_t *dst,
                                 size_t addr_len, uint8_t proto,
                                 uint16_t total_len) {
  uint64_t sum = or_checksum_nofold(src, addr_len, 0);
  sum = or_checksum_nofold(dst, addr_len, sum);
  uint8_t p[2] = {0, proto};
  sum = or_checksum_nofold(p, 2, sum);
  uint8_t t[2];
  put_be16(t, total_len);
  return or_checksum_nofold(t, 2, sum);
}

enum { IPV4_SRC = 12, IPV6_SRC = 8, MAX_U16 = 65535, PROTO_TCP = 6, PROTO_UDP = 17 };
enum { VNET_LEN = 10, F_NEEDS_CSUM = 1, GSO_NONE = 0, GSO_TCPV4 = 1, GSO_TCPV6 = 4,
       GSO_UDP_L4 = 5 };
enum { TCP_FLAGS_OFF = 13, TCP_FIN = 0x01, TCP_PSH = 0x08, TCP_ACK = 0x10, UDPH_LEN = 8 };

/* gro.go:554-612.  The address slices pkt[a:b] (:558-563) are bounded by
 * cap(pkt), not len: a packet shorter than its addresses reads them from the
 * bytes after it (the caller guarantees pkt[0, cap)); pkt[iphLen:] (:611) is
 * bounded by len.  Returns 1 / 0, or OR_ERR_OUT_OF_RANGE where Go panics. */
static int checksum_valid_at(const uint8_t *pkt, size_t len, size_t cap, size_t iph_len,
                             uint8_t proto, int is_v6) {
  size_t src_at = is_v6 ? IPV6_SRC : IPV4_SRC;
  size_t addr = is_v6 ? 16 : 4;
  if (cap < src_at + 2 * addr || len < iph_len) return OR_ERR_OUT_OF_RANGE; /* would panic */
  uint16_t total_len = (uint16_t)(len - iph_len);
  uint64_t ph = or_pseudo_header_nofold(pkt + src_at, pkt + src_at + addr, addr,
                                        proto, total_len);
  return (uint16_t)~or_checksum(pkt + iph_len, len - iph_len, ph) == 0;
}
int or_checksum_valid(const uint8_t *pkt, size_t len, uint8_t iph_len,
                      uint8_t proto, int is_v6) {
  return checksum_valid_at(pkt, len, len, iph_len, proto, is_v6);
}
int or_checksum_valid_cap(const uint8_t *pkt, size_t len, size_t cap, uint8_t iph_len,
                          uint8_t proto, int is_v6) {
  return checksum_valid_at(pkt, len, cap, iph_len, proto, is_v6);
}

/* gro.go:1497-1517 */
int or_gso_none_checksum(uint8_t *rb, size_t len, uint16_t csum_start,
                         uint16_t csum_offset) {
  uint16_t at = (uint16_t)(csum_start + csum_offset); /* u16 arithmetic */
  if ((size_t)at + 2 > len || csum_start > len) return OR_ERR_OUT_OF_RANGE;
  uint16_t initial = be16(rb + at);
  rb[at] = 0; rb[at + 1] = 0;
  put_be16(rb + at, (uint16_t)~or_checksum(rb + csum_start, len - csum_start, initial));
  return OR_OK;
}

/* gro.go:1373-1493.  Every index the reference computes from hdr fields is a
 * uint16 sum (hdr.csumStart+4, +tcpFlagsOffset, +hdr.csumOffset wrap at
 * 2^16); indexes of readBuf are bounded by len(readBuf), and its slices by
 * cap(readBuf): rb[len, cap) is the read buffer's spare capacity, which the
 * pseudo-header address slices reach for a packet shorter than 20 / 40 bytes
 * (:1471-1477; see or_gso_split_need for the bufs side). */
int or_gso_split_cap(uint8_t *rb, size_t len, size_t cap, or_virtio_hdr hdr,
                     uint8_t *const *bufs, const size_t *buf_lens, int nbufs,
                     int *sizes, int offset, int is_v6, int *n_out) {
  int iph_len = hdr.csum_start;
  int src_off = IPV6_SRC, addr_len = 16;
  *n_out = 0;
  if (!is_v6) {
    src_off = IPV4_SRC; addr_len = 4;
    if (len < 12) return OR_ERR_OUT_OF_RANGE; /* readBuf[10], readBuf[11] */
    rb[10] = 0; rb[11] = 0; /* :1388 */
  }
  int csum_at = (uint16_t)(hdr.csum_start + hdr.csum_offset); /* :1391 */
  if ((size_t)csum_at + 2 > len) return OR_ERR_OUT_OF_RANGE;
  rb[csum_at] = 0; rb[csum_at + 1] = 0; /* :1393 */
  const int seq_at = (uint16_t)(hdr.csum_start + 4);              /* hdr.csumStart+4 (u16) */
  const int flags_at = (uint16_t)(hdr.csum_start + TCP_FLAGS_OFF); /* :1458 (u16) */
  uint32_t first_seq = 0;
  uint8_t proto;
  if (hdr.gso_type == GSO_TCPV4 || hdr.gso_type == GSO_TCPV6) { /* :1398-1405 */
    proto = PROTO_TCP;
    if ((size_t)seq_at + 4 > len) return OR_ERR_OUT_OF_RANGE; /* Uint32(readBuf[csumStart+4:]) */
    first_seq = be32(rb + seq_at);
  } else {
    proto = PROTO_UDP;
  }
  size_t next = hdr.hdr_len;
  if (next < len) {
    /* the loop runs: pkt[csumStart:hdrLen] panics if csumStart > hdrLen; the
     * pseudo-header address slices panic past cap(readBuf) */
    if (hdr.csum_start > hdr.hdr_len) return OR_ERR_OUT_OF_RANGE;
    if ((size_t)(src_off + 2 * addr_len) > cap) return OR_ERR_OUT_OF_RANGE;
  }
  int i = 0;
  while (next < len) { /* :1408 */
    if (i == nbufs) { *n_out = i - 1; return OR_ERR_TOO_MANY_SEGMENTS; } /* :1409-1410 */
    size_t seg_end = next + hdr.gso_size;
    if (seg_end > len) seg_end = len;
    size_t seg_len = seg_end - next;
    size_t pkt_len = hdr.hdr_len + seg_len;
    sizes[i] = (int)pkt_len;
    if (buf_lens[i] < (size_t)offset + or_gso_split_need(hdr, is_v6, pkt_len, seg_end == len)) {
      *n_out = i; /* a slice of bufs[i][offset:] would panic */
      return OR_ERR_OUT_OF_RANGE;
    }
    uint8_t *pkt = bufs[i] + offset;
    memcpy(pkt, rb, (size_t)iph_len); /* :1419 */
    if (!is_v6) {
      if (i > 0) { /* :1426-1431 -- quirk: id0 + 1 for every i >= 1 */
        uint16_t id = be16(pkt + 4); /* bytes past iphLen: whatever bufs[i] held */
        id += 1;
        put_be16(pkt + 4, id);
      }
      put_be16(pkt + 2, (uint16_t)pkt_len);                          /* :1433 */
      put_be16(pkt + 10, (uint16_t)~or_checksum(pkt, iph_len, 0));   /* :1434-1436 */
    } else {
      put_be16(pkt + 4, (uint16_t)(pkt_len - iph_len));              /* :1439 */
    }
    memcpy(pkt + hdr.csum_start, rb + hdr.csum_start,
           (size_t)(hdr.hdr_len - hdr.csum_start));                   /* :1442 */
    if (proto == PROTO_TCP) {
      uint32_t seq = first_seq + (uint32_t)(uint16_t)(hdr.gso_size * (uint16_t)i); /* :1445 */
      put_be32(pkt + seq_at, seq);
      if (seg_end != len) pkt[flags_at] &= (uint8_t)~(TCP_FIN | TCP_PSH);
    } else {
      put_be16(pkt + seq_at,
               (uint16_t)((uint16_t)seg_len + (uint16_t)(hdr.hdr_len - hdr.csum_start))); /* :1462-1465 */
    }
    memcpy(pkt + hdr.hdr_len, rb + next, seg_len);                   /* :1468 */
    int th_len = hdr.hdr_len - hdr.csum_start;
    uint16_t t_len = (uint16_t)(th_len + (int)seg_len);              /* :1469-1471 */
    uint64_t ph = or_pseudo_header_nofold(rb + src_off, rb + src_off + addr_len,
                                          (size_t)addr_len, proto, t_len);
    uint16_t c = (uint16_t)~or_checksum(pkt + hdr.csum_start, pkt_len - hdr.csum_start, ph);
    put_be16(pkt + csum_at, c);                                       /* :1485-1488 */
    next += hdr.gso_size;
    i++;
  }
  *n_out = i;
  return OR_OK;
}

int or_gso_split(uint8_t *rb, size_t len, or_virtio_hdr hdr,
                 uint8_t *const *bufs, const size_t *buf_lens, int nbufs,
                 int *sizes, int offset, int is_v6, int *n_out) {
  return or_gso_split_cap(rb, len, len, hdr, bufs, buf_lens, nbufs, sizes, offset, is_v6, n_out);
}

/* Bytes of bufs[i][offset:] one gsoSplit segment touches (gro.go:1419-1488):
 * the packet itself plus fixed-position header writes that may lie past it
 * (IPv4 [2:12), IPv6 [4:6), seq / UDP length at csumStart+4, the flags byte,
 * the checksum field, all u16 positions).  A shorter buffer panics in Go. */
size_t or_gso_split_need(or_virtio_hdr hdr, int is_v6, size_t pkt_len, int last) {
  const int tcp = hdr.gso_type == GSO_TCPV4 || hdr.gso_type == GSO_TCPV6;
  size_t need = pkt_len;
  size_t t = is_v6 ? 6 : 12;
  if (t > need) need = t;
  t = (size_t)(uint16_t)(hdr.csum_start + 4) + (tcp ? 4 : 2);
  if (t > need) need = t;
  if (tcp && !last) {
    t = (size_t)(uint16_t)(hdr.csum_start + TCP_FLAGS_OFF) + 1;
    if (t > need) need = t;
  }
  t = (size_t)(uint16_t)(hdr.csum_start + hdr.csum_offset) + 2;
  if (t > need) need = t;
  return need;
}

/* tun/tun.go:514-632; rb[n, cap) is readBuf's spare capacity (Tun.Read
 * passes tun.readBuf[:n], tun.go:484-503) */
int or_handle_virtio_read_cap(uint8_t *rb, size_t n, size_t cap, uint8_t *const *bufs,
                              const size_t *buf_lens, int nbufs, int *sizes,
                              int offset, int *n_out) {
  *n_out = 0;
  if (n < VNET_LEN) return OR_ERR_SHORT_BUFFER; /* gro.go:84-86 */
  or_virtio_hdr hdr;
  hdr.flags = rb[0];
  hdr.gso_type = rb[1];
  hdr.hdr_len = ne16(rb + 2);
  hdr.gso_size = ne16(rb + 4);
  hdr.csum_start = ne16(rb + 6);
  hdr.csum_offset = ne16(rb + 8);
  rb += VNET_LEN; n -= VNET_LEN; cap -= VNET_LEN; /* :527 */
  if (hdr.gso_type == GSO_NONE) { /* :532-556 */
    if (hdr.flags & F_NEEDS_CSUM) {
      int rc = or_gso_none_checksum(rb, n, hdr.csum_start, hdr.csum_offset);
      if (rc) return rc;
    }
    if (n > buf_lens[0] - (size_t)offset) return OR_ERR_READ_OVERFLOW;
    memcpy(bufs[0] + offset, rb, n);
    sizes[0] = (int)n;
    *n_out = 1;
    return OR_OK;
  }
  if (hdr.gso_type != GSO_TCPV4 && hdr.gso_type != GSO_TCPV6 && hdr.gso_type != GSO_UDP_L4)
    return OR_ERR_UNSUPPORTED_GSO; /* :564-568 */
  if (n < 1) return OR_ERR_OUT_OF_RANGE;
  int ipv = rb[0] >> 4; /* :570 */
  if (ipv == 4) {
    if (hdr.gso_type != GSO_TCPV4 && hdr.gso_type != GSO_UDP_L4) return OR_ERR_IP_GSO_MISMATCH;
  } else if (ipv == 6) {
    if (hdr.gso_type != GSO_TCPV6 && hdr.gso_type != GSO_UDP_L4) return OR_ERR_IP_GSO_MISMATCH;
  } else {
    return OR_ERR_BAD_IP_VERSION;
  }
  if (hdr.gso_type == GSO_UDP_L4) { /* :597-614 */
    hdr.hdr_len = (uint16_t)(hdr.csum_start + 8);
  } else {
    if (n <= (size_t)(uint16_t)(hdr.csum_start + 12)) return OR_ERR_PACKET_TOO_SHORT;
    uint16_t th = (uint16_t)((rb[(uint16_t)(hdr.csum_start + 12)] >> 4) * 4);
    if (th < 20 || th > 60) return OR_ERR_TCP_HDR_LEN;
    hdr.hdr_len = (uint16_t)(hdr.csum_start + th);
  }
  if (n < hdr.hdr_len) return OR_ERR_HDR_LEN; /* :615-621 */
  int csum_at = (uint16_t)(hdr.csum_start + hdr.csum_offset);
  if ((size_t)csum_at + 1 >= n) return OR_ERR_CSUM_OFFSET; /* :622-630 */
  return or_gso_split_cap(rb, n, cap, hdr, bufs, buf_lens, nbufs, sizes, offset, ipv == 6, n_out);
}

int or_handle_virtio_read(uint8_t *rb, size_t n, uint8_t *const *bufs,
                          const size_t *buf_lens, int nbufs, int *sizes,
                          int offset, int *n_out) {
  return or_handle_virtio_read_cap(rb, n, n, bufs, buf_lens, nbufs, sizes, offset, n_out);
}

/* ====================================================================== */
/* GRO: gro.go:95-376 (flow tables), :392-544 (can-coalesce), :614-783      */
/* (coalesce), :801-1095 (tcpGRO/udpGRO), :1099-1268 (apply), :1280-1367.   */
/* Go maps become flat arrays with linear lookup; map iteration order is    */
/* irrelevant because every item is applied independently.                  */
/* ====================================================================== */

typedef struct { uint8_t src[16], dst[16]; uint16_t sport, dport; uint32_t ack; int v6; } tcp_key;
typedef struct { uint8_t src[16], dst[16]; uint16_t sport, dport; int v6; } udp_key;
typedef struct {
  tcp_key key; uint32_t seq; uint16_t bufs_index, num_merged, gso_size;
  uint8_t iph_len, tcph_len; int psh;
} tcp_item;
typedef struct {
  udp_key key; uint16_t bufs_index, num_merged, gso_size; uint8_t iph_len; int csum_bad;
} udp_item;
typedef struct { tcp_key key; tcp_item *items; int n, cap; } tcp_flow;
typedef struct { udp_key key; udp_item *items; int n, cap; } udp_flow;
typedef struct { tcp_flow *f; int n, cap; } tcp_table;
typedef struct { udp_flow *f; int n, cap; } udp_table;

static void *grow(void *p, int *cap, size_t elt) {
  int nc = *cap ? *cap * 2 : 8;
  void *q = realloc(p, (size_t)nc * elt);
  if (!q) abort();
  *cap = nc;
  return q;
}

static tcp_key mk_tcp_key(const uint8_t *pkt, int src_off, int dst_off, int th_off) { /* :111-127 */
  tcp_key k; memset(&k, 0, sizeof k);
  int as = dst_off - src_off;
  memcpy(k.src, pkt + src_off, (size_t)as);
  memcpy(k.dst, pkt + dst_off, (size_t)as);
  k.sport = be16(pkt + th_off); k.dport = be16(pkt + th_off + 2);
  k.ack = be32(pkt + th_off + 8);
  k.v6 = as == 16;
  return k;
}
static udp_key mk_udp_key(const uint8_t *pkt, int src_off, int dst_off, int uh_off) { /* :261-275 */
  udp_key k; memset(&k, 0, sizeof k);
  int as = dst_off - src_off;
  memcpy(k.src, pkt + src_off, (size_t)as);
  memcpy(k.dst, pkt + dst_off, (size_t)as);
  k.sport = be16(pkt + uh_off); k.dport = be16(pkt + uh_off + 2);
  k.v6 = as == 16;
  return k;
}
static int tcp_key_eq(const tcp_key *a, const tcp_key *b) {
  return !memcmp(a->src, b->src, 16) && !memcmp(a->dst, b->dst, 16) && a->sport == b->sport &&
         a->dport == b->dport && a->ack == b->ack && a->v6 == b->v6;
}
static int udp_key_eq(const udp_key *a, const udp_key *b) {
  return !memcmp(a->src, b->src, 16) && !memcmp(a->dst, b->dst, 16) && a->sport == b->sport &&
         a->dport == b->dport && a->v6 == b->v6;
}
static tcp_flow *tcp_find(tcp_table *t, const tcp_key *k) {
  for (int i = 0; i < t->n; i++) if (tcp_key_eq(&t->f[i].key, k)) return &t->f[i];
  return NULL;
}
static udp_flow *udp_find(udp_table *t, const udp_key *k) {
  for (int i = 0; i < t->n; i++) if (udp_key_eq(&t->f[i].key, k)) return &t->f[i];
  return NULL;
}
static void tcp_insert(tcp_table *t, const uint8_t *pkt, size_t plen, int src_off, int dst_off,
                       int th_off, int th_len, int bi) { /* :207-232 */
  tcp_item it; memset(&it, 0, sizeof it);
  it.key = mk_tcp_key(pkt, src_off, dst_off, th_off);
  it.bufs_index = (uint16_t)bi;
  it.gso_size = (uint16_t)(plen - (size_t)(th_off + th_len));
  it.iph_len = (uint8_t)th_off;
  it.tcph_len = (uint8_t)th_len;
  it.seq = be32(pkt + th_off + 4);
  it.psh = (pkt[th_off + TCP_FLAGS_OFF] & TCP_PSH) != 0;
  tcp_flow *f = tcp_find(t, &it.key);
  if (!f) {
    if (t->n == t->cap) t->f = grow(t->f, &t->cap, sizeof *t->f);
    f = &t->f[t->n++];
    memset(f, 0, sizeof *f);
    f->key = it.key;
  }
  if (f->n == f->cap) f->items = grow(f->items, &f->cap, sizeof *f->items);
  f->items[f->n++] = it;
}
static void udp_insert(udp_table *t, const uint8_t *pkt, size_t plen, int src_off, int dst_off,
                       int uh_off, int bi, int bad) { /* :349-371 */
  udp_item it; memset(&it, 0, sizeof it);
  it.key = mk_udp_key(pkt, src_off, dst_off, uh_off);
  it.bufs_index = (uint16_t)bi;
  it.gso_size = (uint16_t)(plen - (size_t)(uh_off + UDPH_LEN));
  it.iph_len = (uint8_t)uh_off;
  it.csum_bad = bad;
  udp_flow *f = udp_find(t, &it.key);
  if (!f) {
    if (t->n == t->cap) t->f = grow(t->f, &t->cap, sizeof *t->f);
    f = &t->f[t->n++];
    memset(f, 0, sizeof *f);
    f->key = it.key;
  }
  if (f->n == f->cap) f->items = grow(f->items, &f->cap, sizeof *f->items);
  f->items[f->n++] = it;
}

/* gro.go:392-427 */
static int ip_headers_can_coalesce(const uint8_t *a, size_t la, const uint8_t *b, size_t lb) {
  if (la < 9 || lb < 9) return 0;
  if (a[0] >> 4 == 6) {
    if (a[0] != b[0] || a[1] >> 4 != b[1] >> 4) return 0;
    if (a[7] != b[7]) return 0;
  } else {
    if (a[1] != b[1]) return 0;
    if (a[6] >> 5 != b[6] >> 5) return 0;
    if (a[8] != b[8]) return 0;
  }
  return 1;
}

enum { CO_PREPEND = -1, CO_UNAVAIL = 0, CO_APPEND = 1 };
enum { R_INSUFF_CAP, R_PSH_ENDING, R_ITEM_BAD, R_PKT_BAD, R_SUCCESS };
enum { GRO_NOOP, GRO_INSERT, GRO_COALESCED };

/* gro.go:433-512 */
static int tcp_can_coalesce(const uint8_t *pkt, size_t plen, uint8_t iph, uint8_t th, uint32_t seq,
                            int psh, uint16_t gso, const tcp_item *it, uint8_t **bufs,
                            const size_t *lens, int offset) {
  const uint8_t *tgt = bufs[it->bufs_index] + offset;
  size_t tlen = lens[it->bufs_index] - (size_t)offset;
  if (th != it->tcph_len) return CO_UNAVAIL;
  if (th > 20) {
    if (memcmp(pkt + iph + 20, tgt + it->iph_len + 20, (size_t)(th - 20))) return CO_UNAVAIL;
  }
  if (!ip_headers_can_coalesce(pkt, plen, tgt, tlen)) return CO_UNAVAIL;
  uint16_t lhs = (uint16_t)(it->gso_size + (uint16_t)(it->gso_size * it->num_merged));
  if (seq == it->seq + (uint32_t)lhs) {
    if (it->psh) return CO_UNAVAIL;
    if ((tlen - (size_t)(iph + th)) % it->gso_size != 0) return CO_UNAVAIL;
    if (gso > it->gso_size) return CO_UNAVAIL;
    return CO_APPEND;
  } else if (seq + (uint32_t)gso == it->seq) {
    if (psh) return CO_UNAVAIL;
    if (gso < it->gso_size) return CO_UNAVAIL;
    if (gso > it->gso_size && it->num_merged > 0) return CO_UNAVAIL;
    return CO_PREPEND;
  }
  return CO_UNAVAIL;
}

/* gro.go:519-544 */
static int udp_can_coalesce(const uint8_t *pkt, size_t plen, uint8_t iph, uint16_t gso,
                            const udp_item *it, uint8_t **bufs, const size_t *lens, int offset) {
  const uint8_t *tgt = bufs[it->bufs_index] + offset;
  size_t tlen = lens[it->bufs_index] - (size_t)offset;
  if (!ip_headers_can_coalesce(pkt, plen, tgt, tlen)) return CO_UNAVAIL;
  if ((tlen - (size_t)(iph + UDPH_LEN)) % it->gso_size != 0) return CO_UNAVAIL;
  if (gso > it->gso_size) return CO_UNAVAIL;
  return CO_APPEND;
}

static void swap_buf(uint8_t **bufs, size_t *lens, size_t *caps, int a, int b) {
  uint8_t *tb = bufs[a]; bufs[a] = bufs[b]; bufs[b] = tb;
  size_t tl = lens[a]; lens[a] = lens[b]; lens[b] = tl;
  size_t tc = caps[a]; caps[a] = caps[b]; caps[b] = tc;
}

/* gro.go:630-741 */
static int coalesce_tcp(int mode, int pkt_bi, uint16_t gso, uint32_t seq, int psh, tcp_item *it,
                        uint8_t **bufs, size_t *lens, size_t *caps, int offset, int v6) {
  const uint8_t *pkt = bufs[pkt_bi] + offset;
  size_t plen = lens[pkt_bi] - (size_t)offset;
  uint8_t hdrs = (uint8_t)(it->iph_len + it->tcph_len);
  size_t pay = plen - hdrs;
  size_t new_len = (lens[it->bufs_index] - (size_t)offset) + pay;
  if (mode == CO_PREPEND) {
    if (caps[pkt_bi] - (size_t)offset < new_len) return R_INSUFF_CAP;
    if (psh) return R_PSH_ENDING;
    if (it->num_merged == 0) {
      if (!or_checksum_valid(bufs[it->bufs_index] + offset, lens[it->bufs_index] - (size_t)offset,
                             it->iph_len, PROTO_TCP, v6))
        return R_ITEM_BAD;
    }
    if (!or_checksum_valid(pkt, plen, it->iph_len, PROTO_TCP, v6)) return R_PKT_BAD;
    it->seq = seq;
    size_t item_pay = new_len - plen;
    size_t old = lens[pkt_bi];
    lens[pkt_bi] += item_pay;
    memcpy(bufs[pkt_bi] + old, bufs[it->bufs_index] + offset + hdrs, item_pay);
    swap_buf(bufs, lens, caps, it->bufs_index, pkt_bi);
  } else {
    if (caps[it->bufs_index] - (size_t)offset < new_len) return R_INSUFF_CAP;
    if (it->num_merged == 0) {
      if (!or_checksum_valid(bufs[it->bufs_index] + offset, lens[it->bufs_index] - (size_t)offset,
                             it->iph_len, PROTO_TCP, v6))
        return R_ITEM_BAD;
    }
    if (!or_checksum_valid(pkt, plen, it->iph_len, PROTO_TCP, v6)) return R_PKT_BAD;
    if (psh) {
      it->psh = 1;
      bufs[it->bufs_index][offset + it->iph_len + TCP_FLAGS_OFF] |= TCP_PSH;
    }
    size_t old = lens[it->bufs_index];
    lens[it->bufs_index] += pay;
    memcpy(bufs[it->bufs_index] + old, pkt + hdrs, pay);
  }
  if (gso > it->gso_size) it->gso_size = gso;
  it->num_merged++;
  return R_SUCCESS;
}

/* gro.go:745-783 */
static int coalesce_udp(int pkt_bi, udp_item *it, uint8_t **bufs, size_t *lens, size_t *caps,
                        int offset, int v6) {
  const uint8_t *pkt = bufs[pkt_bi] + offset;
  size_t plen = lens[pkt_bi] - (size_t)offset;
  size_t head_len = lens[it->bufs_index] - (size_t)offset;
  uint8_t hdrs = (uint8_t)(it->iph_len + UDPH_LEN);
  size_t pay = plen - hdrs;
  size_t new_len = head_len + pay;
  if (caps[it->bufs_index] - (size_t)offset < new_len) return R_INSUFF_CAP;
  if (it->num_merged == 0) {
    if (it->csum_bad ||
        !or_checksum_valid(bufs[it->bufs_index] + offset, head_len, it->iph_len, PROTO_UDP, v6))
      return R_ITEM_BAD;
  }
  if (!or_checksum_valid(pkt, plen, it->iph_len, PROTO_UDP, v6)) return R_PKT_BAD;
  size_t old = lens[it->bufs_index];
  lens[it->bufs_index] += pay;
  memcpy(bufs[it->bufs_index] + old, pkt + hdrs, pay);
  it->num_merged++;
  return R_SUCCESS;
}

/* gro.go:801-963 */
static int tcp_gro(uint8_t **bufs, size_t *lens, size_t *caps, int offset, int bi, tcp_table *t,
                   int v6) {
  const uint8_t *pkt = bufs[bi] + offset;
  size_t plen = lens[bi] - (size_t)offset;
  if (plen > MAX_U16) return GRO_NOOP;
  int iph = (uint8_t)((pkt[0] & 0x0F) * 4);
  if (v6) {
    iph = 40;
    if ((int)be16(pkt + 4) != (int)plen - iph) return GRO_NOOP;
  } else {
    if ((size_t)be16(pkt + 2) != plen) return GRO_NOOP;
  }
  if (plen < (size_t)iph) return GRO_NOOP;
  int th = (uint8_t)((pkt[iph + 12] >> 4) * 4);
  if (th < 20 || th > 60) return GRO_NOOP;
  if (plen < (size_t)(iph + th)) return GRO_NOOP;
  if (!v6) {
    if ((pkt[6] & 0x20) != 0 || (uint8_t)(pkt[6] << 3) != 0 || pkt[7] != 0) return GRO_NOOP;
  }
  uint8_t flags = pkt[iph + TCP_FLAGS_OFF];
  int psh = 0;
  if (flags != TCP_ACK) {
    if (flags != (TCP_ACK | TCP_PSH)) return GRO_NOOP;
    psh = 1;
  }
  uint16_t gso = (uint16_t)(plen - (size_t)iph - (size_t)th);
  if (gso < 1) return GRO_NOOP;
  uint32_t seq = be32(pkt + iph + 4);
  int src_off = v6 ? IPV6_SRC : IPV4_SRC;
  int alen = v6 ? 16 : 4;
  tcp_key key = mk_tcp_key(pkt, src_off, src_off + alen, iph);
  tcp_flow *f = tcp_find(t, &key);
  if (!f) { /* getOrInsert :189-204 */
    tcp_insert(t, pkt, plen, src_off, src_off + alen, iph, th, bi);
    return GRO_INSERT;
  }
  for (int i = f->n - 1; i >= 0; i--) {
    tcp_item item = f->items[i];
    int can = tcp_can_coalesce(pkt, plen, (uint8_t)iph, (uint8_t)th, seq, psh, gso, &item, bufs,
                               lens, offset);
    if (can != CO_UNAVAIL) {
      int r = coalesce_tcp(can, bi, gso, seq, psh, &item, bufs, lens, caps, offset, v6);
      if (r == R_SUCCESS) { f->items[i] = item; return GRO_COALESCED; }
      if (r == R_ITEM_BAD) { /* deleteAt :241-247 */
        memmove(&f->items[i], &f->items[i + 1], (size_t)(f->n - i - 1) * sizeof *f->items);
        f->n--;
      } else if (r == R_PKT_BAD) {
        return GRO_NOOP;
      }
      /* bufs may have been re-pointed only on success; pkt stays valid */
    }
  }
  tcp_insert(t, pkt, plen, src_off, src_off + alen, iph, th, bi);
  return GRO_INSERT;
}

/* gro.go:971-1095 */
static int udp_gro(uint8_t **bufs, size_t *lens, size_t *caps, int offset, int bi, udp_table *t,
                   int v6) {
  const uint8_t *pkt = bufs[bi] + offset;
  size_t plen = lens[bi] - (size_t)offset;
  if (plen > MAX_U16) return GRO_NOOP;
  int iph = (uint8_t)((pkt[0] & 0x0F) * 4);
  if (v6) {
    iph = 40;
    if ((int)be16(pkt + 4) != (int)plen - iph) return GRO_NOOP;
  } else {
    if ((size_t)be16(pkt + 2) != plen) return GRO_NOOP;
  }
  if (plen < (size_t)(iph + UDPH_LEN)) return GRO_NOOP;
  if (!v6) {
    if ((pkt[6] & 0x20) != 0 || (uint8_t)(pkt[6] << 3) != 0 || pkt[7] != 0) return GRO_NOOP;
  }
  uint16_t gso = (uint16_t)(plen - (size_t)iph - UDPH_LEN);
  if (gso < 1) return GRO_NOOP;
  int src_off = v6 ? IPV6_SRC : IPV4_SRC;
  int alen = v6 ? 16 : 4;
  udp_key key = mk_udp_key(pkt, src_off, src_off + alen, iph);
  udp_flow *f = udp_find(t, &key);
  if (!f) {
    udp_insert(t, pkt, plen, src_off, src_off + alen, iph, bi, 0);
    return GRO_INSERT;
  }
  udp_item item = f->items[f->n - 1];
  int can = udp_can_coalesce(pkt, plen, (uint8_t)iph, gso, &item, bufs, lens, offset);
  int bad = 0;
  if (can == CO_APPEND) {
    int r = coalesce_udp(bi, &item, bufs, lens, caps, offset, v6);
    if (r == R_SUCCESS) { f->items[f->n - 1] = item; return GRO_COALESCED; }
    if (r == R_PKT_BAD) bad = 1;
  }
  udp_insert(t, pkt, plen, src_off, src_off + alen, iph, bi, bad);
  return GRO_INSERT;
}

static void encode_vhdr(uint8_t *b, const or_virtio_hdr *h) { /* gro.go:73-82 */
  b[0] = h->flags; b[1] = h->gso_type;
  memcpy(b + 2, &h->hdr_len, 2); memcpy(b + 4, &h->gso_size, 2);
  memcpy(b + 6, &h->csum_start, 2); memcpy(b + 8, &h->csum_offset, 2);
}

/* gro.go:1099-1179 / 1183-1268, one item */
static void apply_item(uint8_t **bufs, size_t *lens, int offset, int bi, int merged, int v6,
                       int is_udp, uint8_t iph, uint8_t l4h, uint16_t gso) {
  or_virtio_hdr h; memset(&h, 0, sizeof h);
  if (!merged) { encode_vhdr(bufs[bi] + offset - VNET_LEN, &h); return; }
  h.flags = F_NEEDS_CSUM;
  h.hdr_len = (uint16_t)(iph + l4h);
  h.gso_size = gso;
  h.csum_start = iph;
  h.csum_offset = is_udp ? 6 : 16;
  uint8_t *pkt = bufs[bi] + offset;
  size_t plen = lens[bi] - (size_t)offset;
  if (is_udp) h.gso_type = GSO_UDP_L4;
  else h.gso_type = v6 ? GSO_TCPV6 : GSO_TCPV4;
  if (v6) {
    put_be16(pkt + 4, (uint16_t)((uint16_t)plen - (uint16_t)iph));
  } else {
    put_be16(pkt + 2, (uint16_t)plen);
    pkt[10] = 0; pkt[11] = 0;
    put_be16(pkt + 10, (uint16_t)~or_checksum(pkt, iph, 0));
  }
  encode_vhdr(bufs[bi] + offset - VNET_LEN, &h);
  if (is_udp) put_be16(pkt + iph + 4, (uint16_t)(plen - iph));
  int alen = v6 ? 16 : 4, aoff = v6 ? IPV6_SRC : IPV4_SRC;
  uint64_t ph = or_pseudo_header_nofold(pkt + aoff, pkt + aoff + alen, (size_t)alen,
                                        is_udp ? PROTO_UDP : PROTO_TCP,
                                        (uint16_t)(plen - iph));
  put_be16(pkt + h.csum_start + h.csum_offset, or_checksum(NULL, 0, ph));
}

/* gro.go:1280-1317 */
static int gro_candidate(const uint8_t *pkt, size_t len, int can_udp) {
  if (len < 28) return 0;
  switch (pkt[0] >> 4) {
    case 4:
      if ((pkt[0] & 0x0F) != 5) return 0;
      if (pkt[9] == PROTO_TCP && len >= 40) return 1;
      if (pkt[9] == PROTO_UDP && can_udp) return 3;
      break;
    case 6:
      if (pkt[6] == PROTO_TCP && len >= 60) return 2;
      if (pkt[6] == PROTO_UDP && len >= 48 && can_udp) return 4;
      break;
  }
  return 0;
}

/* gro.go:1326-1367 */
int or_handle_gro(uint8_t **bufs, size_t *lens, size_t *caps, int n, int offset,
                  int can_udp_gro, int *to_write, int *n_to_write) {
  tcp_table tt = {0};
  udp_table ut = {0};
  int rc = OR_OK;
  *n_to_write = 0;
  for (int i = 0; i < n; i++) {
    if (offset < VNET_LEN || (long)offset > (long)lens[i] - 1) { rc = OR_ERR_INVALID_OFFSET; goto out; }
    int res = GRO_NOOP;
    switch (gro_candidate(bufs[i] + offset, lens[i] - (size_t)offset, can_udp_gro)) {
      case 1: res = tcp_gro(bufs, lens, caps, offset, i, &tt, 0); break;
      case 2: res = tcp_gro(bufs, lens, caps, offset, i, &tt, 1); break;
      case 3: res = udp_gro(bufs, lens, caps, offset, i, &ut, 0); break;
      case 4: res = udp_gro(bufs, lens, caps, offset, i, &ut, 1); break;
    }
    if (res == GRO_NOOP) {
      or_virtio_hdr h; memset(&h, 0, sizeof h);
      encode_vhdr(bufs[i] + offset - VNET_LEN, &h);
    }
    if (res == GRO_NOOP || res == GRO_INSERT) to_write[(*n_to_write)++] = i;
  }
  for (int f = 0; f < tt.n; f++)
    for (int k = 0; k < tt.f[f].n; k++) {
      tcp_item *it = &tt.f[f].items[k];
      apply_item(bufs, lens, offset, it->bufs_index, it->num_merged > 0, it->key.v6, 0,
                 it->iph_len, it->tcph_len, it->gso_size);
    }
  for (int f = 0; f < ut.n; f++)
    for (int k = 0; k < ut.f[f].n; k++) {
      udp_item *it = &ut.f[f].items[k];
      apply_item(bufs, lens, offset, it->bufs_index, it->num_merged > 0, it->key.v6, 1,
                 it->iph_len, UDPH_LEN, it->gso_size);
    }
out:
  for (int f = 0; f < tt.n; f++) free(tt.f[f].items);
  for (int f = 0; f < ut.n; f++) free(ut.f[f].items);
  free(tt.f);
  free(ut.f);
  return rc;
}

/* ====================================================================== */
/* Batch helpers (test / cpu_baseline only).  Modes as in wgcsum.h.         */
/* ====================================================================== */
static void one_pkt(int mode, uint8_t *arena, const or_pkt *p, const uint64_t *initial,
                    uint32_t i, void *out, int inplace) {
  uint8_t *pkt = arena + ((uint64_t)p->off_lo | ((uint64_t)p->off_hi << 32));
  size_t len = p->len;
  int v6 = p->flags & 1;
  uint8_t proto = p->proto;
  size_t aoff = v6 ? IPV6_SRC : IPV4_SRC, alen = v6 ? 16 : 4;
  uint16_t cs = p->csum_start, co = p->csum_offset;
  uint16_t at = (uint16_t)(cs + co); /* u16 field position, gro.go:1391 / :1503 */
  switch (mode) {
    case 0: /* FOLD: checksum(b, initial) */
      ((uint16_t *)out)[i] = or_checksum(pkt, len, initial ? initial[i] : 0);
      break;
    case 1: { /* L4_FILL: gro.go:1469-1488 with the field treated as zero */
      if (cs > len) { ((uint16_t *)out)[i] = 0; break; } /* pkt[cs:] panics: 0, no write */
      uint8_t save0 = pkt[at], save1 = pkt[at + 1];
      pkt[at] = 0; pkt[at + 1] = 0;
      uint64_t ph = or_pseudo_header_nofold(pkt + aoff, pkt + aoff + alen, alen, proto,
                                            (uint16_t)(len - cs));
      uint16_t c = (uint16_t)~or_checksum(pkt + cs, len - cs, ph);
      ((uint16_t *)out)[i] = c;
      /* INPLACE stores into a field inside the packet (WGCS_F_INPLACE) */
      if (inplace && (size_t)at + 2 <= len) put_be16(pkt + at, c);
      else { pkt[at] = save0; pkt[at + 1] = save1; }
      break;
    }
    case 2: /* VALIDATE: checksumValid */
      /* the arena after the packet is its spare capacity; a panic (cs > len) is 0 */
      ((uint8_t *)out)[i] = (uint8_t)(checksum_valid_at(pkt, len, (size_t)-1, cs, proto, v6) == 1);
      break;
    case 3: { /* PARTIAL: gsoNoneChecksum */
      uint8_t save0 = pkt[at], save1 = pkt[at + 1];
      or_gso_none_checksum(pkt, len, cs, co);
      ((uint16_t *)out)[i] = be16(pkt + at);
      if (!inplace) { pkt[at] = save0; pkt[at + 1] = save1; }
      break;
    }
    case 4: { /* IP4HDR: gro.go:1134-1138 */
      uint8_t s10 = pkt[10], s11 = pkt[11];
      pkt[10] = 0; pkt[11] = 0;
      uint16_t c = (uint16_t)~or_checksum(pkt, cs, 0);
      ((uint16_t *)out)[i] = c;
      if (inplace) put_be16(pkt + 10, c);
      else { pkt[10] = s10; pkt[11] = s11; }
      break;
    }
  }
}

void or_checksum_batch(int mode, uint8_t *arena, const or_pkt *pkts, const uint64_t *initial,
                       uint32_t n, void *out, int inplace) {
  for (uint32_t i = 0; i < n; i++) one_pkt(mode, arena, &pkts[i], initial, i, out, inplace);
}

typedef struct { int mode; uint8_t *arena; const or_pkt *pkts; uint32_t lo, hi; void *out; } mt_arg;
static void *mt_worker(void *a_) {
  mt_arg *a = (mt_arg *)a_;
  for (uint32_t i = a->lo; i < a->hi; i++) one_pkt(a->mode, a->arena, &a->pkts[i], NULL, i, a->out, 0);
  return NULL;
}
void or_checksum_batch_mt(int mode, uint8_t *arena, const or_pkt *pkts, uint32_t n, void *out,
                          int threads) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t th[256];
  mt_arg args[256];
  for (int t = 0; t < threads; t++) {
    args[t].mode = mode; args[t].arena = arena; args[t].pkts = pkts; args[t].out = out;
    args[t].lo = (uint32_t)((uint64_t)n * t / threads);
    args[t].hi = (uint32_t)((uint64_t)n * (t + 1) / threads);
    pthread_create(&th[t], NULL, mt_worker, &args[t]);
  }
  for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
}
