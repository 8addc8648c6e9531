/*
 * abi_harness.c -- TEST INFRASTRUCTURE: the C ABI (include/wgcsum.h) driven
 * from plain C, the way the cgo shims of INTEGRATION.md call it (no Python,
 * no torch in the process), checked byte for byte against the CPU oracle
 * (oracle/wg_oracle.c, linked in as the checker).
 *
 *   Tun.Read:  handleVirtioRead (tun/tun.go:514-632) through
 *              wgcs_handle_virtio_read_cap, with readBuf's spare capacity;
 *   Tun.Write: handleGRO (tun/gro.go:1326-1367) through wgcs_handle_gro on the
 *              segments the split produced (they coalesce back);
 *   checksumValid (gro.go:554-612) through wgcs_checksum_valid_cap on each;
 *   the same read through the read stager (push / submit / wait / copy_out)
 *   and the segments through the write stager (its write(2) images);
 *   conn: splitMessages (conn/bind.go:542-597) on a recvmmsg batch.
 *
 * Exit status 0 and "abi_harness: ok" on success; 1 with a message otherwise.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/wgcsum.h"
#include "../../oracle/wg_oracle.h"

enum { NBUFS = 128, OFFSET = 16, CAP = 65535 + OFFSET, SPARE = 48 };

static uint32_t lcg = 12345u;
static uint8_t rnd8(void) { lcg = lcg * 1664525u + 1013904223u; return (uint8_t)(lcg >> 24); }

#define CHECK(cond, ...)                                \
  do {                                                  \
    if (!(cond)) {                                      \
      fprintf(stderr, "abi_harness: FAIL: " __VA_ARGS__); \
      fprintf(stderr, "\n");                            \
      return 1;                                         \
    }                                                   \
  } while (0)

/* [10-byte virtio header | IPv4 | TCP | payload]: one TCPv4 super-packet
 * whose split the reference performs (gsoSize 1460). */
static size_t make_read(uint8_t *rb, size_t total) {
  memset(rb, 0, total);
  rb[0] = 1;                              /* VIRTIO_NET_HDR_F_NEEDS_CSUM */
  rb[1] = 1;                              /* GSO_TCPV4 */
  rb[2] = 40; rb[3] = 0;                  /* hdrLen (recomputed by handleVirtioRead) */
  rb[4] = 1460 & 0xFF; rb[5] = 1460 >> 8; /* gsoSize */
  rb[6] = 20; rb[7] = 0;                  /* csumStart */
  rb[8] = 16; rb[9] = 0;                  /* csumOffset */
  uint8_t *ip = rb + 10;
  const size_t plen = total - 10;
  ip[0] = 0x45; ip[2] = (uint8_t)(plen >> 8); ip[3] = (uint8_t)plen;
  ip[4] = 0x12; ip[5] = 0x34; ip[6] = 0x40; ip[8] = 64; ip[9] = 6;
  for (int k = 12; k < 20; ++k) ip[k] = rnd8();
  uint8_t *tcp = ip + 20;
  tcp[0] = 0x0F; tcp[1] = 0xA0; tcp[2] = 0xCA; tcp[3] = 0x6C;
  for (int k = 4; k < 12; ++k) tcp[k] = rnd8();
  tcp[12] = 0x50; tcp[13] = 0x18; tcp[14] = 0xFF; tcp[15] = 0xFF;
  for (size_t k = 40; k < plen; ++k) ip[k] = rnd8();
  return total;
}

int main(void) {
  wgcs_ctx *ctx = NULL;
  int rc = wgcs_init(0, &ctx);
  CHECK(rc == WGCS_OK, "wgcs_init: %d (%s)", rc, wgcs_strerror(rc));
  CHECK(wgcs_abi_version() == WGCS_ABI_VERSION, "ABI version");

  /* ---- Tun.Read: handleVirtioRead with spare capacity after the read ---- */
  const size_t total = 10 + 65535, cap = total + SPARE;
  uint8_t *rb_p = malloc(cap), *rb_o = malloc(cap);
  make_read(rb_p, total);
  for (size_t k = total; k < cap; ++k) rb_p[k] = rnd8();
  memcpy(rb_o, rb_p, cap);
  uint8_t *rb_pristine = malloc(cap);
  memcpy(rb_pristine, rb_p, cap);
  uint8_t *bp[NBUFS], *bo[NBUFS];
  size_t lens[NBUFS];
  for (int i = 0; i < NBUFS; ++i) {
    bp[i] = malloc(CAP);
    bo[i] = malloc(CAP);
    memset(bp[i], 0xA5, CAP);
    memset(bo[i], 0xA5, CAP);
    lens[i] = CAP;
  }
  int sz_p[NBUFS] = {0}, sz_o[NBUFS] = {0}, n_p = 0, n_o = 0;
  rc = wgcs_handle_virtio_read_cap(ctx, rb_p, total, cap, bp, lens, NBUFS, sz_p, OFFSET, &n_p);
  const int rc_o = or_handle_virtio_read_cap(rb_o, total, cap, bo, lens, NBUFS, sz_o, OFFSET, &n_o);
  CHECK(rc == rc_o && n_p == n_o, "handleVirtioRead: rc %d / %d, n %d / %d", rc, rc_o, n_p, n_o);
  CHECK(n_p == 45, "handleVirtioRead: %d segments", n_p);
  CHECK(memcmp(rb_p, rb_o, cap) == 0, "readBuf mutation differs");
  for (int i = 0; i < NBUFS; ++i) {
    CHECK(i >= n_p || sz_p[i] == sz_o[i], "size %d", i);
    CHECK(memcmp(bp[i], bo[i], CAP) == 0, "buffer %d differs", i);
  }

  /* the split's segments, kept for the stager checks below */
  uint8_t *seg[NBUFS];
  for (int i = 0; i < NBUFS; ++i) {
    seg[i] = malloc(CAP);
    memcpy(seg[i], bo[i], CAP);
  }

  /* ---- Tun.Read through the read stager: push, submit, wait, copy_out ---- */
  {
    wgcs_stager *st = NULL;
    rc = wgcs_stager_create(ctx, 2, 4, 4 * (total + 64), NBUFS, CAP - OFFSET, &st);
    CHECK(rc == WGCS_OK, "wgcs_stager_create: %d", rc);
    int idx = -1;
    uint64_t batch = 0;
    CHECK(wgcs_stager_push(st, rb_pristine, total, &idx) == WGCS_OK && idx == 0, "stager push");
    CHECK(wgcs_stager_submit(st, &batch) == WGCS_OK && wgcs_stager_wait(st, batch) == WGCS_OK, "stager submit/wait");
    uint8_t *sb[NBUFS];
    int ssz[NBUFS] = {0}, sn = 0;
    for (int i = 0; i < NBUFS; ++i) {
      sb[i] = malloc(CAP);
      memset(sb[i], 0xA5, CAP);
    }
    rc = wgcs_stager_copy_out(st, batch, 0, sb, lens, NBUFS, ssz, OFFSET, &sn);
    CHECK(rc == WGCS_OK && sn == n_o, "stager copy_out: rc %d n %d", rc, sn);
    for (int i = 0; i < NBUFS; ++i) {
      CHECK(i >= sn || ssz[i] == sz_o[i], "stager size %d", i);
      CHECK(memcmp(sb[i], seg[i], CAP) == 0, "stager buffer %d differs", i);
      free(sb[i]);
    }
    CHECK(wgcs_stager_destroy(st) == WGCS_OK, "stager destroy");
  }

  /* ---- Tun.Write through the write stager: the write(2) images ---- */
  {
    wgcs_wstager *ws = NULL;
    rc = wgcs_wstager_create(ctx, 2, 4, 4 * NBUFS, 4 * NBUFS * 1600, &ws);
    CHECK(rc == WGCS_OK, "wgcs_wstager_create: %d", rc);
    size_t wl[NBUFS], wc[NBUFS], ol[NBUFS], oc[NBUFS];
    uint8_t *wb[NBUFS], *ob[NBUFS];
    for (int i = 0; i < n_o; ++i) {
      wb[i] = malloc(CAP);
      ob[i] = malloc(CAP);
      memcpy(wb[i], seg[i], CAP);
      memcpy(ob[i], seg[i], CAP);
      wl[i] = ol[i] = (size_t)(OFFSET + sz_o[i]);
      wc[i] = oc[i] = CAP;
    }
    int widx = -1;
    uint64_t wbatch = 0;
    rc = wgcs_wstager_push(ws, (const uint8_t *const *)wb, wl, wc, n_o, OFFSET, 1, &widx);
    CHECK(rc == WGCS_OK && widx == 0, "wstager push: %d", rc);
    CHECK(wgcs_wstager_submit(ws, &wbatch) == WGCS_OK && wgcs_wstager_wait(ws, wbatch) == WGCS_OK, "wstager submit/wait");
    int wst = -1, nw = -1, wtw[NBUFS];
    const uint8_t *imgs[NBUFS];
    size_t ilen[NBUFS];
    rc = wgcs_wstager_result(ws, wbatch, widx, &wst, &nw, wtw, imgs, ilen);
    int otw[NBUFS], onw = -1;
    uint8_t *obp[NBUFS];
    memcpy(obp, ob, sizeof(uint8_t *) * (size_t)n_o);
    const int orc = or_handle_gro(obp, ol, oc, n_o, OFFSET, 1, otw, &onw);
    CHECK(rc == WGCS_OK && wst == orc && nw == onw, "wstager result: rc %d status %d/%d writes %d/%d", rc, wst, orc,
          nw, onw);
    for (int k = 0; k < nw; ++k) {
      const int i = otw[k];
      CHECK(wtw[k] == i, "wstager toWrite[%d]", k);
      /* the write(2) image: the virtio header and the packet, bufs[i][offset-10:len] */
      CHECK(ilen[k] == ol[i] - (OFFSET - 10) && memcmp(imgs[k], obp[i] + OFFSET - 10, ilen[k]) == 0,
            "wstager image %d differs", k);
    }
    CHECK(wgcs_wstager_destroy(ws) == WGCS_OK, "wstager destroy");
    for (int i = 0; i < n_o; ++i) {
      free(wb[i]);
      free(ob[i]);
    }
  }

  /* ---- checksumValid of every segment (any capacity: the buffer's) ---- */
  for (int i = 0; i < n_p; ++i) {
    int valid = -1;
    rc = wgcs_checksum_valid_cap(ctx, bp[i] + OFFSET, (size_t)sz_p[i], CAP - OFFSET, 20, 6, 0, &valid);
    CHECK(rc == WGCS_OK && valid == 1, "checksumValid segment %d: rc %d valid %d", i, rc, valid);
    CHECK(or_checksum_valid(bo[i] + OFFSET, (size_t)sz_o[i], 20, 6, 0) == 1, "oracle checksumValid %d", i);
  }

  /* ---- Tun.Write: handleGRO over the segments (Go slices: len, cap) ---- */
  size_t gl_p[NBUFS], gc_p[NBUFS], gl_o[NBUFS], gc_o[NBUFS];
  for (int i = 0; i < n_p; ++i) {
    gl_p[i] = gl_o[i] = (size_t)(OFFSET + sz_p[i]);
    gc_p[i] = gc_o[i] = CAP;
  }
  int tw_p[NBUFS], tw_o[NBUFS], ntw_p = -1, ntw_o = -1;
  uint8_t *gp[NBUFS], *go[NBUFS];
  memcpy(gp, bp, sizeof gp);
  memcpy(go, bo, sizeof go);
  rc = wgcs_handle_gro(ctx, gp, gl_p, gc_p, n_p, OFFSET, 1, tw_p, &ntw_p);
  const int grc = or_handle_gro(go, gl_o, gc_o, n_o, OFFSET, 1, tw_o, &ntw_o);
  CHECK(rc == grc && ntw_p == ntw_o, "handleGRO: rc %d / %d, writes %d / %d", rc, grc, ntw_p, ntw_o);
  CHECK(ntw_p >= 1 && ntw_p < n_p, "handleGRO coalesced %d segments into %d writes", n_p, ntw_p);
  for (int k = 0; k < ntw_p; ++k) CHECK(tw_p[k] == tw_o[k], "toWrite[%d]", k);
  for (int i = 0; i < n_p; ++i) {
    /* prepends swap slices (gro.go:696-697): the same permutation on both sides */
    int j = 0;
    while (j < n_p && gp[i] != bp[j]) ++j;
    CHECK(j < n_p && go[i] == bo[j], "slice %d moved differently", i);
    CHECK(gl_p[i] == gl_o[i] && gc_p[i] == gc_o[i], "slice %d len/cap", i);
  }
  for (int i = 0; i < n_p; ++i) CHECK(memcmp(bp[i], bo[i], CAP) == 0, "GRO buffer %d differs", i);

  /* ---- handleGRO with a zero-capacity buffer after two segments: the cgo
   * shim passes a NULL pointer with len = cap = 0 for it,
   * the reference returns "invalid offset" at that buffer (gro.go:1334-1337)
   * after the earlier ones went through tcpGRO, and apply* never runs ---- */
  {
    uint8_t *zp[3], *zo[3];
    size_t zl_p[3], zc_p[3], zl_o[3], zc_o[3];
    for (int i = 0; i < 2; ++i) {
      zp[i] = malloc(CAP);
      zo[i] = malloc(CAP);
      memcpy(zp[i], seg[i], CAP);
      memcpy(zo[i], seg[i], CAP);
      zl_p[i] = zl_o[i] = (size_t)(OFFSET + sz_o[i]);
      zc_p[i] = zc_o[i] = CAP;
    }
    zp[2] = zo[2] = NULL;
    zl_p[2] = zl_o[2] = zc_p[2] = zc_o[2] = 0;
    int ztw_p[3], ztw_o[3], zn_p = -1, zn_o = -1;
    rc = wgcs_handle_gro(ctx, zp, zl_p, zc_p, 3, OFFSET, 1, ztw_p, &zn_p);
    const int zrc = or_handle_gro(zo, zl_o, zc_o, 3, OFFSET, 1, ztw_o, &zn_o);
    CHECK(rc == WGCS_ERR_INVALID_OFFSET && zrc == OR_ERR_INVALID_OFFSET,
          "zero-capacity buffer: rc %d / %d, want invalid offset", rc, zrc);
    CHECK(zn_p == zn_o, "zero-capacity buffer: writes %d / %d", zn_p, zn_o);
    for (int k = 0; k < zn_p; ++k) CHECK(ztw_p[k] == ztw_o[k], "zero-capacity buffer: toWrite[%d]", k);
    CHECK(zp[2] == NULL && zl_p[2] == 0 && zc_p[2] == 0, "zero-capacity buffer: its slice header changed");
    CHECK(zo[2] == NULL && zl_o[2] == 0 && zc_o[2] == 0, "zero-capacity buffer: oracle slice header changed");
    for (int i = 0; i < 2; ++i) {
      CHECK(zl_p[i] == zl_o[i] && zc_p[i] == zc_o[i], "zero-capacity call: slice %d len/cap", i);
      CHECK(memcmp(zp[i], zo[i], CAP) == 0, "zero-capacity call: buffer %d differs", i);
    }
    for (int i = 0; i < 2; ++i) {
      free(zp[i]);
      free(zo[i]);
    }
  }

  /* ---- conn: splitMessages on a recvmmsg batch (2 UDP_GRO datagrams) ---- */
  {
    enum { NM = 128, FIRST = 126, BL = 65535, SEG = 1452, NSEG = 45 };
    uint8_t *mp[NM], *mo[NM], cm[NM][24];
    const uint8_t *oobs[NM];
    size_t nns[NM];
    int ns_p[NM], ns_o[NM], asrc[NM];
    or_msg msgs[NM];
    for (int i = 0; i < NM; ++i) {
      mp[i] = malloc(BL);
      mo[i] = malloc(BL);
      for (int k = 0; k < BL; ++k) mp[i][k] = rnd8();
      memcpy(mo[i], mp[i], BL);
      memset(cm[i], 0, sizeof cm[i]);
      nns[i] = 0;
      ns_p[i] = ns_o[i] = 0;
      if (i >= FIRST) { /* a UDP_GRO cmsg {Len 18, SOL_UDP 17, UDP_GRO 104, gso} (conn/gso.go:55-64) */
        const uint64_t hl = 18;
        const int32_t lvl = 17, typ = 104;
        const uint16_t g = SEG;
        memcpy(cm[i], &hl, 8);
        memcpy(cm[i] + 8, &lvl, 4);
        memcpy(cm[i] + 12, &typ, 4);
        memcpy(cm[i] + 16, &g, 2);
        nns[i] = 24;
        ns_p[i] = ns_o[i] = SEG * NSEG;
      }
      oobs[i] = cm[i];
      msgs[i].buf = mo[i];
      msgs[i].buf_len = msgs[i].buf_cap = BL;
      msgs[i].n = ns_o[i];
      msgs[i].oob = cm[i];
      msgs[i].oob_len = msgs[i].oob_cap = 24;
      msgs[i].nn = (int)nns[i];
      msgs[i].addr = i;
    }
    int np_p = -1, np_o = -1;
    rc = wgcs_split_messages(ctx, mp, BL, ns_p, oobs, nns, NM, FIRST, asrc, &np_p);
    const int src = or_split_messages(msgs, NM, FIRST, &np_o);
    CHECK(rc == src && np_p == np_o && np_p == 2 * NSEG, "splitMessages: rc %d / %d, n %d / %d", rc, src, np_p, np_o);
    for (int i = 0; i < NM; ++i) {
      CHECK(ns_p[i] == msgs[i].n && asrc[i] == msgs[i].addr, "splitMessages msg %d", i);
      CHECK(memcmp(mp[i], mo[i], BL) == 0, "splitMessages buffer %d differs", i);
      free(mp[i]);
      free(mo[i]);
    }
  }

  /* ---- the error contract: a bad mode names itself, per thread ---- */
  rc = wgcs_checksum_batch(ctx, 99, 0, NULL, NULL, NULL, 1, NULL, NULL);
  CHECK(rc == WGCS_ERR_INVALID_ARG && strstr(wgcs_last_error(ctx), "99"), "error message: %s", wgcs_last_error(ctx));

  for (int i = 0; i < NBUFS; ++i) {
    free(bp[i]);
    free(bo[i]);
    free(seg[i]);
  }
  free(rb_pristine);
  free(rb_p);
  free(rb_o);
  CHECK(wgcs_destroy(ctx) == WGCS_OK, "wgcs_destroy");
  printf("abi_harness: ok (handleVirtioRead 45 segments, read stager, write stager, checksumValid x%d, handleGRO %d "
         "writes, splitMessages 90 packets, bit-exact)\n", n_p, ntw_p);
  return 0;
}
