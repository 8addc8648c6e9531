// sanitize_driver.cpp -- TEST INFRASTRUCTURE: the host-side C/C++ of this
// repository under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md
// §5), built with g++ by tests/test_sanitize.py:
//   * the GRO planner (wireguard_amd/csrc/wgcs_gro_plan.h), driven exactly as
//     wgcs_handle_gro drives it (gro_host.cpp): candidates, a plan on assumed
//     checksums, a second plan on the real bits when a consulted bit is false;
//     its toWrite, slice lengths and prepend permutation are compared with the
//     oracle's handleGRO (/root/reference/tun/gro.go:1326-1367) on a copy;
//   * the GSO output-layout bounds (wgcs_host.h: gso_out_layout,
//     gso_split_need, gso_touches_caller_bytes) against what the oracle's
//     handleVirtioRead / gsoSplit (tun/tun.go:514-632, gro.go:1373-1493)
//     actually writes;
//   * the C oracle itself (oracle/wg_oracle.c, compiled into this binary with
//     the same sanitizers) on every case.
// Reads a corpus written by tests/test_sanitize.py (records below) from
// argv[1]; exit 0 and "sanitize_driver: ok ..." when every record agrees,
// 1 on a mismatch; a sanitizer report aborts the run (-fno-sanitize-recover).
//
// Records (little-endian):
//   u32 tag = 1  GRO call: u32 n, i32 offset, u32 can_udp,
//                n x {u32 len, u32 cap, u8 bytes[len]}   (bufs[i][:len], cap(bufs[i]))
//   u32 tag = 2  handleVirtioRead: u32 n_read, u32 cap, u8 rb[cap], u32 nbufs, u32 bufsize, u32 fill, i32 offset
//   u32 tag = 3  gsoSplit: as tag 2, then u8 hdr[10] (virtio header fields, LE), u32 is_v6
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "wgcs_gro_plan.h"
#include "wgcs_host.h"

extern "C" {
#include "wg_oracle.h"
}

using namespace wgcs;
using namespace wgcs::gro;

namespace {

struct Reader {
  std::vector<uint8_t> d;
  size_t p = 0;
  bool more() const { return p < d.size(); }
  uint32_t u32() {
    uint32_t v;
    if (p + 4 > d.size()) { fprintf(stderr, "sanitize_driver: truncated corpus\n"); exit(2); }
    memcpy(&v, &d[p], 4);
    p += 4;
    return v;
  }
  void bytes(uint8_t* out, size_t n) {
    if (p + n > d.size()) { fprintf(stderr, "sanitize_driver: truncated corpus\n"); exit(2); }
    if (n) memcpy(out, &d[p], n);
    p += n;
  }
};

int fail(int rec, const char* what) {
  fprintf(stderr, "sanitize_driver: record %d: %s\n", rec, what);
  return 1;
}

// One Write call through the planner, as wgcs_handle_gro (gro_host.cpp:66-150) runs it.
int gro_call(Reader& R, int rec) {
  const int n = (int)R.u32();
  const int offset = (int)R.u32();
  const int can_udp = (int)R.u32();
  std::vector<std::vector<uint8_t>> mem_p(n), mem_o(n);
  std::vector<uint8_t*> bp(n), bo(n);
  std::vector<size_t> lp(n), cp(n), lo(n), co(n);
  for (int i = 0; i < n; ++i) {
    const uint32_t len = R.u32(), cap = R.u32();
    if (len > cap) return fail(rec, "corpus: len > cap");
    mem_p[i].assign(cap ? cap : 1, 0);  // a non-empty allocation so a 0-cap slice still has an address
    R.bytes(mem_p[i].data(), len);
    mem_o[i] = mem_p[i];
    bp[i] = mem_p[i].data();
    bo[i] = mem_o[i].data();
    lp[i] = lo[i] = len;
    cp[i] = co[i] = cap;
  }
  // ---- the oracle on its own copy
  std::vector<int> tw_o(n > 0 ? n : 1);
  int ntw_o = 0;
  const int rc_o = or_handle_gro(bo.data(), lo.data(), co.data(), n, offset, can_udp, tw_o.data(), &ntw_o);
  // ---- the planner
  int n_eff = n;
  for (int i = 0; i < n; ++i)
    if (offset < kVnetLen || (long)offset > (long)lp[i] - 1) {
      n_eff = i;
      break;
    }
  const bool bad_offset = n_eff < n;
  std::vector<const uint8_t*> orig(n, nullptr);
  std::vector<int> cand(n, NOT_CAND);
  std::vector<uint64_t> stage_off(n, 0);
  std::vector<uint8_t> assume(n, 0), real(n, 0);
  uint64_t stage = 0;
  for (int i = 0; i < n_eff; ++i) {
    orig[i] = bp[i] + offset;
    cand[i] = gro_candidate(orig[i], lp[i] - offset, can_udp != 0);
    if (cand[i] != NOT_CAND) {
      stage_off[i] = stage;
      stage += (lp[i] - offset + 15) & ~(size_t)15;
      assume[i] = 1;
      const bool v6 = cand[i] == TCP6 || cand[i] == UDP6, udp = cand[i] == UDP4 || cand[i] == UDP6;
      real[i] = (uint8_t)or_checksum_valid(orig[i], lp[i] - offset, v6 ? 40 : 20, udp ? 17 : 6, v6);
    }
  }
  const std::vector<uint8_t*> b0(bp);
  const std::vector<size_t> l0(lp), c0(cp);
  Planner P;
  init_planner(P, bp.data(), lp.data(), cp.data(), n_eff, offset, orig, assume);
  Plan pl;
  make_plan(P, cand, stage_off, n_eff, bad_offset, pl);
  bool redo = false;
  for (int i = 0; i < n_eff && !redo; ++i) redo = P.consulted[i] && !real[i];
  if (redo) {
    bp = b0;
    lp = l0;
    cp = c0;
    Planner Q;
    init_planner(Q, bp.data(), lp.data(), cp.data(), n_eff, offset, orig, real);
    pl = Plan();
    make_plan(Q, cand, stage_off, n_eff, bad_offset, pl);
  }
  // ---- what the planner decided vs the oracle
  const int rc_p = bad_offset ? OR_ERR_INVALID_OFFSET : 0;
  if (rc_p != rc_o) return fail(rec, "GRO status differs");
  if ((int)pl.to_write.size() != ntw_o) return fail(rec, "GRO toWrite count differs");
  for (int k = 0; k < ntw_o; ++k)
    if (pl.to_write[k] != tw_o[k]) return fail(rec, "GRO toWrite differs");
  for (int i = 0; i < n; ++i) {
    if (lp[i] != lo[i] || cp[i] != co[i]) return fail(rec, "GRO slice length / capacity differs");
    // the same prepend permutation: slot i holds the same original buffer on both sides
    const int jp = (int)(std::find(b0.begin(), b0.end(), bp[i]) - b0.begin());
    int jo = -1;
    for (int j = 0; j < n; ++j)
      if (bo[i] == mem_o[j].data()) jo = j;
    if (jp != jo) return fail(rec, "GRO slice permutation differs");
  }
  // ---- the plan's own bounds: every piece inside the staged packets, every
  // item inside the output region
  for (const GroSeg& sg : pl.segs)
    if ((uint64_t)sg.src_off + sg.len > stage || (uint64_t)sg.dst_off + sg.len > pl.out_bytes)
      return fail(rec, "GRO plan piece out of bounds");
  for (const GroItem& it : pl.items)
    if (it.out_off + kVnetLen + it.pkt_len > pl.out_bytes) return fail(rec, "GRO plan item out of bounds");
  return 0;
}

// One handleVirtioRead (tag 2) or gsoSplit (tag 3) through the oracle, and the
// host-side layout bounds the GPU entry points size their staging with.
int gso_call(Reader& R, int rec, bool raw) {
  const uint32_t n_read = R.u32(), cap = R.u32();
  std::vector<uint8_t> rb(cap ? cap : 1, 0);
  R.bytes(rb.data(), cap);
  const int nbufs = (int)R.u32();
  const uint32_t bufsize = R.u32(), fill = R.u32();
  const int offset = (int)R.u32();
  or_virtio_hdr h;
  memset(&h, 0, sizeof h);
  int is_v6 = 0;
  if (raw) {
    uint8_t hb[10];
    R.bytes(hb, 10);
    h.flags = hb[0];
    h.gso_type = hb[1];
    h.hdr_len = (uint16_t)(hb[2] | (hb[3] << 8));
    h.gso_size = (uint16_t)(hb[4] | (hb[5] << 8));
    h.csum_start = (uint16_t)(hb[6] | (hb[7] << 8));
    h.csum_offset = (uint16_t)(hb[8] | (hb[9] << 8));
    is_v6 = (int)R.u32();
  }
  if (n_read > cap) return fail(rec, "corpus: n_read > cap");
  std::vector<std::vector<uint8_t>> mem(nbufs, std::vector<uint8_t>(bufsize ? bufsize : 1, (uint8_t)fill));
  std::vector<uint8_t*> bufs(nbufs);
  std::vector<size_t> lens(nbufs, bufsize);
  for (int i = 0; i < nbufs; ++i) bufs[i] = mem[i].data();
  std::vector<int> sizes(nbufs > 0 ? nbufs : 1, 0);
  int nout = 0, rc;
  // the virtio header the layout helpers read: the read's own (handleVirtioRead)
  // or the caller's (gsoSplit, a RAW job: [hdr | readBuf])
  std::vector<uint8_t> vb;
  uint32_t jflags = 0;
  if (raw) {
    vb.resize(10 + n_read);
    vb[0] = h.flags;
    vb[1] = h.gso_type;
    memcpy(&vb[2], &h.hdr_len, 2);
    memcpy(&vb[4], &h.gso_size, 2);
    memcpy(&vb[6], &h.csum_start, 2);
    memcpy(&vb[8], &h.csum_offset, 2);
    if (n_read) memcpy(&vb[10], rb.data(), n_read);
    jflags = WGCS_GSO_JOB_RAW | (is_v6 ? WGCS_GSO_JOB_V6 : 0u);
    rc = or_gso_split_cap(rb.data(), n_read, cap, h, bufs.data(), lens.data(), nbufs, sizes.data(), offset, is_v6,
                          &nout);
  } else {
    vb.assign(rb.begin(), rb.begin() + n_read);
    rc = or_handle_virtio_read_cap(rb.data(), n_read, cap, bufs.data(), lens.data(), nbufs, sizes.data(), offset,
                                   &nout);
  }
  uint32_t pitch = 0, segs = 0;
  gso_out_layout(vb.data(), vb.size(), jflags, (uint32_t)nbufs, &pitch, &segs);
  (void)gso_touches_caller_bytes(vb.data(), vb.size(), jflags);
  if (rc == 0 || rc == OR_ERR_TOO_MANY_SEGMENTS) {
    const int written = rc == OR_ERR_TOO_MANY_SEGMENTS ? nbufs : nout;
    if ((uint32_t)written > segs) return fail(rec, "GSO layout: more segments than gso_out_layout bounds");
    for (int i = 0; i < written && i < nbufs; ++i) {
      if ((uint32_t)sizes[i] > pitch) return fail(rec, "GSO layout: a segment larger than the packed pitch");
      const bool last = i + 1 == written;
      if (!raw && vb.size() > 10 && vb[1] == 0) continue;  // GSO_NONE: the packet only
      if (gso_split_need(vb.data(), vb.size(), jflags, (size_t)sizes[i], last) + (size_t)offset > bufsize &&
          rc == 0)
        return fail(rec, "GSO: the oracle wrote a segment the host bound says does not fit");
    }
  }
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: sanitize_driver <corpus>\n");
    return 2;
  }
  FILE* f = fopen(argv[1], "rb");
  if (!f) {
    perror(argv[1]);
    return 2;
  }
  Reader R;
  uint8_t buf[1 << 16];
  size_t got;
  while ((got = fread(buf, 1, sizeof buf, f)) > 0) R.d.insert(R.d.end(), buf, buf + got);
  fclose(f);
  int counts[4] = {0, 0, 0, 0};
  for (int rec = 0; R.more(); ++rec) {
    const uint32_t tag = R.u32();
    int bad;
    if (tag == 1) bad = gro_call(R, rec);
    else if (tag == 2 || tag == 3) bad = gso_call(R, rec, tag == 3);
    else return fail(rec, "unknown record tag");
    if (bad) return 1;
    counts[tag]++;
  }
  printf("sanitize_driver: ok (%d handleGRO calls through the planner, %d handleVirtioRead, %d gsoSplit)\n",
         counts[1], counts[2], counts[3]);
  return 0;
}
