/*
 * wg_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the muhtutorials/wireguard `tun` package hot path
 * (tun/checksum.go, tun/gro.go, tun/tun.go:514-632), used as the parity
 * checker for the HIP product in wireguard_amd/.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * It is never linked into, called by, or used as a fallback for the product.
 *
 * Parity pinning: the reference ships no tests, fixtures or golden vectors and
 * its Go toolchain is absent here, so the reference cannot be run.  This
 * restatement is pinned by independent known-answer vectors (RFC 1071 §3,
 * the classic IPv4 header example, a pseudo-header example) and by a
 * closed-form cross-check (tests/test_oracle.py).  It is NOT pinned by outputs
 * of the reference itself: "parity unpinned" in the sense of the task
 * contract.
 *
 * Byte order: the reference uses binary.NativeEndian; this restatement
 * assumes a little-endian host (x86-64), as the reference does in practice.
 */
#ifndef WG_ORACLE_H
#define WG_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes: identical values to include/wgcsum.h */
#define OR_OK 0
#define OR_ERR_SHORT_BUFFER (-2)
#define OR_ERR_TOO_MANY_SEGMENTS (-3)
#define OR_ERR_INVALID_OFFSET (-4)
#define OR_ERR_UNSUPPORTED_GSO (-5)
#define OR_ERR_IP_GSO_MISMATCH (-6)
#define OR_ERR_BAD_IP_VERSION (-7)
#define OR_ERR_PACKET_TOO_SHORT (-8)
#define OR_ERR_TCP_HDR_LEN (-9)
#define OR_ERR_HDR_LEN (-10)
#define OR_ERR_CSUM_OFFSET (-11)
#define OR_ERR_READ_OVERFLOW (-12)
#define OR_ERR_OUT_OF_RANGE (-13) /* reference would panic (slice out of range) */
#define OR_ERR_CMSG (-16)           /* "error parsing socket control message: %w"  conn/gso.go:45 */
#define OR_ERR_SPLIT_OVERFLOW (-17) /* "splitting coalesced packet resulted in overflow" conn/bind.go:565 */

/* conn/bind.go:25-36 */
#define OR_MAX_IPV4_PAYLOAD ((1 << 16) - 1 - 20 - 8)
#define OR_MAX_IPV6_PAYLOAD ((1 << 16) - 1 - 8)
#define OR_MAX_UDP_SEGMENTS 64

typedef struct or_virtio_hdr {
  uint8_t flags;
  uint8_t gso_type;
  uint16_t hdr_len;
  uint16_t gso_size;
  uint16_t csum_start;
  uint16_t csum_offset;
} or_virtio_hdr;

/* checksum.go:8-120 */
uint64_t or_checksum_nofold(const uint8_t *b, size_t n, uint64_t initial);
/* checksum.go:152-167 */
uint16_t or_checksum(const uint8_t *b, size_t n, uint64_t initial);
/* checksum.go:127-150 */
uint64_t or_pseudo_header_nofold(const uint8_t *src, const uint8_t *dst,
                                 size_t addr_len, uint8_t proto,
                                 uint16_t total_len);
/* gro.go:554-612 */
int or_checksum_valid(const uint8_t *pkt, size_t len, uint8_t iph_len,
                      uint8_t proto, int is_v6);
/* the same with cap(pkt) >= len: the address slices may read pkt[len, cap);
 * OR_ERR_OUT_OF_RANGE where Go panics (past cap, or iph_len > len) */
int or_checksum_valid_cap(const uint8_t *pkt, size_t len, size_t cap, uint8_t iph_len,
                          uint8_t proto, int is_v6);
/* gro.go:1497-1517 (in place on read_buf) */
int or_gso_none_checksum(uint8_t *read_buf, size_t len, uint16_t csum_start,
                         uint16_t csum_offset);
/* gro.go:1373-1493.  bufs[i] has buf_lens[i] bytes. */
int or_gso_split(uint8_t *read_buf, size_t len, or_virtio_hdr hdr,
                 uint8_t *const *bufs, const size_t *buf_lens, int nbufs,
                 int *sizes, int offset, int is_v6, int *n_out);
/* the same with cap(readBuf): read_buf[len, cap) is its spare capacity, which
 * the pseudo-header address slices may reach (gro.go:1471-1477) */
int or_gso_split_cap(uint8_t *read_buf, size_t len, size_t cap, or_virtio_hdr hdr,
                     uint8_t *const *bufs, const size_t *buf_lens, int nbufs,
                     int *sizes, int offset, int is_v6, int *n_out);
/* bytes of bufs[i][offset:] a gsoSplit segment of pkt_len bytes writes */
size_t or_gso_split_need(or_virtio_hdr hdr, int is_v6, size_t pkt_len, int last);
/* tun/tun.go:514-632.  read_buf starts with the 10-byte virtio header. */
int or_handle_virtio_read(uint8_t *read_buf, size_t n, uint8_t *const *bufs,
                          const size_t *buf_lens, int nbufs, int *sizes,
                          int offset, int *n_out);
/* the same with cap(readBuf) >= n (Tun.Read passes tun.readBuf[:n]) */
int or_handle_virtio_read_cap(uint8_t *read_buf, size_t n, size_t cap, uint8_t *const *bufs,
                              const size_t *buf_lens, int nbufs, int *sizes,
                              int offset, int *n_out);
/* gro.go:1326-1367 (+ tcpGRO/udpGRO/coalesce/apply).  bufs[i] is a Go slice:
 * lens[i] = len(bufs[i]), caps[i] = cap(bufs[i]).  bufs/lens/caps are updated
 * in place (appends grow lens[i]; prepends swap entries), to_write receives
 * the indices to write. */
int or_handle_gro(uint8_t **bufs, size_t *lens, size_t *caps, int n,
                  int offset, int can_udp_gro, int *to_write,
                  int *n_to_write);

/* Batch helpers used by tests and by bench.py's cpu_baseline leg. */
typedef struct or_pkt { /* same layout as wgcs_pkt (include/wgcsum.h) */
  uint32_t off_lo;
  uint16_t off_hi;
  uint8_t proto;
  uint8_t flags; /* bit0 IPv6 */
  uint32_t len;
  uint16_t csum_start;
  uint16_t csum_offset;
} or_pkt;
/* mode values match include/wgcsum.h WGCS_MODE_* */
void or_checksum_batch(int mode, uint8_t *arena, const or_pkt *pkts,
                       const uint64_t *initial, uint32_t n, void *out,
                       int inplace);
/* Multithreaded VALIDATE/L4_FILL batch for the CPU baseline (pthreads). */
void or_checksum_batch_mt(int mode, uint8_t *arena, const or_pkt *pkts,
                          uint32_t n, void *out, int threads);

/* All-cores CPU baselines (wg_oracle_bench.c): calls per second summed over
 * `threads` pthreads, each on private copies of the inputs, timing only the calls. */
double or_gso_bench_mt(const uint8_t *arena, const size_t *offs, const size_t *lens, int n_jobs, int nbufs,
                       int buf_len, int offset, int threads, double seconds, uint64_t *calls_out);
double or_gro_bench_mt(const uint8_t *pkts, const size_t *pkt_lens, size_t stride, int n, int offset, int can_udp,
                       int threads, double seconds, uint64_t *calls_out);
double or_checksum_bench_mt(int mode, const uint8_t *arena, size_t arena_len, const or_pkt *pkts, uint32_t n,
                            int threads, double seconds, uint64_t *passes_out);

/* ---- outer-UDP message batching (conn/bind.go, conn/gso.go; wg_oracle_conn.c) ---- */
/* one ipv6.Message: Buffers[0] (len/cap), N, OOB (len/cap), NN, Addr (opaque id) */
typedef struct or_msg {
  uint8_t *buf;
  size_t buf_len, buf_cap;
  int n;
  uint8_t *oob;
  size_t oob_len, oob_cap;
  int nn;
  int addr;
} or_msg;
/* conn/gso.go:35-67 */
int or_get_gso_size(const uint8_t *control, size_t len, int *gso);
/* conn/gso.go:71-100 */
void or_set_gso_size(uint8_t *control, size_t *len, size_t cap, uint16_t gso);
/* conn/sticky.go:101-107 */
void or_set_src_control(uint8_t *control, size_t *len, size_t cap, const uint8_t *src, size_t src_len);
/* conn/bind.go:542-597 */
int or_split_messages(or_msg *msgs, int n_msgs, int first_msg_at, int *n_packets);
/* conn/bind.go:599-662 */
int or_coalesce_messages(or_msg *msgs, int n_msgs_cap, uint8_t *const *bufs, const size_t *lens,
                         const size_t *caps, int nbufs, int dst_is_v6, const uint8_t *src_ctl,
                         size_t src_len, int addr, int *n_msgs);
/* batch drivers (tests, cpu_baseline): slot q = b*n + s at base + q*stride */
void or_split_batch(uint8_t *bufs, size_t stride, size_t buf_len, int *ns, uint8_t *oobs, size_t oob_stride,
                    const int *nns, int n_msgs, int first, int n_batches, int *counts, int *statuses);
void or_coalesce_batch(uint8_t *bufs, size_t stride, const size_t *lens, const size_t *caps, const int *nbufs,
                       int max_bufs, int n_batches, int dst_is_v6, int *n_msgs_out);

#ifdef __cplusplus
}
#endif
#endif
