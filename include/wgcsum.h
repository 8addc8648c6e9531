/*
 * wgcsum.h -- C ABI of the MI355X-native (gfx950) Internet-checksum hot path
 * of muhtutorials/wireguard's `tun` package.
 *
 * Plain C types only (pointers and sizes); no torch, no HIP types in the
 * signatures (streams are passed as `void*` = hipStream_t, NULL = the
 * context's own stream, a blocking stream: ordered both ways with work on the
 * HIP null stream, e.g. torch's default stream).  Every entry point is thread-safe: calls on one
 * context are serialized by a context mutex (the reference serializes Read
 * with Tun.readMu and Write with Tun.writeMu, tun/tun.go:101,:105).
 *
 * Reference interfaces replaced (file:line in /root/reference):
 *   wgcs_checksum_batch       batch form of checksum()            tun/checksum.go:152-167
 *                             + checksumValid()                   tun/gro.go:554-612
 *                             + gsoSplit's per-segment L4 sum      tun/gro.go:1469-1488
 *                             + gsoNoneChecksum()                 tun/gro.go:1497-1517
 *                             + IPv4 header checksum sites        tun/gro.go:1134-1138,1217-1221,1434-1436
 *   wgcs_checksum_batches     many such batches enqueued by one call over several streams
 *                             (consecutive Tun.Read / Tun.Write batches, tun/tun.go:477-508, :654-700)
 *   wgcs_checksum             checksum(b, initial)                tun/checksum.go:152-167
 *   wgcs_checksum_valid       checksumValid(pkt, iphLen, proto, isV6)  tun/gro.go:554-612
 *   wgcs_gso_none_checksum    gsoNoneChecksum(readBuf, start, off)     tun/gro.go:1497-1517
 *   wgcs_gso_split            gsoSplit(readBuf, hdr, bufs, sizes, offset, isV6)  tun/gro.go:1373-1493
 *   wgcs_gso_split_batch      device-resident batch of gsoSplit calls  (one per Tun.Read)
 *   wgcs_handle_virtio_read   handleVirtioRead(readBuf, bufs, sizes, offset)  tun/tun.go:514-632
 *   wgcs_*_cap                the same two with cap(readBuf)  (spare capacity, gro.go:1471-1477)
 *   wgcs_handle_gro           handleGRO(bufs, offset, tcpTable, udpTable, canUDPGRO, &toWrite)
 *                                                                 tun/gro.go:1326-1367
 *   wgcs_handle_gro_batch     device-resident batch of handleGRO calls (one per Tun.Write)
 *   wgcs_get_gso_size         getGSOSize(control)                 conn/gso.go:35-67
 *   wgcs_set_gso_size         setGSOSize(&control, gsoSize)       conn/gso.go:71-100
 *   wgcs_split_messages       splitMessages(msgs, firstMsgAt)     conn/bind.go:542-597
 *   wgcs_split_messages_batch device-resident batch of splitMessages calls (one per recvmmsg)
 *   wgcs_coalesce_messages    coalesceMessages(msgs, bufs, ep, addr)  conn/bind.go:599-662
 *   wgcs_coalesce_messages_batch  device-resident batch of coalesceMessages calls (one per Send)
 *   wgcs_stager_*             Tun.Read batch staging              tun/tun.go:477-508
 *   wgcs_wstager_*            Tun.Write batch staging             tun/tun.go:654-700
 * Status codes map 1:1 onto the reference's Go errors (see WGCS_ERR_*).
 */
#ifndef WGCSUM_H
#define WGCSUM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WGCS_ABI_VERSION 2 /* 2: wgcs_pkt carries proto and a u16 csum_offset */

/* ---- status codes (negative); Go sentinel / error each one maps to ---- */
#define WGCS_OK 0
#define WGCS_ERR_INVALID_ARG (-1)       /* API misuse (NULL ctx, n too large, ...) */
#define WGCS_ERR_SHORT_BUFFER (-2)      /* io.ErrShortBuffer                 gro.go:75,86 */
#define WGCS_ERR_TOO_MANY_SEGMENTS (-3) /* tun.ErrTooManySegments            tun.go:30, gro.go:1410 */
#define WGCS_ERR_INVALID_OFFSET (-4)    /* errors.New("invalid offset")     gro.go:1336 */
#define WGCS_ERR_UNSUPPORTED_GSO (-5)   /* "unsupported virtio GSO type: %d" tun.go:567 */
#define WGCS_ERR_IP_GSO_MISMATCH (-6)   /* "IP header version: %d, GSO type: %d" tun.go:575,584 */
#define WGCS_ERR_BAD_IP_VERSION (-7)    /* "invalid IP header version: %d"  tun.go:591 */
#define WGCS_ERR_PACKET_TOO_SHORT (-8)  /* "packet is too short"            tun.go:603 */
#define WGCS_ERR_TCP_HDR_LEN (-9)       /* "TCP header length is invalid: %d" tun.go:611 */
#define WGCS_ERR_HDR_LEN (-10)          /* "length of packet (%d) < virtioNetHdr.hdrLen (%d)" tun.go:616 */
#define WGCS_ERR_CSUM_OFFSET (-11)      /* "end of checksum offset (%d) exceeds packet length (%d)" tun.go:625 */
#define WGCS_ERR_READ_OVERFLOW (-12)    /* "read length %d overflows bufs element length %d" tun.go:546 */
#define WGCS_ERR_OUT_OF_RANGE (-13)     /* input on which the Go code would panic (slice bounds) */
#define WGCS_ERR_BATCH_FULL (-14)       /* stager: the open batch has no room; submit it first */
#define WGCS_ERR_NOT_READY (-15)        /* stager: batch id not submitted / recycled */
#define WGCS_ERR_CMSG (-16)             /* "error parsing socket control message: %w" conn/gso.go:45 */
#define WGCS_ERR_SPLIT_OVERFLOW (-17)   /* "splitting coalesced packet resulted in overflow" conn/bind.go:565 */
#define WGCS_ERR_HIP (-100)             /* HIP runtime error (message: wgcs_last_error) */
#define WGCS_ERR_NOMEM (-101)
#define WGCS_ERR_NO_DEVICE (-102)

/* ---- batch descriptor: one packet (or byte range) in a device arena ----
 * 16 bytes, loaded by the kernels as one dwordx4.  The arena offset is 48 bits
 * (off_lo | off_hi << 32); the checksum field sits at the uint16 position
 * (csum_start + csum_offset) & 0xFFFF, as the reference computes it
 * (gro.go:1391, :1503).  wgcs_pkt_set() fills one. */
typedef struct wgcs_pkt {
  uint32_t off_lo;      /* byte offset of the packet (IP header) in the arena, bits 0-31 */
  uint16_t off_hi;      /* bits 32-47                                                    */
  uint8_t proto;        /* pseudo-header protocol (checksumValid's `protocol`, any u8)   */
  uint8_t flags;        /* WGCS_PKT_*                                                    */
  uint32_t len;         /* packet length in bytes (< 2^31)                               */
  uint16_t csum_start;  /* L4 start = IP header length (iphLen / virtio csumStart)       */
  uint16_t csum_offset; /* checksum field offset from csum_start (16 TCP, 6 UDP, any)    */
} wgcs_pkt;

#define WGCS_PKT_V6 0x01 /* isV6: addresses at 8/24 (16 B) instead of 12/16 (4 B) */

static inline void wgcs_pkt_set(wgcs_pkt *p, uint64_t off, uint32_t len, uint16_t csum_start,
                                uint16_t csum_offset, uint8_t proto, uint8_t flags) {
  p->off_lo = (uint32_t)off;
  p->off_hi = (uint16_t)(off >> 32);
  p->proto = proto;
  p->flags = flags;
  p->len = len;
  p->csum_start = csum_start;
  p->csum_offset = csum_offset;
}

/* ---- batch modes (out element: u16, except VALIDATE: u8 0/1) ---- */
#define WGCS_MODE_FOLD 0     /* out = checksum(pkt[0:len], initial[i])                 checksum.go:152 */
#define WGCS_MODE_L4_FILL 1  /* out = ^checksum(pkt[cs:len] with field zeroed,
                                pseudoHeaderChecksumNoFold(src,dst,proto,len-cs))     gro.go:1469-1488 */
#define WGCS_MODE_VALIDATE 2 /* out = checksumValid(pkt, cs, proto, isV6)             gro.go:554-612 */
#define WGCS_MODE_PARTIAL 3  /* out = ^checksum(pkt[cs:len] field zeroed, BE16(field)) gro.go:1497-1517 */
#define WGCS_MODE_IP4HDR 4   /* out = ^checksum(pkt[0:cs] with [10:12] zeroed, 0)      gro.go:1134-1138 */

#define WGCS_F_INPLACE 0x1 /* also store the result big-endian into the packet's field
                              (when the field lies inside the packet's len bytes) */

typedef struct wgcs_ctx wgcs_ctx;

/* virtioNetHdr, tun/gro.go:42-67 (10 bytes on the wire, native byte order) */
typedef struct wgcs_virtio_hdr {
  uint8_t flags;
  uint8_t gso_type;
  uint16_t hdr_len;
  uint16_t gso_size;
  uint16_t csum_start;
  uint16_t csum_offset;
} wgcs_virtio_hdr;

/* one job of wgcs_gso_split_batch: a Tun.Read super-packet */
typedef struct wgcs_gso_job {
  uint64_t off;   /* offset of the 10-byte virtio header in the device arena */
  uint32_t len;   /* bytes read from the TUN fd (virtio header included)     */
  uint32_t flags; /* WGCS_GSO_JOB_*                                          */
} wgcs_gso_job;

/* default (0): handleVirtioRead semantics -- validate the header, recompute
 * hdrLen, GSO_NONE copy (+ gsoNoneChecksum), tun/tun.go:514-632.
 * RAW: gsoSplit(readBuf, hdr, ...) semantics with the header fields taken as
 * given (gro.go:1373-1493); WGCS_GSO_JOB_V6 then gives isV6. */
#define WGCS_GSO_JOB_RAW 0x1u
#define WGCS_GSO_JOB_V6 0x2u
/* bits 8-15: how many bytes after the job's len bytes in the arena belong to
 * the read buffer's spare capacity (cap(readBuf) - len(readBuf), at most 255).
 * The pseudo-header address slices of a packet shorter than 20 / 40 bytes
 * reach into it (gro.go:1471-1477: a slice up to cap is legal Go); past it
 * the reference panics (OUT_OF_RANGE).  0: cap == len. */
#define WGCS_GSO_JOB_SPARE(n) ((uint32_t)((n) > 255 ? 255 : (n)) << 8)

/* ---- lifecycle / diagnostics ---- */
int wgcs_abi_version(void);
int wgcs_device_count(int *count);
int wgcs_init(int device, wgcs_ctx **out);
/* INVALID_ARG (the context stays usable) while a read or write stager made
 * on it is alive: destroy the stagers first. */
int wgcs_destroy(wgcs_ctx *ctx);
const char *wgcs_strerror(int status);
/* The calling thread's last error message on ctx (like errno: per thread, so
 * concurrent callers never share one buffer); "" when this thread's last
 * failure was on another context.  Valid until the thread's next failing call. */
const char *wgcs_last_error(wgcs_ctx *ctx);
int wgcs_sync(wgcs_ctx *ctx);
/* CU count of the context's device (grid sizing, reporting) */
int wgcs_num_cu(wgcs_ctx *ctx);
/* Pinned host memory mapped into the device's address space at the same
 * address (bytes rounded up to 16): the buffers of wgcs_wstager_push_pinned. */
int wgcs_host_alloc(wgcs_ctx *ctx, size_t bytes, void **p);
/* NOT_READY while a write-stager slot still reads the allocation (a recorded
 * zero-copy push, open or in flight); safe against concurrent
 * wgcs_wstager_push_pinned calls: either the push is refused (INVALID_ARG) or
 * the free is (NOT_READY). */
int wgcs_host_free(wgcs_ctx *ctx, void *p);

/* ---- device-resident batch entry points (HBM in, HBM out; async on stream) ----
 * The arena must be readable through align_up(off+len, 16) for every packet
 * (always true for hipMalloc / torch allocations, which are page-granular).
 * VALIDATE / L4_FILL read the pseudo-header addresses at [12, 20) / [8, 40)
 * whatever len is: a packet shorter than them has them read from the arena
 * bytes after it, its Go slice's spare capacity (gro.go:558-563), which must
 * then be readable too.  A csum_start past len (pkt[iphLen:] panics in Go)
 * gives VALIDATE 0 and L4_FILL 0 with no field write. */
int wgcs_checksum_batch(wgcs_ctx *ctx, int mode, unsigned flags, uint8_t *d_arena,
                        const wgcs_pkt *d_pkts, const uint64_t *d_initial, uint32_t n,
                        void *d_out, void *stream);

/* A series of independent device-resident batches enqueued by one call (e.g.
 * consecutive Tun.Read/Write batches, tun/tun.go:477-508, :654-700, already in
 * HBM): batch k is launched on streams[k % n_streams] (n_streams 0: the
 * context's stream), in order, with wgcs_checksum_batch's semantics.  Optional
 * bracket events (hipEvent_t as void*, created by the caller): ev_begin is
 * recorded on streams[0] before the first launch and the other streams wait on
 * it before their first; after the last launch every other stream that got a
 * batch is joined to streams[0] and ev_end is recorded there, so the pair
 * spans every launch.
 * All arguments are checked before anything is enqueued. */
typedef struct wgcs_batch {
  uint8_t *arena;
  const wgcs_pkt *pkts;
  const uint64_t *initial; /* FOLD only; may be NULL */
  void *out;
  uint32_t n;
  uint32_t pad;
} wgcs_batch;
#define WGCS_MAX_BATCH_STREAMS 16
int wgcs_checksum_batches(wgcs_ctx *ctx, int mode, unsigned flags, const wgcs_batch *batches,
                          uint32_t n_batches, void *const *streams, uint32_t n_streams,
                          void *ev_begin, void *ev_end);

/* A doorbell: work enqueued on `stream` (NULL: the context's) after this call
 * starts only once *flag == value.  `flag` is a 4-byte-aligned word of
 * wgcs_host_alloc memory (the device polls it); the host rings it with a plain
 * store.  A receive / send ring posts its batches ahead of time and rings once
 * they are due, so no host enqueue cost sits between a batch being ready and
 * its launch.  The caller must ring before it waits on the stream. */
int wgcs_stream_wait_flag(wgcs_ctx *ctx, void *stream, const uint32_t *flag, uint32_t value);

/* gsoSplit for n_jobs super-packets.  Job j writes its segments into output
 * slots [j*max_segs, (j+1)*max_segs), slot s at d_out + s*out_stride + offset
 * (like bufs[s][offset:]).  d_sizes[slot] = packet size; d_count[j] = the
 * return value n (>= 0) and d_status[j] = 0 or a WGCS_ERR_* code, with the
 * reference's ErrTooManySegments semantics (n = max_segs-1, gro.go:1409-1410).
 * Includes handleVirtioRead's GSO validation (tun/tun.go:557-631).
 * INVALID_ARG for max_segs == 0, max_segs >= 2^31 (len(bufs) is a Go int) or
 * n_jobs * max_segs >= 2^32. */
int wgcs_gso_split_batch(wgcs_ctx *ctx, const uint8_t *d_arena, const wgcs_gso_job *d_jobs,
                         uint32_t n_jobs, uint8_t *d_out, uint32_t out_stride, uint32_t offset,
                         uint32_t max_segs, int32_t *d_sizes, int32_t *d_count,
                         int32_t *d_status, void *stream);
/* the shape wgcs_gso_split_batch was compiled to (not a reference interface:
 * benches and profiles name the kernel from it): lds_waves waves per
 * workgroup, parts workgroups per read, u chunks per lane in flight; rows = 1
 * when WGCS_GSO_KERNEL=rows selects the round-4 gso_rows_kernel grid. */
int wgcs_gso_kernel_shape(int *lds_waves, int *parts, int *u, int *rows);

/* ---- reference-shaped entry points on host buffers (Go-call granularity) ----
 * These stage through the context's pinned ring, run the HIP kernels and copy
 * results back; they keep the reference's argument meaning and errors. */
int wgcs_checksum(wgcs_ctx *ctx, const uint8_t *b, size_t n, uint64_t initial, uint16_t *out);
int wgcs_checksum_valid(wgcs_ctx *ctx, const uint8_t *pkt, size_t len, uint8_t iph_len,
                        uint8_t proto, int is_v6, int *valid);
/* the same with the slice's capacity: pkt[0, cap) is readable, and a packet
 * shorter than its addresses (20 / 40 B) has them read from pkt[len, cap), as
 * Go's pkt[a:b] up to cap does (gro.go:558-563); OUT_OF_RANGE past cap or for
 * iph_len > len.  wgcs_checksum_valid is this with cap == len. */
int wgcs_checksum_valid_cap(wgcs_ctx *ctx, const uint8_t *pkt, size_t len, size_t cap,
                            uint8_t iph_len, uint8_t proto, int is_v6, int *valid);
int wgcs_gso_none_checksum(wgcs_ctx *ctx, uint8_t *read_buf, size_t len, uint16_t csum_start,
                           uint16_t csum_offset);
/* host batch: same semantics as wgcs_checksum_batch on a host arena of
 * arena_len bytes; VALIDATE / L4_FILL packets whose pseudo-header addresses
 * would lie past it are refused (OUT_OF_RANGE: the arena is their capacity) */
int wgcs_checksum_batch_host(wgcs_ctx *ctx, int mode, unsigned flags, uint8_t *h_arena,
                             size_t arena_len, const wgcs_pkt *h_pkts, const uint64_t *h_initial,
                             uint32_t n, void *h_out);
/* bufs[i] points at a buffer of buf_lens[i] bytes; sizes[] receives packet sizes. */
int wgcs_gso_split(wgcs_ctx *ctx, uint8_t *read_buf, size_t len, const wgcs_virtio_hdr *hdr,
                   uint8_t *const *bufs, const size_t *buf_lens, int nbufs, int *sizes,
                   int offset, int is_v6, int *n_out);
/* read_buf: the bytes read from the TUN fd, virtio header first (tun/tun.go:490). */
int wgcs_handle_virtio_read(wgcs_ctx *ctx, uint8_t *read_buf, size_t n, uint8_t *const *bufs,
                            const size_t *buf_lens, int nbufs, int *sizes, int offset,
                            int *n_out);
/* The same with the slice's capacity: read_buf[0, cap) is readable and
 * read_buf[n, cap) is the spare capacity Tun.Read's tun.readBuf[:n] carries
 * (tun/tun.go:484-503); only the pseudo-header address slices of a packet
 * shorter than its IP addresses reach it (gro.go:1471-1477).  cap >= n;
 * wgcs_handle_virtio_read is this with cap == n.  Same for gsoSplit. */
int wgcs_handle_virtio_read_cap(wgcs_ctx *ctx, uint8_t *read_buf, size_t n, size_t cap,
                                uint8_t *const *bufs, const size_t *buf_lens, int nbufs,
                                int *sizes, int offset, int *n_out);
int wgcs_gso_split_cap(wgcs_ctx *ctx, uint8_t *read_buf, size_t len, size_t cap,
                       const wgcs_virtio_hdr *hdr, uint8_t *const *bufs, const size_t *buf_lens,
                       int nbufs, int *sizes, int offset, int is_v6, int *n_out);
/* Go-slice form of handleGRO: lens[i] = len(bufs[i]), caps[i] = cap(bufs[i]).
 * bufs/lens/caps are updated in place (appends grow lens[i]; prepends swap
 * entries, gro.go:696-697); to_write receives the indices to write. */
int wgcs_handle_gro(wgcs_ctx *ctx, uint8_t **bufs, size_t *lens, size_t *caps, int n,
                    int offset, int can_udp_gro, int *to_write, int *n_to_write);

/* ---- the resident per-call ring (round 6) ----
 * The per-call forms above pay one kernel launch plus one completion wait per
 * Go call (~20 us).  A ring keeps a small kernel resident on a few CUs of its
 * own stream: a call writes a request record in fine-grained pinned host
 * memory and spins on a completion word the kernel bumps, so one Tun.Read /
 * checksumValid costs a PCIe round trip instead of a launch.  Same arguments,
 * bytes and errors as wgcs_checksum_valid[_cap] / wgcs_handle_virtio_read[_cap]
 * (tun/gro.go:554-612, tun/tun.go:514-632).  Request bytes in wgcs_host_alloc
 * memory are read in place; other caller memory is copied into the ring's
 * staging.  The kernel leaves after idle_us (0: 100 ms) without a request and
 * a later call launches it again; one call at a time per ring (it locks).
 * wgcs_ring_destroy stops the kernel and waits for it. */
typedef struct wgcs_ring wgcs_ring;
int wgcs_ring_create(wgcs_ctx *ctx, uint32_t idle_us, wgcs_ring **out);
int wgcs_ring_destroy(wgcs_ring *ring);
/* requests served, kernel launches made, 1 while the kernel is resident */
int wgcs_ring_info(wgcs_ring *ring, uint64_t *requests, uint64_t *launches, int *running);
int wgcs_ring_checksum_valid(wgcs_ring *ring, const uint8_t *pkt, size_t len, uint8_t iph_len, uint8_t proto,
                             int is_v6, int *valid);
int wgcs_ring_checksum_valid_cap(wgcs_ring *ring, const uint8_t *pkt, size_t len, size_t cap, uint8_t iph_len,
                                 uint8_t proto, int is_v6, int *valid);
int wgcs_ring_handle_virtio_read(wgcs_ring *ring, uint8_t *read_buf, size_t n, uint8_t *const *bufs,
                                 const size_t *buf_lens, int nbufs, int *sizes, int offset, int *n_out);
int wgcs_ring_handle_virtio_read_cap(wgcs_ring *ring, uint8_t *read_buf, size_t n, size_t cap,
                                     uint8_t *const *bufs, const size_t *buf_lens, int nbufs, int *sizes,
                                     int offset, int *n_out);

/* ---- device-resident batch of Tun.Write calls (handleGRO per call) ----
 * bufs[i] of a call is the Go slice d_arena[off : off+len] with cap(bufs[i]) =
 * cap; every slice owns d_arena[off, off+cap), and the arena must be readable
 * through align_up(off+cap, 16).  Call c runs handleGRO(bufs[first :
 * first+n], offset, ..., canUDPGRO = flags & WGCS_GRO_CAN_UDP) on the device,
 * in place, as the reference mutates its slices: the slice headers in d_bufs
 * after the prepend swaps and appends (gro.go:685-697), d_status[c] = 0,
 * WGCS_ERR_INVALID_OFFSET (gro.go:1335-1337: the earlier buffers keep what the
 * coalescing wrote, nothing is applied, d_n_write[c] = 0) or
 * WGCS_ERR_INVALID_ARG (n > WGCS_GRO_MAX_CALL or offset < 0: nothing touched),
 * and toWrite in d_to_write[first : first + d_n_write[c]].  Every byte that
 * Tun.Write hands to write(2) -- bufs[i][offset-10:len] for i in toWrite --
 * equals the reference's, and so does every other byte of every slice.
 * One workgroup per call, async on stream. */
typedef struct wgcs_gro_buf {
  uint64_t off; /* slice start in the arena */
  uint32_t len; /* len(bufs[i]) (offset + packet length) */
  uint32_t cap; /* cap(bufs[i]) */
} wgcs_gro_buf;
typedef struct wgcs_gro_call {
  uint32_t first; /* index of bufs[0] in d_bufs (and of toWrite[0] in d_to_write) */
  uint32_t n;     /* len(bufs) */
  int32_t offset; /* Tun.Write's offset */
  uint32_t flags; /* WGCS_GRO_CAN_UDP */
} wgcs_gro_call;
#define WGCS_GRO_CAN_UDP 0x1u
#define WGCS_GRO_MAX_CALL 128 /* conn.BatchSize (conn/conn.go:14): the largest Write batch */
int wgcs_handle_gro_batch(wgcs_ctx *ctx, uint8_t *d_arena, wgcs_gro_buf *d_bufs, const wgcs_gro_call *d_calls,
                          uint32_t n_calls, int32_t *d_status, int32_t *d_n_write, int32_t *d_to_write,
                          void *stream);

/* ---- Tun.Read batch staging (tun/tun.go:477-508) ----
 * A ring of `depth` batches.  Each batch stages up to max_reads TUN reads
 * (virtio header + packet, as read(2) returns them into tun.readBuf) in pinned
 * host memory; wgcs_stager_submit queues H2D -> GSO split (the kernel of
 * wgcs_gso_split_batch, handleVirtioRead semantics) -> D2H of sizes, counts,
 * statuses and the output slots on the batch's own stream, so consecutive
 * batches overlap both copy directions with compute.  Segment s of read r
 * lands in pinned memory at segs + s*seg_stride (seg_stride >= the largest
 * segment, e.g. 65535 for 64 KiB GSO_NONE reads, 1536 for MSS 1460).
 * Only the stager's own copy of each read is used (tun.readBuf is free again
 * as soon as push/commit returns); the reference's in-place readBuf edits are
 * not replayed there (they are invisible to Read's callers).
 * Ring discipline (depth >= 2): one slot is always open for pushes, so the results of a
 * batch stay readable until depth-1 further batches have been submitted
 * (the submit after that recycles its slot, waiting for it if still running). */
typedef struct wgcs_stager wgcs_stager;
int wgcs_stager_create(wgcs_ctx *ctx, uint32_t depth, uint32_t max_reads, size_t max_bytes,
                       uint32_t max_segs, uint32_t seg_stride, wgcs_stager **out);
int wgcs_stager_destroy(wgcs_stager *st);
/* copy one read into the open batch (waits for the ring slot if it is still in flight) */
int wgcs_stager_push(wgcs_stager *st, const uint8_t *read_buf, size_t n, int *read_idx);
/* push `count` reads in one call (read_idx of the first one in *first_idx); on
 * WGCS_ERR_BATCH_FULL *pushed tells how many went in */
int wgcs_stager_push_many(wgcs_stager *st, const uint8_t *const *read_bufs, const size_t *ns, int count,
                          int *first_idx, int *pushed);
/* zero-copy form: reserve room for up to max_n bytes (read(2) goes straight
 * into *dst), then commit the byte count read (0 drops the reservation).  If
 * the read's output region does not fit the open batch, commit returns
 * WGCS_ERR_BATCH_FULL and keeps the bytes: the next wgcs_stager_submit queues
 * the batch without them and carries them in as read 0 of the new batch. */
int wgcs_stager_reserve(wgcs_stager *st, size_t max_n, uint8_t **dst, int *read_idx);
int wgcs_stager_commit(wgcs_stager *st, int read_idx, size_t n);
/* queue the open batch (no-op id for an empty batch) and open the next one */
int wgcs_stager_submit(wgcs_stager *st, uint64_t *batch);
int wgcs_stager_wait(wgcs_stager *st, uint64_t batch);
/* results of read r of a completed batch, handleVirtioRead's (n, err) */
int wgcs_stager_result(wgcs_stager *st, uint64_t batch, int read_idx, int *status, int *n,
                       const int32_t **sizes, const uint8_t **segs);
/* copy read r's segments into bufs[i][offset:] exactly as handleVirtioRead
 * leaves them (sizes[], n, ErrTooManySegments / slice-bound checks).  `segs`
 * of wgcs_stager_result holds the packets only: for a read whose header
 * geometry writes past a segment's end or reads bufs[i][4:6] (an IPv4 header
 * shorter than 6 bytes), copy_out runs the read again through the per-call
 * path with these bufs, so that every byte matches (gro.go:1419-1488).  That
 * rerun is a synchronous GPU round trip under the context's lock; it runs on a
 * copy of the read with the stager unlocked, so other calls on the stager do
 * not wait for it. */
int wgcs_stager_copy_out(wgcs_stager *st, uint64_t batch, int read_idx, uint8_t *const *bufs,
                         const size_t *buf_lens, int nbufs, int *sizes, int offset, int *n_out);

/* ---- Tun.Write batch staging (tun/tun.go:654-700) ----
 * A ring of `depth` slots; a slot aggregates up to max_writes Tun.Write calls
 * (<= max_pkts packets and <= max_bytes packet bytes in all).
 * wgcs_wstager_push stages one Write call (n <= WGCS_GRO_MAX_CALL buffers) --
 * bufs[i][offset-10:lens[i]], the packets as device/receive.go:483 slices
 * them, caps[i] = cap(bufs[i]) -- into pinned memory; no host planning.
 * wgcs_wstager_submit queues, on the slot's own stream, one H2D of every staged
 * packet, ONE device-resident handleGRO launch over every staged call (the
 * kernel of wgcs_handle_gro_batch: flow tables, checksumValid, coalescing and
 * apply* per call, on Go-sized slices in HBM), a gather of every call's
 * toWrite images and one D2H, so results are exactly handleGRO's
 * (gro.go:1326-1367).  wgcs_wstager_wait waits for the slot.
 * wgcs_wstager_result hands back, per call, what
 * Tun.Write passes to write(2) (tun.go:687-698): to_write[k] = handleGRO's
 * toWrite and pkts[k][0:pkt_lens[k]] = bufs[to_write[k]][offset-10:] after
 * handleGRO (10-byte virtio header + packet) in pinned memory, valid until the
 * slot is recycled; status WGCS_ERR_INVALID_OFFSET (gro.go:1336) writes
 * nothing.  The caller's bufs are only read.  Ring discipline as the Read
 * stager's: results stay readable until depth-1 more submits. */
typedef struct wgcs_wstager wgcs_wstager;
int wgcs_wstager_create(wgcs_ctx *ctx, uint32_t depth, uint32_t max_writes, uint32_t max_pkts, size_t max_bytes,
                        wgcs_wstager **out);
int wgcs_wstager_destroy(wgcs_wstager *ws);
/* stage one Tun.Write(bufs, offset) call; *write_idx = its index in the open slot
 * (WGCS_ERR_BATCH_FULL: submit first) */
int wgcs_wstager_push(wgcs_wstager *ws, const uint8_t *const *bufs, const size_t *lens, const size_t *caps, int n,
                      int offset, int can_udp_gro, int *write_idx);
/* Zero-copy form: every bufs[i] lies in memory from wgcs_host_alloc and stays
 * unchanged until the slot's results have been read; push records descriptors
 * only and the slot's scatter kernel reads the packets from host memory over
 * PCIe (a buffer pool allocated this way, e.g. device.pools.messageBufs, lets
 * Write skip the staging copy). */
int wgcs_wstager_push_pinned(wgcs_wstager *ws, const uint8_t *const *bufs, const size_t *lens, const size_t *caps,
                             int n, int offset, int can_udp_gro, int *write_idx);
int wgcs_wstager_submit(wgcs_wstager *ws, uint64_t *batch);
int wgcs_wstager_wait(wgcs_wstager *ws, uint64_t batch);
/* to_write / pkts / pkt_lens hold at least n (the call's packet count) entries */
int wgcs_wstager_result(wgcs_wstager *ws, uint64_t batch, int write_idx, int *status, int *n_write, int *to_write,
                        const uint8_t **pkts, size_t *pkt_lens);

/* ---- outer-UDP message batching (conn/bind.go, conn/gso.go) ----
 * The UDP side of the same batch loop: recvmmsg with UDP_GRO hands back up to
 * BatchSize/64 coalesced datagrams that splitMessages cuts into packets, and
 * Send coalesces runs of equal-size packets for UDP_SEGMENT (conn/bind.go:25-36:
 * maxIPv4PayloadLen 65507, maxIPv6PayloadLen 65527, maxUDPSegments 64). */

/* getGSOSize(msg.OOB[:msg.NN]): the UDP_GRO size (0 if absent) or WGCS_ERR_CMSG */
int wgcs_get_gso_size(const uint8_t *control, size_t len, int *gso_size);
/* setGSOSize(&control, gsoSize): appends a SOL_UDP/UDP_SEGMENT cmsg (24 bytes)
 * when it fits in cap; *len is len(control) in and out */
int wgcs_set_gso_size(uint8_t *control, size_t *len, size_t cap, uint16_t gso_size);

/* splitMessages over n_batches recvmmsg batches of n_msgs messages each.
 * At most 128 source messages (n_msgs - first_msg_at <= 128; BatchSize is 128,
 * conn/conn.go:14).  Message slot q = b*n_msgs + s.  Input: the recvmmsg landing buffers only --
 * msgs[s].Buffers[0] for s >= first_msg_at (buf_len bytes, len == cap) at
 * d_in + (b*(n_msgs - first_msg_at) + s - first_msg_at)*in_stride;
 * d_n_in[q] = msgs[s].N (all s), d_gso[q] = getGSOSize result (>= 0) or WGCS_ERR_CMSG.
 * Output, out of place: packet k of batch b at d_out + (b*n_msgs + k)*out_stride
 * (16-byte aligned, out_stride >= the largest packet), d_n_out[q] = the final
 * msgs[s].N (packet length, 0 for a source zeroed by :589-594, else unchanged),
 * d_src[q] = index s' whose Addr the slot now carries (:570) or -1 if unchanged;
 * d_count[b] = nPackets, d_status[b] = 0 / WGCS_ERR_CMSG / WGCS_ERR_SPLIT_OVERFLOW /
 * WGCS_ERR_OUT_OF_RANGE (Buffers[0][0:gsoSize] beyond cap) / WGCS_ERR_INVALID_ARG
 * (N > buf_len or a packet larger than out_stride).  On an error status the
 * packets before it are written, as the reference copies them before returning. */
int wgcs_split_messages_batch(wgcs_ctx *ctx, const uint8_t *d_in, uint64_t in_stride, uint32_t buf_len,
                              const int32_t *d_n_in, const int32_t *d_gso, uint32_t n_msgs,
                              uint32_t first_msg_at, uint32_t n_batches, uint8_t *d_out,
                              uint64_t out_stride, int32_t *d_n_out, int32_t *d_src, int32_t *d_count,
                              int32_t *d_status, void *stream);

/* coalesceMessages over n_batches Send batches, in place.  Batch b has
 * d_nbufs[b] <= max_bufs buffers; buffer j is slot q = b*max_bufs + j at
 * d_bufs + q*buf_stride (16-byte aligned), len(bufs[j]) = d_lens[q],
 * cap(bufs[j]) = min(d_caps[q], buf_cap) (d_caps NULL: buf_cap; buf_cap <= buf_stride).
 * Appends land in the first buffer of each run, as Go's append within cap does.
 * Per batch: d_n_msgs[b] = nMsgs; per message m (index b*max_bufs + m):
 * d_msg_first = the buffer j that msgs[m].Buffers[0] aliases, d_msg_len = its
 * final length, d_msg_gso = the UDP_SEGMENT size set by setGSOSize, or -1 if none. */
int wgcs_coalesce_messages_batch(wgcs_ctx *ctx, uint8_t *d_bufs, uint64_t buf_stride, uint32_t buf_cap,
                                 const int32_t *d_caps, const int32_t *d_lens, const int32_t *d_nbufs,
                                 uint32_t max_bufs, uint32_t n_batches, int dst_is_v6, int32_t *d_n_msgs,
                                 int32_t *d_msg_first, int32_t *d_msg_len, int32_t *d_msg_gso,
                                 void *stream);

/* splitMessages(msgs, firstMsgAt) on host buffers: bufs[i] = msgs[i].Buffers[0]
 * (buf_len bytes each, len == cap, as device/receive.go:119 passes them),
 * ns[i] = msgs[i].N (in/out), oobs[i][0:nns[i]] = msgs[i].OOB[:msgs[i].NN];
 * addr_src[i] = the message whose Addr msgs[i] carries afterwards (i if unchanged).
 * Returns the status, *n_packets = nPackets. */
int wgcs_split_messages(wgcs_ctx *ctx, uint8_t *const *bufs, size_t buf_len, int *ns,
                        const uint8_t *const *oobs, const size_t *nns, int n_msgs, int first_msg_at,
                        int *addr_src, int *n_packets);
/* coalesceMessages(msgs, bufs, endpoint, addr) on host buffers (len/cap per
 * buffer, len <= 65536): appends into bufs[msg_first[m]] within its capacity;
 * msg_len[m] = len(msgs[m].Buffers[0]).  oobs (optional, m < nbufs): msgs[m].OOB
 * with oob_lens in/out and oob_caps -- setSrcControl(src_ctl) then setGSOSize
 * for runs of > 1 packet, as conn/bind.go:634,647,657 do.  *n_msgs = nMsgs. */
int wgcs_coalesce_messages(wgcs_ctx *ctx, uint8_t *const *bufs, const size_t *lens, const size_t *caps,
                           int nbufs, int dst_is_v6, const uint8_t *src_ctl, size_t src_len,
                           uint8_t *const *oobs, size_t *oob_lens, const size_t *oob_caps,
                           int *msg_first, size_t *msg_len, int *n_msgs);

#ifdef __cplusplus
}
#endif
#endif /* WGCSUM_H */
