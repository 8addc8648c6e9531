// wgcs_host.h -- the plain-C++ part of the kernels' interface: launch
// tuning, the GSO output layout and its host-side bounds, the GRO plan and
// write-stager records.  No HIP types, so host-only code (the GRO planner,
// wgcs_gro_plan.h) and its sanitizer build (tests/sanitize/) include it alone.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include "../../include/wgcsum.h"

namespace wgcs {

struct LaunchTuning {
  // 256-thread blocks per CU at most.  Round 5: 1,024, so a batch of up to 2M
  // frames is one pass of the grid (every wave its own frames, no grid
  // stride): with 32 passes (the old 16 per CU) the waves drift apart and the
  // 128-byte line two neighbouring frames share was read twice, 5.6 % extra
  // HBM reads on cfg5 (profiles/r5_traf2_*); one pass: 1.1 %, and 5 % faster
  int blocks_per_cu = 1024;
  int lanes_per_pkt = 32;  // 16: one DPP row per packet (4 per wave); 32: half wave (2 per wave); 64: one wave
  int unroll = 4;          // 16-byte loads in flight per lane per iteration
  int nt = 1;              // non-temporal (streaming) loads: each byte is read once
  // chunk grid origin: packet start rounded down to this many bytes.  Round 5:
  // 128, and the interior iterations start on a line too, so no line is read
  // by two iterations of a row (cfg3's 9000-B frames: 6.3 % -> 1.5 % extra reads)
  int align = 128;
  int xcd = 1;             // XCD-aware block order (each XCD streams contiguous eighths)
};

// Optional packed output layout: segment i of job j at out + base + i*pitch
// (+ offset); pitch must hold the job's largest segment.  The room checks
// (handleVirtioRead's bufs element length) then use `room` instead of
// out_stride - offset.  Without kOutPosTails the kernel writes the packets
// only: gsoSplit's header writes that land past a segment's end (a field
// beyond hdrLen) are skipped, so a pitch sized for the packets is never
// overrun.  With it (the caller's buffers staged into the region, a pitch of
// at least gso_field_reach) they are written as into fixed slots.
enum : uint32_t { kOutPosTails = 1 };
struct GsoOutPos {
  uint64_t base;
  uint32_t pitch;
  uint32_t flags;  // kOutPosTails
};
// The resident per-call ring (ring.cpp, ring_kernel in gso_kernels.hip): one
// request record the host fills and then publishes by storing `seq` last, and
// the device's completion record on a line of its own; both in fine-grained
// (coherent) pinned host memory.
enum : uint32_t { kRingOpChecksumValid = 1, kRingOpVirtioRead = 2, kRingOpChecksumInline = 3 };
// The request record: eight 16-byte chunks, each {seq, 3 fields}.  The host
// stores the fields, then seq into every chunk (x86 stores become visible in
// order); the GPU reads the record with ONE wave load (lane k: chunk k) and
// takes it only when all eight seq words agree -- each 16-byte read is a
// snapshot, so a chunk whose seq is new holds that request's fields, and a
// record torn between two requests is read again.
struct RingReq {
  uint32_t c[8][4];
};
// field positions: chunk, word (word 0 of every chunk is seq)
enum : uint32_t {
  kRqOp = 0 * 4 + 1, kRqStop = 0 * 4 + 2, kRqLen = 0 * 4 + 3,           // checksumValid: len
  kRqCs = 1 * 4 + 1, kRqProto = 1 * 4 + 2, kRqFlags = 1 * 4 + 3,       // iphLen, proto, WGCS_PKT_V6
  kRqPktLo = 2 * 4 + 1, kRqPktHi = 2 * 4 + 2, kRqVlen = 2 * 4 + 3,     // pkt; virtio read: vlen
  kRqVbufLo = 3 * 4 + 1, kRqVbufHi = 3 * 4 + 2, kRqJflags = 3 * 4 + 3, // [virtio hdr | packet], job flags
  kRqKbufs = 4 * 4 + 1, kRqPitch = 4 * 4 + 2, kRqRoom = 4 * 4 + 3,     // slots, segment pitch, bufs[0] room
  kRqPosFlags = 5 * 4 + 1, kRqOutLo = 5 * 4 + 2, kRqOutHi = 5 * 4 + 3, // kOutPosTails; segment i at out + i pitch
  kRqMetaLo = 6 * 4 + 1, kRqMetaHi = 6 * 4 + 2,                        // int32 sizes[kbufs] | count | status
  kRqHdrInl = 6 * 4 + 3,                                               // virtio read: inline header bytes (0: none)
  kRqInl = kRqVlen,                                                    // inline checksumValid: bytes carried
};
// Inline checksumValid: the packet's bytes travel with the request, 12 per
// 16-byte chunk {seq, 3 data words} right after the record, so the poll that
// finds the request already holds them (one PCIe round trip fewer than reading
// pkt).  One poll reads kRingPollChunks chunks (wave 0: three 16-B loads per
// lane); the record takes 8 of them.
// A handleVirtioRead request carries the first bytes of its readBuf the same
// way (kRingHdrBytes, behind vbuf & 15 bytes of padding so that their phase
// mod 16 is the buffer's): the header decode and the verdict start from them
// while the payload loads go out.
enum : uint32_t { kRingPollChunks = 192, kRingInlineChunks = kRingPollChunks - 8, kRingInlineMax = kRingInlineChunks * 12 };
enum : uint32_t { kRingHdrBytes = 272, kRingHdrChunks = (15 + kRingHdrBytes + 11) / 12 };  // 24 chunks, 288 B
// One per workgroup, each on a 64-B line of its own: {seq, valid} is written
// by ONE 8-byte write-through store after the request's results.
struct RingDone {
  uint32_t seq;     // the request this workgroup finished last
  uint32_t valid;   // checksumValid's result (workgroup 0)
  uint32_t exited;  // times this workgroup left the kernel
  uint32_t pad[13];
};
enum : uint32_t { kRingMaxBlocks = 8 };
// The ring's workgroups: kRingWaves waves each (4 segment rows per wave), as
// many as hold the 48 rows of a 65,535-B read at MSS 1,460 (45 segments) --
// more, smaller workgroups spread the payload's host-memory reads over more CUs
#ifndef WGCS_RING_WAVES
#define WGCS_RING_WAVES 4  // (2: six 2-wave workgroups, measured: the device part 1.7 us shorter, the call no faster)
#endif
enum : uint32_t { kRingWaves = WGCS_RING_WAVES, kRingBlocks = 12 / WGCS_RING_WAVES };
static_assert(kRingBlocks >= 1 && kRingBlocks <= kRingMaxBlocks && 12 % WGCS_RING_WAVES == 0, "ring shape");
struct RingCtl {
  RingReq req;
  uint32_t inl[kRingInlineChunks][4];  // inline payload chunks (follow req: one poll reads both)
  uint32_t pad[16];
  RingDone dn[kRingMaxBlocks];
};
static_assert(sizeof(RingReq) % 64 == 0 && offsetof(RingCtl, dn) % 64 == 0 && sizeof(RingDone) == 64 &&
                  offsetof(RingCtl, inl) == sizeof(RingReq) && sizeof(RingReq) + sizeof(((RingCtl*)0)->inl) ==
                                                                   16 * kRingPollChunks,
              "the records on lines of their own");

// Packed-layout pitch and segment bound of one job ([10-byte virtio header |
// packet], n bytes) from its virtio header and job flags: every segment
// gso_rows_kernel can write for it fits in `pitch` (a segment is at most
// min(len, hdrLen + gsoSize) bytes; hdrLen is the caller's for RAW jobs and at
// most csumStart + 60 after handleVirtioRead's recompute), and it writes at
// most `segs` of them; 0/0 when it writes none.
inline void gso_out_layout(const uint8_t* vb, size_t n, uint32_t jflags, uint32_t max_segs, uint32_t* pitch,
                           uint32_t* segs) {
  *pitch = 0;
  *segs = 0;
  if (n <= 10) return;  // short buffer / empty packet: nothing written
  const size_t plen = n - 10;
  const size_t gso = (size_t)vb[4] | ((size_t)vb[5] << 8);
  const bool raw = (jflags & WGCS_GSO_JOB_RAW) != 0;
  if (!raw && vb[1] == 0) {  // GSO_NONE: the packet itself
    *pitch = (uint32_t)((plen + 15) & ~(size_t)15);
    *segs = 1;
    return;
  }
  const size_t cs = (size_t)vb[6] | ((size_t)vb[7] << 8);
  const size_t hdr = raw ? ((size_t)vb[2] | ((size_t)vb[3] << 8)) : cs + 60;
  size_t seg = hdr + gso < plen ? hdr + gso : plen;
  if (seg < 16) seg = 16;
  *pitch = (uint32_t)((seg + 15) & ~(size_t)15);
  const size_t nseg = gso ? (plen + gso - 1) / gso + 1 : (size_t)max_segs;
  *segs = (uint32_t)(nseg < max_segs ? nseg : max_segs);
}

// Bytes of bufs[i][offset:] that segment i (pkt_len bytes, `last` or not) of
// the job vb ([10-byte virtio header | packet], n bytes) writes: the packet
// plus gsoSplit's fixed-position header writes (gro.go:1419-1488 -- IPv4
// [2:12) or IPv6 [4:6), seq / UDP length at csumStart+4, the TCP flags byte on
// non-last segments, the checksum field; u16 positions).  A shorter Go slice
// panics, so the host entry points report OUT_OF_RANGE there.  GSO_NONE
// (handleVirtioRead semantics) writes the packet only.
inline size_t gso_split_need(const uint8_t* vb, size_t n, uint32_t jflags, size_t pkt_len, bool last) {
  if (n < 10) return pkt_len;
  const bool raw = (jflags & WGCS_GSO_JOB_RAW) != 0;
  const uint8_t t = vb[1];
  if (!raw && t == 0) return pkt_len;
  const bool v4 = raw ? (jflags & WGCS_GSO_JOB_V6) == 0 : (n > 10 && (vb[10] >> 4) == 4);
  const bool tcp = t == 1 || t == 4;
  const uint16_t cs = (uint16_t)(vb[6] | (vb[7] << 8)), co = (uint16_t)(vb[8] | (vb[9] << 8));
  size_t need = pkt_len > (size_t)(v4 ? 12 : 6) ? pkt_len : (size_t)(v4 ? 12 : 6);
  size_t f = (size_t)(uint16_t)(cs + 4) + (tcp ? 4 : 2);
  if (f > need) need = f;
  if (tcp && !last && (f = (size_t)(uint16_t)(cs + 13) + 1) > need) need = f;
  if ((f = (size_t)(uint16_t)(cs + co) + 2) > need) need = f;
  return need;
}

// gsoSplit's fixed-position header writes' reach for job vb: the last byte + 1
// of IPv4 [2:12) / IPv6 [4:6), seq or UDP length, the flags byte (non-last
// segments) and the checksum field.
inline size_t gso_field_reach(const uint8_t* vb, size_t n, uint32_t jflags) {
  return gso_split_need(vb, n, jflags, 0, false);
}

// Does gsoSplit's result for job vb involve bytes of bufs[i] other than the
// segments it produces?  Either a header write can land past a segment's end
// (a field beyond the smallest hdrLen the job can have), or the IPv4 id update
// reads bufs[i][4:6] (an IP header shorter than 6 bytes, gro.go:1426-1431).
// Host entry points then stage the caller's buffers through the kernel.
// Never for a well-formed TCP / UDP header (every field inside hdrLen).
inline bool gso_touches_caller_bytes(const uint8_t* vb, size_t n, uint32_t jflags) {
  if (n <= 10) return false;
  const bool raw = (jflags & WGCS_GSO_JOB_RAW) != 0;
  const uint8_t t = vb[1];
  if (!raw && t == 0) return false;  // GSO_NONE: the packet only
  const bool v4 = raw ? (jflags & WGCS_GSO_JOB_V6) == 0 : (vb[10] >> 4) == 4;
  const bool tcp = t == 1 || t == 4;
  const size_t cs = (size_t)vb[6] | ((size_t)vb[7] << 8);
  if (v4 && cs <= 5) return true;
  size_t lb;  // hdrLen's lower bound (handleVirtioRead's u16 recompute may wrap: then 0)
  if (raw) lb = (size_t)vb[2] | ((size_t)vb[3] << 8);
  else if (tcp) lb = cs + 60 <= 0xFFFF ? cs + 20 : 0;
  else lb = cs + 8 <= 0xFFFF ? cs + 8 : 0;
  return gso_field_reach(vb, n, jflags) > lb;
}

// One coalesced GRO output (applyTCPCoalesce / applyUDPCoalesce item).
struct GroItem {
  uint64_t out_off;   // [10-byte virtio header | packet] written at out + out_off
  uint32_t head_off;  // stage offset of the head packet (header source)
  uint32_t pkt_len;   // final IP packet length
  uint32_t seg_first, seg_count;  // payload segments in segs[]
  uint16_t gso_size;
  uint8_t iph, l4h;
  uint8_t kind;  // GRO_KIND_*
  uint8_t pad[7];
};
struct GroSeg {
  uint32_t src_off, len;  // stage offset / length of one payload piece
  uint32_t dst_off, pad;  // output offset of the piece (host-computed: pieces copy in parallel)
};
// RAW: the coalesced bytes only (head packet header + PSH, no apply*, no virtio
// header) -- handleGRO stopped at an invalid offset before applyTCPCoalesce.
enum : uint8_t { GRO_KIND_V6 = 1, GRO_KIND_UDP = 2, GRO_KIND_PSH = 4, GRO_KIND_RAW = 8 };

// Write stager around the batched handleGRO (wstager.cpp): packets staged
// back to back are moved into their Go-sized slices of the device arena, and
// after the handleGRO launch the toWrite images of each call are packed into
// that call's output region.  Source and destination of both copies share
// their phase mod 16, so both move whole aligned 16-byte chunks.
struct WsMove {
  uint64_t src, dst;    // 16-byte aligned source (stage offset, or a device-visible address) / arena offset
  uint32_t n16, flags;  // 16-byte chunks; WS_MOVE_ABS: src is an address (pinned host memory)
};
enum : uint32_t { WS_MOVE_ABS = 1 };
struct WsOut {
  uint64_t base;  // the call's output region (16-byte aligned)
  uint32_t room;  // its size in bytes
  uint32_t pad;
};
}  // namespace wgcs
