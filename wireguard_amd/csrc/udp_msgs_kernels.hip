// udp_msgs_kernels.hip -- gfx950 outer-UDP message batching (SURVEY.md §8f
// row 3): the byte work of splitMessages / coalesceMessages
// (/root/reference/conn/bind.go:542-662) on device-resident batches of
// recvmmsg / sendmmsg messages.  Both loops are order-dependent only through
// a little integer state over message lengths (which message a packet lands
// in, at what offset); the bytes are then independent copies.  So each block
// replays that integer loop (scalar, from lengths only) and its 16-lane DPP
// rows move one packet each with 16-byte loads/stores (wgcs_rows.h).
//
// split (RX, UDP_GRO): message s >= firstMsgAt of a batch holds N bytes that
// the kernel coalesced at gsoSize; splitMessages cuts it into packets placed
// in msgs[0..nPackets).  Out-of-place here (read the landing slots, write the
// packet slots): the reference's in-place order never reads a byte after
// writing it (destinations of message i are slots <= i, and the last packet
// landing in msgs[i] itself reads [start, N) with start >= gsoSize >= its
// length), so a snapshot read is the same function.
//
// coalesce (TX, UDP_SEGMENT): runs of equal-size packets are appended into
// the first buffer of each run (spare capacity of that buffer), in place:
// no append reads a byte another append writes.
#include <hip/hip_runtime.h>

#include "../../include/wgcsum.h"
#include "wgcs_common.h"
#include "wgcs_copy.h"
#include "wgcs_kernels.h"
#include "wgcs_rows.h"

namespace wgcs {

namespace {

constexpr int kMaxUdpSegments = 64;                    // conn/bind.go:36
constexpr int kMaxIPv4Payload = (1 << 16) - 1 - 20 - 8;  // conn/bind.go:25
constexpr int kMaxIPv6Payload = (1 << 16) - 1 - 8;       // conn/bind.go:28

__device__ __forceinline__ int rl(int v, int lane) { return __builtin_amdgcn_readlane(v, lane); }

// DPP row_ror:1 -- lane r of each 16-lane row receives lane (r - 1) & 15.
__device__ __forceinline__ uint32_t row_prev_ror(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x121, 0xF, 0xF, false);
}
__device__ __forceinline__ uint4 row_prev_ror4(const uint4& v) {
  return make_uint4(row_prev_ror(v.x), row_prev_ror(v.y), row_prev_ror(v.z), row_prev_ror(v.w));
}

template <bool NT>
__device__ __forceinline__ uint4 ld16_nt(const uint8_t* p) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const u32x4* q = reinterpret_cast<const u32x4*>(__builtin_assume_aligned(p, 16));
  const u32x4 t = NT ? __builtin_nontemporal_load(q) : *q;
  return make_uint4(t.x, t.y, t.z, t.w);
}

// Full 16-byte chunks go out as one dwordx4 (non-temporal with
// WGCS_UDP_NTS: the packets are not re-read by this kernel); partial chunks
// through store_chunk's byte-exact pieces.
#ifndef WGCS_UDP_COAL_ROWS
#define WGCS_UDP_COAL_ROWS 16  // buffers (16-lane rows) per coalesce block (16: 85 us, 32: 93 us, 64: 102 us on the bench)
#endif
#ifndef WGCS_UDP_SPLIT_NT
#define WGCS_UDP_SPLIT_NT 1  // splitMessages' source windows non-temporal (0: regular loads; A/B builds)
#endif
#ifndef WGCS_UDP_SPLIT_EDGE_T
#define WGCS_UDP_SPLIT_EDGE_T 0  // 1: windows in a 128-B line the row shares with its neighbours load temporal
#endif
#ifndef WGCS_UDP_NTS
#define WGCS_UDP_NTS 0
#endif
#ifndef WGCS_UDP_SPLIT_OWN
#define WGCS_UDP_SPLIT_OWN 1  // splitMessages: each 128-B source line loaded by one row, shared through LDS (0: A/B builds)
#endif
// A row's LDS image: 16 lanes x 16 B x kOwnU windows.  A packet of g bytes
// needs at most g + 15 (its first window's phase) + 127 (its last line) of it.
constexpr int kOwnU = 7;
constexpr int kOwnImg = 16 * 16 * kOwnU;
constexpr int kOwnMaxG = kOwnImg - 15 - 127;
__device__ __forceinline__ void put_chunk(uint8_t* dchunk, const uint4& v, int x0, int len) {
  if (WGCS_UDP_NTS && x0 >= 0 && x0 + 16 <= len) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    u32x4 t = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(t, reinterpret_cast<u32x4*>(__builtin_assume_aligned(dchunk, 16)));
    return;
  }
  store_chunk(dchunk, v, x0, len);
}

// Row copy to a 16-byte aligned destination from any source alignment:
// destination chunk k = bytes [sb, sb + 16) of the dword-aligned source
// window k plus the first dword of window k + 1 (next lane, DPP row_ror:15).
template <int U>
__device__ __forceinline__ void row_copy_dst_aligned(const uint8_t* src, int len, uint8_t* dst, int r) {
  const int sb = (int)((uintptr_t)src & 3u);
  const uint8_t* abase = src - sb;  // same dword as src: never a new page
  const uint8_t* src_hi = src + len;
  const int nk = (len + 15) >> 4;
  const uint4 z = make_uint4(0, 0, 0, 0);
  for (int k0 = 0; k0 < nk; k0 += 16 * U) {
    uint4 A[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint8_t* ca = abase + 16 * (k0 + r + 16 * u);
      if (WGCS_UDP_SPLIT_EDGE_T) {
        // the first and last lines of a packet are the neighbouring packets'
        // too: loaded temporal they stay in L2 for the other row's read
        const uintptr_t line = (uintptr_t)ca & ~(uintptr_t)127;
        const bool shared = line < (uintptr_t)src || line + 128 > (uintptr_t)src_hi;
        A[u] = ca >= src_hi ? z : shared ? ld_window<false>(ca, src_hi) : ld_window<WGCS_UDP_SPLIT_NT != 0>(ca, src_hi);
      } else {
        A[u] = ca < src_hi ? ld_window<WGCS_UDP_SPLIT_NT != 0>(ca, src_hi) : z;
      }
    }
    uint32_t E = 0;
    if (r == 15) {
      const uint8_t* ce = abase + 16 * (k0 + 16 * U);
      if (ce < src_hi) E = *reinterpret_cast<const uint32_t*>(__builtin_assume_aligned(ce, 4));
    }
    uint32_t Rc = row_next(A[0].x);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = k0 + r + 16 * u;
      const uint32_t Rx = u + 1 < U ? row_next(A[u + 1 < U ? u + 1 : u].x) : E;
      const uint32_t nx = r == 15 ? Rx : Rc;
      Rc = Rx;
      if (k < nk) {
        const uint4 v = make_uint4(__builtin_amdgcn_alignbyte(A[u].y, A[u].x, sb),
                                   __builtin_amdgcn_alignbyte(A[u].z, A[u].y, sb),
                                   __builtin_amdgcn_alignbyte(A[u].w, A[u].z, sb),
                                   __builtin_amdgcn_alignbyte(nx, A[u].w, sb));
        put_chunk(dst + 16 * k, v, 16 * k, len);
      }
    }
  }
}

}  // namespace

// ---------------------------------------------------------------------------
// splitMessages (conn/bind.go:542-597) over n_batches recvmmsg batches.
// Block = 256 threads = 16 rows = 16 consecutive message slots k of one batch;
// grid = (batch, slot group).  Every wave replays the batch's split loop from
// (N, gsoSize) of the source messages (lane l holds sources first + l and
// first + 64 + l; the loop reads them with readlane), so no LDS or barrier.
// Row k then copies its packet (or settles its final N when it gets none).
template <int U>
__global__ __launch_bounds__(256) void udp_split_kernel(const uint8_t* __restrict__ in, uint64_t in_stride,
                                                        uint32_t buf_len, const int32_t* __restrict__ n_in,
                                                        const int32_t* __restrict__ gso_in, uint32_t n_msgs,
                                                        uint32_t first, uint8_t* __restrict__ out,
                                                        uint64_t out_stride, int32_t* __restrict__ n_out,
                                                        int32_t* __restrict__ src_out, int32_t* __restrict__ count,
                                                        int32_t* __restrict__ status) {
  const int lane = threadIdx.x & 63, r = lane & 15;
  const int wv = threadIdx.x >> 6;
  const uint32_t b = blockIdx.x;
  const uint64_t slot0 = (uint64_t)b * n_msgs;
  const int k = (int)(blockIdx.y * 16u) + wv * 4 + (lane >> 4);  // this row's message slot

  // sources of this batch into VGPRs (two per lane)
  const int ns = (int)n_msgs - (int)first;
  int vn0 = 0, vg0 = 0, vn1 = 0, vg1 = 0;
  if (lane < ns) {
    vn0 = n_in[slot0 + first + lane];
    vg0 = gso_in[slot0 + first + lane];
  }
  if (64 + lane < ns) {
    vn1 = n_in[slot0 + first + 64 + lane];
    vg1 = gso_in[slot0 + first + 64 + lane];
  }

  // ---- the split loop (scalar state), recording this row's packet
  int base = 0, st = 0;
  int my_i = -1, my_start = 0, my_len = 0;
  int my_j = 0, my_ncopy = 0, my_g = 0, my_N = 0;  // packet index, packets landed, gsoSize, N of its message
  bool my_zeroed = false;
  for (int t = 0; t < ns; ++t) {
    const int i = (int)first + t;
    const int N = t < 64 ? rl(vn0, t) : rl(vn1, t - 64);
    if (N == 0) break;  // :545-547
    const int g = t < 64 ? rl(vg0, t) : rl(vg1, t - 64);
    if (g < 0) { st = g; break; }  // getGSOSize error (:554-557)
    if (N < 0 || (uint32_t)N > buf_len) { st = WGCS_ERR_INVALID_ARG; break; }  // N beyond the buffer
    if ((uint32_t)g > buf_len) { st = WGCS_ERR_OUT_OF_RANGE; break; }      // Buffers[0][0:g] panics
    const int seg_max = g > 0 ? g : N;
    if ((uint64_t)seg_max > out_stride) { st = WGCS_ERR_INVALID_ARG; break; }  // API: slot too small
    const int num = g > 0 ? (N + g - 1) / g : 1;  // :558-562
    const int room = i - base + 1;                // packets before nPackets > i (:564-567)
    const int ncopy = num < room ? num : room;
    const int j = k - base;
    if (j >= 0 && j < ncopy) {
      my_i = i;
      my_start = j * g;  // start of packet j; end_0 = gsoSize (may pass N), end_j = min((j+1)g, N)
      const int end = g == 0 ? N : (j == 0 ? g : min((j + 1) * g, N));
      my_len = end - my_start;
      my_j = j;
      my_ncopy = ncopy;
      my_g = g;
      my_N = N;
    }
    base += ncopy;
    if (ncopy < num) { st = WGCS_ERR_SPLIT_OVERFLOW; break; }
    if (k == i && i != base - 1) my_zeroed = true;  // msg.N = 0 (:589-594)
  }
  if (blockIdx.y == 0 && threadIdx.x == 0) {
    count[b] = base;
    status[b] = st;
  }
  const uint64_t sk = slot0 + (uint64_t)k;
  const bool active = k < (int)n_msgs && k < base;
  if (k < (int)n_msgs && r == 0) {
    n_out[sk] = active ? my_len : my_zeroed ? 0 : n_in[sk];  // copy() length: within buf_len here
    src_out[sk] = active ? my_i : -1;
  }
  const uint64_t src_slot = (uint64_t)b * (uint64_t)ns + (uint64_t)(my_i - (int)first);  // landing slots only
  const uint8_t* msg = in + src_slot * in_stride;  // the source message (valid when active)
  uint8_t* dst = out + sk * out_stride;
  if constexpr (!WGCS_UDP_SPLIT_OWN) {
    if (active) row_copy_dst_aligned<U>(msg + my_start, my_len, dst, r);
    return;
  }
  // ---- each 128-B source line loaded by ONE row.  Packets j - 1 and j of a
  // message (rows k - 1 and k of this block) share the line holding byte j*g;
  // it belongs to row k - 1, which loads up to the end of that line and puts
  // the windows from floor16(j*g) on in row k's image too.  Row k loads from
  // the next line boundary on.  Block edges and packets outside
  // [128, kOwnMaxG] bytes keep the direct row copy (no neighbour shares).
  __shared__ __attribute__((aligned(16))) uint8_t s_img[16 * kOwnImg];
  const int row = wv * 4 + (lane >> 4);
  const bool own = active && my_g >= 128 && my_g <= kOwnMaxG;
  // offsets from the 128-B line that holds the message's first byte
  const int o = (int)((uintptr_t)msg & 127u);
  const uint8_t* line0 = msg - o;
  const int s = my_start + o, e = my_start + my_len + o, a0 = s & ~15;
  if (own) {
    const bool prev = row > 0 && my_j >= 1;               // row k - 1 holds packet j - 1 of this message
    const bool next = row < 15 && my_j + 1 < my_ncopy;     // row k + 1 holds packet j + 1
    const int lo = prev ? (s + 127) & ~127 : a0;
    // next: up to the end of the shared line, within packet j + 1's bytes
    const int hi = next ? min((e + 127) & ~127, min((my_j + 2) * my_g, my_N) + o) : e;
    const int e16 = e & ~15;
    const uint8_t* lim = line0 + hi;
    uint8_t* img = s_img + row * kOwnImg;
    uint4 A[kOwnU];
#pragma unroll
    for (int u = 0; u < kOwnU; ++u) {
      const int x = lo + 16 * (r + 16 * u);
      A[u] = x < hi ? ld_window<WGCS_UDP_SPLIT_NT != 0>(line0 + x, lim) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < kOwnU; ++u) {
      const int x = lo + 16 * (r + 16 * u);
      if (x < hi) {
        *reinterpret_cast<uint4*>(img + (x - a0)) = A[u];
        if (next && x >= e16) *reinterpret_cast<uint4*>(img + kOwnImg + (x - e16)) = A[u];
      }
    }
  }
  __syncthreads();
  if (own) {
    // chunk c = bytes [s + 16c, s + 16c + 16): five dwords of the image from
    // floor4(s - a0) + 16c, funnelled by s & 3
    const uint8_t* img = s_img + row * kOwnImg + ((s - a0) & ~3);
    const int sb = s & 3, nk = (my_len + 15) >> 4;
#pragma unroll
    for (int u = 0; u < kOwnU; ++u) {
      const int c = r + 16 * u;
      if (c < nk) {
        const uint32_t* q = reinterpret_cast<const uint32_t*>(__builtin_assume_aligned(img + 16 * c, 4));
        const uint32_t d0 = q[0], d1 = q[1], d2 = q[2], d3 = q[3], d4 = q[4];
        const uint4 v = make_uint4(__builtin_amdgcn_alignbyte(d1, d0, sb), __builtin_amdgcn_alignbyte(d2, d1, sb),
                                   __builtin_amdgcn_alignbyte(d3, d2, sb), __builtin_amdgcn_alignbyte(d4, d3, sb));
        put_chunk(dst + 16 * c, v, 16 * c, my_len);
      }
    }
  } else if (active) {
    row_copy_dst_aligned<U>(msg + my_start, my_len, dst, r);
  }
}

// ---------------------------------------------------------------------------
// coalesceMessages (conn/bind.go:599-662) over n_batches sendmmsg batches, in
// place.  Block = ROWS x 16 threads = ROWS consecutive buffers of one batch
// (ROWS = 16 by default: more, smaller blocks per CU keep loads and stores of
// different blocks overlapped); grid = (batch, buffer group).  Every row first loads its buffer's
// first 16*U source chunks (aligned; they need only len(bufs[j])), while wave
// 0 replays the coalescing loop over the batch's lengths and publishes each
// of the block's buffers' destination offset through LDS.  After the barrier
// a row whose buffer was appended shifts its chunks to the destination phase
// (previous lane's chunk via DPP row_ror:1 + funnel) and stores them.
template <int U, int ROWS>
__global__ __launch_bounds__(ROWS * 16) void udp_coalesce_kernel(uint8_t* __restrict__ bufs, uint64_t stride,
                                                            uint32_t buf_cap, const int32_t* __restrict__ caps,
                                                            const int32_t* __restrict__ lens,
                                                            const int32_t* __restrict__ nbufs_arr, uint32_t max_bufs,
                                                            int dst_is_v6, int32_t* __restrict__ n_msgs_out,
                                                            int32_t* __restrict__ msg_first,
                                                            int32_t* __restrict__ msg_len,
                                                            int32_t* __restrict__ msg_gso) {
  __shared__ int64_t s_dst[ROWS];  // destination byte offset of the row's buffer, or -1 (not moved)
  const int lane = threadIdx.x & 63, r = lane & 15;
  const int wv = threadIdx.x >> 6;
  const uint32_t b = blockIdx.x;
  const uint64_t slot0 = (uint64_t)b * max_bufs;
  const int nb = min(nbufs_arr[b], (int)max_bufs);
  const int jb0 = (int)blockIdx.y * ROWS;
  const int row = wv * 4 + (lane >> 4);
  const int j = jb0 + row;  // this row's buffer

  // ---- speculative source loads (need only len(bufs[j]))
  const uint4 z = make_uint4(0, 0, 0, 0);
  int L = 0;
  if (j < nb) {
    const int cj = caps ? max(0, min(caps[slot0 + j], (int)buf_cap)) : (int)buf_cap;
    L = max(0, min(lens[slot0 + j], cj));  // a slice length is within [0, cap]
  }
  const int nsrc = (L + 15) >> 4;
  const uint8_t* sbase = bufs + (slot0 + (uint64_t)(j < nb ? j : 0)) * stride;
  uint4 A[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int c = r + 16 * u;
    A[u] = c < nsrc ? ld16_nt<true>(sbase + 16 * c) : z;
  }

  // ---- wave 0: the coalescing loop (scalar state over the lengths)
  if (wv == 0) {
    const int maxp = dst_is_v6 ? kMaxIPv6Payload : kMaxIPv4Payload;  // :615-618
    int i = -1, npk = 0, gso = 0, end_batch = 0;
    int first = 0, mlen = 0, mcap = 0;
    const bool pub = blockIdx.y == 0;  // one block per batch writes the message table
    for (int c0 = 0; c0 < nb; c0 += 64) {
      int vl = 0, vc = (int)buf_cap;
      if (c0 + lane < nb) {
        vc = caps ? max(0, min(caps[slot0 + c0 + lane], (int)buf_cap)) : (int)buf_cap;
        vl = max(0, min(lens[slot0 + c0 + lane], vc));
      }
      const int cend = min(64, nb - c0);
      // lanes whose buffer is exactly gsoSize long: candidates for a bulk append
      uint64_t eq_mask = 0;
      int eq_gso = -1;
      for (int t = 0; t < cend;) {
        const int jj = c0 + t;
        const int bl = rl(vl, t);
        const bool mine = jj >= jb0 && jj < jb0 + ROWS;
        if (jj > 0 && bl + mlen <= maxp && bl <= gso && bl <= mcap - mlen && npk < kMaxUdpSegments &&
            !end_batch) {  // :620-643 append
          int m = 1;
          if (bl == gso) {
            // Bulk: the next m buffers all have len == gsoSize, so each of them
            // passes the same test as long as npk < 64 and the run still fits
            // (no endBatch: bl < gsoSize is false for all of them).
            if (eq_gso != gso) {
              eq_mask = __ballot(vl == gso);
              eq_gso = gso;
            }
            const uint64_t run = ~(eq_mask >> t);  // first lane >= t whose len != gsoSize
            int m_eq = run ? (int)__builtin_ctzll(run) : 64 - t;
            m_eq = min(m_eq, cend - t);
            const int lim = min(maxp, mcap);
            const int m_sz = gso > 0 ? (lim - mlen) / gso : m_eq;
            m = max(1, min(min(m_eq, kMaxUdpSegments - npk), m_sz));
          }
          const int64_t dbase = (int64_t)(slot0 + (uint64_t)first) * (int64_t)stride + mlen;
          const int jl = c0 + lane;
          if (lane >= t && lane < t + m && jl >= jb0 && jl < jb0 + ROWS)
            s_dst[jl - jb0] = dbase + (int64_t)(lane - t) * bl;
          (void)mine;
          mlen += m * bl;
          npk += m;
          if (bl < gso) end_batch = 1;
          t += m;
          continue;
        }
        if (i >= 0 && pub && lane == 0) {  // close message i (:647-649: UDP_SEGMENT when > 1 packet)
          msg_first[slot0 + i] = first;
          msg_len[slot0 + i] = mlen;
          msg_gso[slot0 + i] = npk > 1 ? gso : -1;
        }
        ++i;  // :650-659
        npk = 1;
        gso = bl;
        end_batch = 0;
        first = jj;
        mlen = bl;
        mcap = rl(vc, t);
        if (mine && lane == 0) s_dst[jj - jb0] = -1;
        ++t;
      }
    }
    if (pub && lane == 0) {
      if (i >= 0) {
        msg_first[slot0 + i] = first;
        msg_len[slot0 + i] = mlen;
        msg_gso[slot0 + i] = npk > 1 ? gso : -1;
      }
      n_msgs_out[b] = i + 1;
    }
  }
  lds_barrier();  // publishes s_dst; the speculative source loads stay in flight
  if (j >= nb || L == 0) return;
  const int64_t doff = s_dst[row];
  if (doff < 0) return;  // first buffer of a message: stays where it is

  // ---- destination chunk k = bytes [16 - dd, 32 - dd) of source chunks (k-1 | k)
  uint8_t* dst = bufs + doff;
  const int dd = (int)((uintptr_t)dst & 15u);
  uint8_t* dbase = dst - dd;
  const int nk = (L + dd + 15) >> 4;
  uint4 carry = z;  // lane 0: lane 15's last chunk of the previous batch
  for (int k0 = 0; k0 < nk; k0 += 16 * U) {
    if (k0 > 0) {  // wave-uniform; the first batch was loaded speculatively
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int c = k0 + r + 16 * u;
        A[u] = c < nsrc ? ld16_nt<true>(sbase + 16 * c) : z;
      }
    }
    uint4 Q[U];
#pragma unroll
    for (int u = 0; u < U; ++u) Q[u] = row_prev_ror4(A[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kk = k0 + r + 16 * u;
      const uint4 prev = r != 0 ? Q[u] : (u > 0 ? Q[u > 0 ? u - 1 : 0] : carry);
      if (kk < nk) {
        const uint4 v = dd ? funnel_v(prev, A[u], 16 - dd) : A[u];
        put_chunk(dbase + 16 * kk, v, 16 * kk - dd, L);
      }
    }
    carry = Q[U - 1];
  }
}

hipError_t launch_udp_split(const uint8_t* in, uint64_t in_stride, uint32_t buf_len, const int32_t* n_in,
                            const int32_t* gso, uint32_t n_msgs, uint32_t first, uint32_t n_batches, uint8_t* out,
                            uint64_t out_stride, int32_t* n_out, int32_t* src, int32_t* count, int32_t* status,
                            hipStream_t s) {
  if (n_batches == 0 || n_msgs == 0) return hipSuccess;
  const dim3 grid(n_batches, (n_msgs + 15) / 16);
  hipLaunchKernelGGL(udp_split_kernel<6>, grid, dim3(256), 0, s, in, in_stride, buf_len, n_in, gso, n_msgs, first,
                     out, out_stride, n_out, src, count, status);
  return hipGetLastError();
}

hipError_t launch_udp_coalesce(uint8_t* bufs, uint64_t stride, uint32_t buf_cap, const int32_t* caps,
                               const int32_t* lens, const int32_t* nbufs, uint32_t max_bufs, uint32_t n_batches,
                               int dst_is_v6, int32_t* n_msgs, int32_t* msg_first, int32_t* msg_len,
                               int32_t* msg_gso, hipStream_t s) {
  if (n_batches == 0 || max_bufs == 0) return hipSuccess;
  constexpr int kRows = WGCS_UDP_COAL_ROWS;
  const dim3 grid(n_batches, (max_bufs + kRows - 1) / kRows);
  hipLaunchKernelGGL((udp_coalesce_kernel<6, kRows>), grid, dim3(kRows * 16), 0, s, bufs, stride, buf_cap, caps, lens, nbufs,
                     max_bufs, dst_is_v6, n_msgs, msg_first, msg_len, msg_gso);
  return hipGetLastError();
}

}  // namespace wgcs
