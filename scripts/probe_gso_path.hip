// probe_gso_path.hip -- NOT product code.  Bisects the cfg4 GSO split from a
// bare row copy toward the product kernel, one feature at a time (timing
// only; outputs are not checked except by the copy-only modes' self test).
// Geometry is cfg4's: 256 jobs of 65,535 B ([10-B virtio hdr | 40-B header |
// 45 x 1460-B payload]), segment i of job j -> slot (j*max_segs + i) of
// `stride` bytes, packet at slot + `doff`.  One 16-lane row per segment,
// 16 rows per 256-thread block, grid (job, 3).
//  F_DOFF   payload lands at slot + doff + 40 (not 16-byte aligned): byte-exact
//           head / tail chunks through store_chunk (else full chunks from slot+0)
//  F_HDR    the 40-byte header chunks stored too (row lanes 0..3, before the payload)
//  F_CHAIN  job descriptor and virtio header read from memory first (dependent
//           loads before the payload loads) instead of kernel-argument constants
//  F_SUM    v_dot2 sums of the payload chunks, written per row
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../wireguard_amd/csrc/wgcs_common.h"
#include "../wireguard_amd/csrc/wgcs_copy.h"
#include "../wireguard_amd/csrc/wgcs_rows.h"

using namespace wgcs;

enum { F_DOFF = 1, F_HDR = 2, F_CHAIN = 4, F_SUM = 8, F_BUF = 16 };

struct Job {
  uint64_t off;
  uint32_t len, flags;
};

template <int F>
__global__ __launch_bounds__(256) void probe_gso(const uint8_t* __restrict__ arena, const Job* __restrict__ jobs,
                                                  uint8_t* __restrict__ out, uint32_t max_segs, uint32_t stride,
                                                  uint32_t doff, uint32_t* __restrict__ sums) {
  constexpr int U = 6;
  const int lane = threadIdx.x & 63, r = lane & 15, wv = threadIdx.x >> 6;
  const uint32_t jb = blockIdx.x;
  int hdr = 40, gso = 1460, plen = 65525;
  uint64_t joff = (uint64_t)jb * 65535u;
  if (F & F_CHAIN) {
    const Job j = jobs[jb];
    joff = j.off;
    const uint8_t* vb = arena + joff;
    hdr = vb[2] | (vb[3] << 8);
    gso = vb[4] | (vb[5] << 8);
    plen = (int)j.len - 10;
  }
  const uint8_t* rb = arena + joff + 10;
  const int nseg = (plen - hdr + gso - 1) / gso;
  for (int grp = (int)blockIdx.y; grp * 16 < nseg; grp += (int)gridDim.y) {
    const int i = grp * 16 + wv * 4 + (lane >> 4);
    if (i >= nseg) continue;
    const int seg_start = hdr + i * gso, seg_end = min(plen, seg_start + gso);
    const int pkt_len = hdr + seg_end - seg_start;
    uint8_t* dst = out + ((uint64_t)jb * max_segs + i) * stride + ((F & F_DOFF) ? doff : 0);
    const int dalign = (int)((uintptr_t)dst & 15u);
    uint8_t* dbase = dst - dalign;
    // destination chunk k covers packet positions [16k - dalign, +16); payload
    // positions >= hdr come from rb + i*gso + position
    const uint8_t* w0 = rb + (int64_t)i * gso - dalign;
    const int sb = (int)((uintptr_t)w0 & 3u);
    const uint8_t* ab = w0 - sb;
    const uint8_t* lo = rb + seg_start;
    const uint8_t* hi = rb + seg_end;
    const int nk = (pkt_len + dalign + 15) >> 4;
    uint32_t acc = 0;
    if (F & F_HDR) {  // header chunks: rb[0:hdr) rewritten stand-in (copy), lanes r < hk
      const int hk = (hdr + dalign + 15) >> 4;
      if (r < hk) {
        const uint8_t* hs = rb - dalign + 16 * r;
        uint4 h = make_uint4(0, 0, 0, 0);
        const int hph = (int)((uintptr_t)hs & 3u);
        const uint8_t* ha = hs - hph;
        uint4 a = ld16_a4<false>(ha);
        const uint32_t e = *reinterpret_cast<const uint32_t*>(__builtin_assume_aligned(ha + 16, 4));
        h = make_uint4(__builtin_amdgcn_alignbyte(a.y, a.x, hph), __builtin_amdgcn_alignbyte(a.z, a.y, hph),
                       __builtin_amdgcn_alignbyte(a.w, a.z, hph), __builtin_amdgcn_alignbyte(e, a.w, hph));
        store_chunk(dbase + 16 * r, h, 16 * r - dalign, hdr);
      }
    }
    for (int k0 = 0; k0 < nk; k0 += 16 * U) {
      uint4 A[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint8_t* ca = ab + 16 * (k0 + r + 16 * u);
        A[u] = (ca < hi && ca + 16 > lo) ? ld16_a4<true>(ca) : make_uint4(0, 0, 0, 0);
      }
      uint32_t E = 0;
      if (r == 15) {
        const uint8_t* ce = ab + 16 * (k0 + 16 * U);
        if (ce < hi) E = *reinterpret_cast<const uint32_t*>(__builtin_assume_aligned(ce, 4));
      }
      uint32_t Rc = row_next(A[0].x);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = k0 + r + 16 * u;
        const uint32_t Rx = u + 1 < U ? row_next(A[u + 1 < U ? u + 1 : u].x) : E;
        const uint32_t nx = r == 15 ? Rx : Rc;
        Rc = Rx;
        const int x0 = 16 * k - dalign;
        if (k < nk && x0 + 16 > hdr) {
          const uint4 v = make_uint4(__builtin_amdgcn_alignbyte(A[u].y, A[u].x, sb),
                                     __builtin_amdgcn_alignbyte(A[u].z, A[u].y, sb),
                                     __builtin_amdgcn_alignbyte(A[u].w, A[u].z, sb),
                                     __builtin_amdgcn_alignbyte(nx, A[u].w, sb));
          if (F & F_SUM) acc = add_halves(add_halves(add_halves(add_halves(acc, v.x), v.y), v.z), v.w);
          if (F & F_DOFF)
            store_chunk(dbase + 16 * k, v, x0 - hdr, pkt_len - hdr);
          else
            *reinterpret_cast<uint4*>(dbase + 16 * k) = v;
        }
      }
    }
    if (F & F_SUM) {
      acc = row16_sum_u32(acc);
      if (r == 0) sums[jb * max_segs + i] = acc;
    }
  }
}

extern "C" int probe_gso_launch(const void* arena, const void* jobs, void* out, uint32_t n_jobs, uint32_t max_segs,
                                uint32_t stride, uint32_t doff, void* sums, int flags, void* stream) {
  const dim3 grid(n_jobs, 3);
  hipStream_t s = (hipStream_t)stream;
  auto A = (const uint8_t*)arena;
  auto J = (const Job*)jobs;
  auto O = (uint8_t*)out;
  auto S = (uint32_t*)sums;
#define P(f) \
  case f: hipLaunchKernelGGL((probe_gso<f>), grid, dim3(256), 0, s, A, J, O, max_segs, stride, doff, S); break
  switch (flags) {
    P(0); P(1); P(2); P(3); P(4); P(5); P(6); P(7); P(8); P(9); P(10); P(11); P(12); P(13); P(14); P(15);
    default: return -1;
  }
#undef P
  return (int)hipGetLastError();
}
