// Roofline probe (NOT product code): the fastest plain streaming read this
// chip sustains -- each wave sums U x 1 KiB aligned contiguous blocks with
// global_load_dwordx4 and writes one word.  Built on the GPU box by
// scripts/probe_stream.py; gives the practical HBM-read ceiling that the
// checksum kernel is compared against.
#include <hip/hip_runtime.h>
#include <stdint.h>
template <int U, bool NT>
__global__ __launch_bounds__(256) void probe(const uint4* __restrict__ src, size_t n16, uint32_t* __restrict__ out) {
  const size_t wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  const size_t nw = (size_t)gridDim.x * 4;
  const int lane = threadIdx.x & 63;
  uint32_t acc = 0;
  for (size_t b = wave * 64 * U; b < n16; b += nw * 64 * U) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      size_t c = b + u * 64 + lane;
      if (NT) {
        typedef unsigned int u4 __attribute__((ext_vector_type(4)));
        u4 t = c < n16 ? __builtin_nontemporal_load((const u4*)(src + c)) : u4{0, 0, 0, 0};
        v[u] = make_uint4(t.x, t.y, t.z, t.w);
      } else {
        v[u] = c < n16 ? src[c] : make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u].x + v[u].y + v[u].z + v[u].w;
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}
// Access pattern of checksum_batch_kernel<G=16,U>, minus all per-packet work:
// each wave takes 4 consecutive packets of `stride` bytes, each 16-lane row
// reads its packet's 16-B aligned chunks c = sub + 16u.
template <int U, bool NT>
__global__ __launch_bounds__(256) void probe_rows(const uint8_t* __restrict__ arena, uint32_t npk, uint32_t stride,
                                                  uint32_t* __restrict__ out) {
  const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint32_t nw = gridDim.x * 4;
  const int lane = threadIdx.x & 63, grp = lane >> 4, sub = lane & 15;
  uint32_t acc = 0;
  for (uint32_t base = wave * 4; base < npk; base += nw * 4) {
    const uint32_t p = base + grp;
    const uint8_t* pkt = arena + (size_t)p * stride;
    const int rel0 = 12 - (int)(((uintptr_t)pkt + 12) & 15);
    const int nch = p < npk ? ((int)stride - rel0 + 15) >> 4 : 0;
    const uint4* src = (const uint4*)(pkt + rel0);
    for (int c0 = sub; c0 < nch; c0 += 16 * U) {
      uint4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        int c = c0 + 16 * u;
        if (NT) {
          typedef unsigned int u4 __attribute__((ext_vector_type(4)));
          u4 t = c < nch ? __builtin_nontemporal_load((const u4*)(src + c)) : u4{0, 0, 0, 0};
          v[u] = make_uint4(t.x, t.y, t.z, t.w);
        } else {
          v[u] = c < nch ? src[c] : make_uint4(0, 0, 0, 0);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) acc += v[u].x + v[u].y + v[u].z + v[u].w;
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}
extern "C" int probe_rows_launch(const void* src, uint32_t npk, uint32_t stride, void* out, int grid, int nt,
                                 void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (nt) hipLaunchKernelGGL((probe_rows<6, true>), dim3(grid), dim3(256), 0, s, (const uint8_t*)src, npk, stride, (uint32_t*)out);
  else hipLaunchKernelGGL((probe_rows<6, false>), dim3(grid), dim3(256), 0, s, (const uint8_t*)src, npk, stride, (uint32_t*)out);
  return (int)hipGetLastError();
}
extern "C" int probe_launch(const void* src, size_t bytes, void* out, int grid, int u, int nt, void* stream) {
  size_t n16 = bytes / 16;
  hipStream_t s = (hipStream_t)stream;
#define L(U, NT) hipLaunchKernelGGL((probe<U, NT>), dim3(grid), dim3(256), 0, s, (const uint4*)src, n16, (uint32_t*)out)
  if (nt) { if (u == 2) L(2, true); else if (u == 4) L(4, true); else L(8, true); }
  else { if (u == 2) L(2, false); else if (u == 4) L(4, false); else L(8, false); }
  return (int)hipGetLastError();
}

// Whole-wave-per-packet pattern with F packets in flight per wave: packet f's
// chunk c = lane + 64u (u < 2: 2 KiB covers a 1500-B packet), so every load
// instruction reads 1 KiB contiguous.
template <int F>
__global__ __launch_bounds__(256) void probe_wavef(const uint8_t* __restrict__ arena, uint32_t npk, uint32_t stride,
                                                   uint32_t* __restrict__ out) {
  const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint32_t nw = gridDim.x * 4;
  const int lane = threadIdx.x & 63;
  uint32_t acc = 0;
  typedef unsigned int u4 __attribute__((ext_vector_type(4)));
  for (uint32_t base = wave * F; base < npk; base += nw * F) {
    u4 v[F][2];
#pragma unroll
    for (int f = 0; f < F; ++f) {
      const uint32_t p = base + f;
      const uint8_t* pkt = arena + (size_t)p * stride;
      const int rel0 = 12 - (int)(((uintptr_t)pkt + 12) & 15);
      const int nch = p < npk ? ((int)stride - rel0 + 15) >> 4 : 0;
      const u4* src = (const u4*)(pkt + rel0);
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int c = lane + 64 * u;
        v[f][u] = c < nch ? __builtin_nontemporal_load(src + c) : u4{0, 0, 0, 0};
      }
    }
#pragma unroll
    for (int f = 0; f < F; ++f)
#pragma unroll
      for (int u = 0; u < 2; ++u) acc += v[f][u].x + v[f][u].y + v[f][u].z + v[f][u].w;
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}
extern "C" int probe_wavef_launch(const void* src, uint32_t npk, uint32_t stride, void* out, int grid, int f,
                                  void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (f == 1) hipLaunchKernelGGL((probe_wavef<1>), dim3(grid), dim3(256), 0, s, (const uint8_t*)src, npk, stride, (uint32_t*)out);
  else if (f == 2) hipLaunchKernelGGL((probe_wavef<2>), dim3(grid), dim3(256), 0, s, (const uint8_t*)src, npk, stride, (uint32_t*)out);
  else hipLaunchKernelGGL((probe_wavef<4>), dim3(grid), dim3(256), 0, s, (const uint8_t*)src, npk, stride, (uint32_t*)out);
  return (int)hipGetLastError();
}

// LDS-DMA stream (global_load_lds_dwordx4, 1 KiB per wave-instruction into a
// wave-private 2-stage LDS ring), then ds_read_b128 of the lane's own slot:
// does the DMA path read HBM faster than register loads (the guide's
// ldsdma-fill row quotes 6.5-6.8 TB/s chip-wide with nt)?  Data is
// wave-private, so one counted vmcnt + s_barrier orders it (4 waves per block
// all run the same trip count: grid-stride by block).
template <int U, int AUX>
__global__ __launch_bounds__(256) void probe_glds(const uint4* __restrict__ src, size_t n16, uint32_t* __restrict__ out) {
  __shared__ uint4 ring[4][2][U][64];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t per_blk = (size_t)4 * U * 64;
  const size_t nblk_items = (n16 + per_blk - 1) / per_blk;
  uint32_t acc = 0;
  size_t it = blockIdx.x;
  auto issue = [&](size_t item, int stage) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      size_t c = item * per_blk + ((size_t)wv * U + u) * 64 + lane;
      if (c >= n16) c = n16 - 1;
      // asm, so hipcc does not count it and drain it with vmcnt(0) before the ds_read
      const uint32_t lds_dst = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)&ring[wv][stage][u][0];
      const uint4* g = src + c;
      uint32_t keep;
      if (AUX == 2)
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(g), "s"(__builtin_amdgcn_readfirstlane(lds_dst)) : "memory");
      else
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(g), "s"(__builtin_amdgcn_readfirstlane(lds_dst)) : "memory");
    }
  };
  int stage = 0;
  if (it < nblk_items) issue(it, 0);
  for (; it < nblk_items; it += gridDim.x) {
    const size_t nx = it + gridDim.x;
    if (nx < nblk_items) {
      issue(nx, stage ^ 1);
      if (U == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      else if (U == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int u = 0; u < U; ++u) {
      uint4 v = ring[wv][stage][u][lane];
      acc += v.x + v.y + v.z + v.w;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    stage ^= 1;
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}
extern "C" int probe_glds_launch(const void* src, size_t bytes, void* out, int grid, int u, int nt, void* stream) {
  size_t n16 = bytes / 16;
  hipStream_t s = (hipStream_t)stream;
#define G(U, A) hipLaunchKernelGGL((probe_glds<U, A>), dim3(grid), dim3(256), 0, s, (const uint4*)src, n16, (uint32_t*)out)
  if (nt) { if (u == 2) G(2, 2); else if (u == 4) G(4, 2); else G(8, 2); }
  else { if (u == 2) G(2, 0); else if (u == 4) G(4, 0); else G(8, 0); }
  return (int)hipGetLastError();
}

// G-lane rows (G = 32: two packets per wave), U loads in flight per lane, grid-
// stride over packets like checksum_batch_kernel<.., G, U, ..>, minus all
// per-packet arithmetic.  DESC: the packet's offset and length come from a
// 16-byte descriptor array (a dependent load before the data loads), as in
// the kernel; otherwise they are computed from the index.
template <int G, int U, bool DESC>
__global__ __launch_bounds__(256) void probe_rowsg(const uint8_t* __restrict__ arena, const uint4* __restrict__ desc,
                                                   uint32_t npk, uint32_t stride, uint32_t* __restrict__ out) {
  constexpr int PPW = 64 / G;
  const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint32_t nw = gridDim.x * 4;
  const int lane = threadIdx.x & 63, grp = lane / G, sub = lane % G;
  uint32_t acc = 0;
  typedef unsigned int u4 __attribute__((ext_vector_type(4)));
  for (uint32_t base = wave * PPW; base < npk; base += nw * PPW) {
    const uint32_t p = base + grp;
    uint64_t off = (uint64_t)p * stride;
    uint32_t len = stride;
    if (DESC) {
      const uint4 d = p < npk ? desc[p] : make_uint4(0, 0, 0, 0);
      off = ((uint64_t)d.y << 32) | d.x;
      len = d.z;
    }
    const uint8_t* pkt = arena + off;
    const int rel0 = 12 - (int)(((uintptr_t)pkt + 12) & 15);
    const int nch = p < npk ? ((int)len - rel0 + 15) >> 4 : 0;
    const u4* src = (const u4*)(pkt + rel0);
    for (int c0 = sub; c0 < nch; c0 += G * U) {
      u4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int c = c0 + G * u;
        v[u] = c < nch ? __builtin_nontemporal_load(src + c) : u4{0, 0, 0, 0};
      }
#pragma unroll
      for (int u = 0; u < U; ++u) acc += v[u].x + v[u].y + v[u].z + v[u].w;
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}
extern "C" int probe_rowsg_launch(const void* src, const void* desc, uint32_t npk, uint32_t stride, void* out,
                                  int grid, int g, int u, int use_desc, void* stream) {
  hipStream_t s = (hipStream_t)stream;
#define RG(G_, U_, D_) hipLaunchKernelGGL((probe_rowsg<G_, U_, D_>), dim3(grid), dim3(256), 0, s, (const uint8_t*)src, (const uint4*)desc, npk, stride, (uint32_t*)out)
  if (g == 16) { if (use_desc) RG(16, 6, true); else RG(16, 6, false); }
  else if (g == 32) {
    if (u == 3) { if (use_desc) RG(32, 3, true); else RG(32, 3, false); }
    else { if (use_desc) RG(32, 4, true); else RG(32, 4, false); }
  } else { if (use_desc) RG(64, 2, true); else RG(64, 2, false); }
  return (int)hipGetLastError();
}

// Flat stream in items of ITEM_KB KiB per wave, each item preceded by a
// dependent 16-byte "descriptor" load (the item's offset comes from it) and
// closed by NRED wave reductions + one store per reduction: the per-group
// prologue / epilogue of a per-packet kernel on top of the flat pattern.
__device__ __forceinline__ uint32_t probe_wave_sum(uint32_t v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor((int)v, o);
  return v;
}
template <int ITEM_KB, int NRED>
__global__ __launch_bounds__(256) void probe_items(const uint4* __restrict__ src, size_t n16,
                                                   const uint4* __restrict__ desc, uint32_t* __restrict__ out) {
  typedef unsigned int u4 __attribute__((ext_vector_type(4)));
  const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint32_t nw = gridDim.x * 4;
  const int lane = threadIdx.x & 63;
  const size_t n_items = n16 / (64 * ITEM_KB);
  for (size_t it = wave; it < n_items; it += nw) {
    const uint4 d = desc[it];  // dependent: the item's chunk base comes from memory
    const size_t b = ((size_t)d.y << 32) | d.x;
    uint32_t acc[NRED];
#pragma unroll
    for (int q = 0; q < NRED; ++q) acc[q] = 0;
#pragma unroll
    for (int k0 = 0; k0 < ITEM_KB; k0 += 4) {
      u4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        v[u] = k0 + u < ITEM_KB ? __builtin_nontemporal_load((const u4*)(src + b + (k0 + u) * 64 + lane)) : u4{0, 0, 0, 0};
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[(k0 + u) % NRED] += v[u].x + v[u].y + v[u].z + v[u].w;
    }
#pragma unroll
    for (int q = 0; q < NRED; ++q) {
      const uint32_t s = probe_wave_sum(acc[q]);
      if (lane == q) out[it * NRED + q] = s;
    }
  }
}
extern "C" int probe_items_launch(const void* src, size_t bytes, const void* desc, void* out, int grid, int item_kb,
                                  void* stream) {
  const size_t n16 = bytes / 16;
  hipStream_t s = (hipStream_t)stream;
#define PI(K, R) hipLaunchKernelGGL((probe_items<K, R>), dim3(grid), dim3(256), 0, s, (const uint4*)src, n16, (const uint4*)desc, (uint32_t*)out)
  if (item_kb == 6) PI(6, 4);
  else if (item_kb == 12) PI(12, 8);
  else PI(24, 16);
  return (int)hipGetLastError();
}

// Shader clock over ~3 us: s_memtime (core clock) against s_memrealtime
// (100 MHz), one lane; out[0] = clock ticks, out[1] = 100-MHz ticks.
__global__ void probe_clock(unsigned long long* __restrict__ out) {
  if (threadIdx.x != 0) return;
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  unsigned long long r1;
  do {
    r1 = __builtin_amdgcn_s_memrealtime();
  } while (r1 - r0 < 300);
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[0] = t1 - t0;
  out[1] = r1 - r0;
}
extern "C" int probe_clock_launch(void* out, void* stream) {
  hipLaunchKernelGGL(probe_clock, dim3(1), dim3(64), 0, (hipStream_t)stream, (unsigned long long*)out);
  return (int)hipGetLastError();
}
