// wgcs_kernels.h -- host-side launch entry points of the gfx950 kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/wgcsum.h"
#include "wgcs_host.h"

namespace wgcs {

hipError_t launch_checksum_batch(int mode, unsigned flags, uint8_t* arena, const wgcs_pkt* pkts,
                                 const uint64_t* init, uint32_t n, void* out, hipStream_t s, int num_cu,
                                 const LaunchTuning& tune);

// the resident per-call ring (gso_kernels.hip): nb workgroups serve the
// requests of ctl (coherent pinned host memory) until its stop word or
// idle_ticks (100 MHz) without a request
hipError_t launch_ring(RingCtl* ctl, uint32_t nb, uint32_t last, uint64_t idle_ticks, hipStream_t s);
void gso_kernel_shape(int* lds_waves, int* parts, int* u, int* rows);
hipError_t launch_gso_split_batch(const uint8_t* arena, const wgcs_gso_job* jobs, uint32_t n_jobs,
                                  uint8_t* out, uint32_t out_stride, uint32_t offset, uint32_t max_segs,
                                  int32_t* sizes, int32_t* count, int32_t* status,
                                  hipStream_t s, const GsoOutPos* outpos = nullptr, uint32_t room = 0);

// Device-resident batch of handleGRO calls (gro_batch_kernels.hip).
hipError_t launch_gro_batch(uint8_t* arena, wgcs_gro_buf* bufs, const wgcs_gro_call* calls, uint32_t n_calls,
                            int32_t* status, int32_t* n_write, int32_t* to_write, hipStream_t s);

hipError_t launch_ws_scatter(const uint8_t* stage, uint8_t* arena, const WsMove* mv, uint32_t n, hipStream_t s);
hipError_t launch_ws_gather(const uint8_t* arena, const wgcs_gro_buf* bufs, const wgcs_gro_call* calls,
                            const WsOut* outs, uint32_t n_calls, int32_t* status, const int32_t* n_write,
                            const int32_t* to_write, int32_t* wlen, int32_t* wpos, uint8_t* out, hipStream_t s);

hipError_t launch_gro_coalesce(const uint8_t* stage, const GroItem* items, uint32_t n_items, const GroSeg* segs,
                               uint32_t n_segs, uint8_t* out, hipStream_t s);

// Outer-UDP message batching (conn/bind.go:542-662), udp_msgs_kernels.hip.
hipError_t launch_udp_split(const uint8_t* in, uint64_t in_stride, uint32_t buf_len, const int32_t* n_in,
                            const int32_t* gso, uint32_t n_msgs, uint32_t first, uint32_t n_batches, uint8_t* out,
                            uint64_t out_stride, int32_t* n_out, int32_t* src, int32_t* count, int32_t* status,
                            hipStream_t s);
hipError_t launch_udp_coalesce(uint8_t* bufs, uint64_t stride, uint32_t buf_cap, const int32_t* caps,
                               const int32_t* lens, const int32_t* nbufs, uint32_t max_bufs, uint32_t n_batches,
                               int dst_is_v6, int32_t* n_msgs, int32_t* msg_first, int32_t* msg_len,
                               int32_t* msg_gso, hipStream_t s);

}  // namespace wgcs
