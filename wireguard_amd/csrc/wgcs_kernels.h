// wgcs_kernels.h -- host-side launch entry points of the gfx950 kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/wgcsum.h"

namespace wgcs {

struct LaunchTuning {
  int blocks_per_cu = 8;   // 256-thread blocks per CU for the persistent grid
  int lanes_per_pkt = 16;  // 16: one DPP row per packet (4 per wave); 64: one wave per packet
  int unroll = 6;          // 16-byte loads in flight per lane per iteration
  int nt = 0;              // non-temporal (streaming) loads
};

hipError_t launch_checksum_batch(int mode, unsigned flags, uint8_t* arena, const wgcs_pkt* pkts,
                                 const uint64_t* init, uint32_t n, void* out, hipStream_t s, int num_cu,
                                 const LaunchTuning& tune);

hipError_t launch_gso_split_batch(const uint8_t* arena, const wgcs_gso_job* jobs, uint32_t n_jobs,
                                  uint8_t* out, uint32_t out_stride, uint32_t offset, uint32_t max_segs,
                                  int32_t* sizes, int32_t* count, int32_t* status, hipStream_t s,
                                  int num_cu);

}  // namespace wgcs
