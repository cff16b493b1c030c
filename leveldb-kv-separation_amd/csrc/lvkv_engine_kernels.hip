// Kernels dispatched by the AQL engine (lvkv_engine.cpp). Compiled on their
// own into a gfx950 code object (--cuda-device-only, unbundled) that is
// embedded in liblvkv_crc32c.so and loaded through the HSA loader, so the
// engine can write dispatch packets straight into its own hardware queues.
// The entry points are extern "C" (stable symbol names) and read no hidden
// kernel arguments: the workgroup count comes from UniformArgs::ngroups.
//
// Arithmetic and schedule: crc32c_burst.h (util/crc32c.cc:276-377 restated
// as an end-aligned Horner walk over 256-byte rows).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_burst.h"
#include "crc32c_ragged_body.h"
#include "lvkv_kernel_args.h"

namespace {
constexpr int kLds = lvkv::kCompactLdsBytes / 4;
}

// Production: one 512-thread workgroup per CU per dispatch, 8 waves x 5
// chains (40 blocks of <= 16 rows). It holds half of a CU's waves and 64 KiB
// of its LDS, so the next dispatch (another queue) runs beside it. Chain 0's
// row loads go out before the LDS image is built, the other chains' after.
extern "C" __global__ void __launch_bounds__(512, 2)
    lvkv_ek_uniform(lvkv::UniformArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kLds];
  lvkv::burst_kernel_body<lvkv::kBurstLate, 8, 5>(a, lds, a.ngroups);
}

// Ordered dispatches (a batch alone on the chip): two workgroups per CU,
// 8 waves x 3 chains, chain-pipelined — each chain is walked and stored as
// soon as its rows land and the next chain's rows go out after it
// (tools/probe/iso_probe.py: 9.7 us against 10.4 us for all rows first).
extern "C" __global__ void __launch_bounds__(512, 2)
    lvkv_ek_uniform_pair(lvkv::UniformArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kLds];
  lvkv::burst_kernel_body<lvkv::kBurstPipe1, 8, 3>(a, lds, a.ngroups);
}

// Timestamp builds of the two (per-wave s_memrealtime into
// UniformArgs::stamps; lvkv_engine_set_stamps, tools/probe/timeline.py).
extern "C" __global__ void __launch_bounds__(512, 2)
    lvkv_ek_uniform_stamps(lvkv::UniformArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kLds];
  lvkv::burst_kernel_body<lvkv::kBurstLate | lvkv::kBurstStamps, 8, 5>(a, lds, a.ngroups);
}
extern "C" __global__ void __launch_bounds__(512, 2)
    lvkv_ek_uniform_pair_stamps(lvkv::UniformArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kLds];
  lvkv::burst_kernel_body<lvkv::kBurstPipe1 | lvkv::kBurstStamps, 8, 3>(a, lds, a.ngroups);
}

// General-layout batches (lvkv_engine_crc32c_batch, the verify and fill
// submits, uniform blocks beyond the burst kernel's 16 rows): the HIP path's
// ragged walk (crc32c_ragged_body.h, ragged_run) over a.k.nblocks blocks,
// two 512-thread workgroups per CU. 8 waves x 2 chains x 24-row chunks for
// SST blocks and compute batches; 8 x 4 x 8 for WAL records (mostly short).
extern "C" __global__ void __launch_bounds__(512, 2)
    lvkv_ek_ragged(lvkv::EngineRaggedArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[lvkv::RagLds<8>::kDwords];
  lvkv::ragged_run<8, 2, 24>(a.k, a.zpow, a.lane_cols, lds, blockIdx.x, a.ngroups, a.k.nblocks,
                             false);
}
extern "C" __global__ void __launch_bounds__(512, 2)
    lvkv_ek_ragged_small(lvkv::EngineRaggedArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[lvkv::RagLds<8>::kDwords];
  lvkv::ragged_run<8, 4, 8>(a.k, a.zpow, a.lane_cols, lds, blockIdx.x, a.ngroups, a.k.nblocks,
                            false);
}

// One round per workgroup, one workgroup per CU per dispatch (the engine cuts
// a batch into dispatches of cus x 8 x NCH blocks and rotates them over its
// queues, so the next dispatch's workgroup runs beside this one, as the
// uniform burst kernel's): every chain's rows are requested before any walk.
// 8 waves x 4 chains x 17 rows (SST blocks up to 4352 B in one chunk) and
// 8 x 6 x 8 (records up to 2 KiB: WAL records, small values).
extern "C" __global__ void __launch_bounds__(512, 2)
    lvkv_ek_ragged_burst(lvkv::EngineRaggedArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[lvkv::RagLds<8>::kDwords];
  lvkv::ragged_run<8, 4, 17>(a.k, a.zpow, a.lane_cols, lds, blockIdx.x, a.ngroups, a.k.nblocks,
                             false);
}
extern "C" __global__ void __launch_bounds__(512, 2)
    lvkv_ek_ragged_burst_small(lvkv::EngineRaggedArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[lvkv::RagLds<8>::kDwords];
  lvkv::ragged_run<8, 6, 8>(a.k, a.zpow, a.lane_cols, lds, blockIdx.x, a.ngroups, a.k.nblocks,
                            false);
}
