// Kernels dispatched by the AQL engine (lvkv_engine.cpp). Compiled on their
// own into a gfx950 code object (--genco) that is embedded in
// liblvkv_crc32c.so and loaded through the HSA loader, so the engine can
// write dispatch packets straight into its own hardware queue. The entry
// points are extern "C" (stable symbol names) and read no hidden kernel
// arguments: the workgroup count comes from UniformArgs::ngroups.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_burst.h"
#include "lvkv_kernel_args.h"

// Uniform batches of blocks <= 16 rows (4 KiB + 252 B), <= 24 blocks per
// workgroup of 8 waves, two workgroups per CU (crc32c_burst.h).
extern "C" __global__ void __launch_bounds__(512, 2)
    lvkv_engine_uniform_burst(lvkv::UniformArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[lvkv::kCompactLdsBytes / 4];
  lvkv::burst_kernel_body<0, 8, 3>(a, lds, a.ngroups);
}

// The same with the row tables copied from the Z_256 set of zpow (HBM/L2)
// instead of generated from the columns.
extern "C" __global__ void __launch_bounds__(512, 2)
    lvkv_engine_uniform_burst_rows(lvkv::UniformArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[lvkv::kCompactLdsBytes / 4];
  lvkv::burst_kernel_body<lvkv::kBurstRowsHbm, 8, 3>(a, lds, a.ngroups);
}

// One workgroup per CU per dispatch (8 waves x 5 chains = 40 blocks): a
// dispatch takes half of each CU's LDS and waves, so the next dispatch's
// workgroups are resident beside it and the two overlap (the engine issues
// dispatches without the barrier bit).
extern "C" __global__ void __launch_bounds__(512, 2)
    lvkv_engine_uniform_half(lvkv::UniformArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[lvkv::kCompactLdsBytes / 4];
  lvkv::burst_kernel_body<0, 8, 5>(a, lds, a.ngroups);
}

// The same, chain 0's loads before the LDS image, the others after it.
extern "C" __global__ void __launch_bounds__(512, 2)
    lvkv_engine_uniform_half_late(lvkv::UniformArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[lvkv::kCompactLdsBytes / 4];
  lvkv::burst_kernel_body<lvkv::kBurstLate, 8, 5>(a, lds, a.ngroups);
}

// 8 x 3, chain 0 first (the HIP path's compact schedule).
extern "C" __global__ void __launch_bounds__(512, 2)
    lvkv_engine_uniform_burst_late(lvkv::UniformArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[lvkv::kCompactLdsBytes / 4];
  lvkv::burst_kernel_body<lvkv::kBurstLate, 8, 3>(a, lds, a.ngroups);
}

// Timing builds: per-wave s_memrealtime stamps into UniformArgs::stamps
// (tools/probe; selected by lvkv_engine_set_stamps).
extern "C" __global__ void __launch_bounds__(512, 2)
    lvkv_engine_uniform_burst_stamps(lvkv::UniformArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[lvkv::kCompactLdsBytes / 4];
  lvkv::burst_kernel_body<lvkv::kBurstStamps, 8, 3>(a, lds, a.ngroups);
}
extern "C" __global__ void __launch_bounds__(512, 2)
    lvkv_engine_uniform_half_stamps(lvkv::UniformArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[lvkv::kCompactLdsBytes / 4];
  lvkv::burst_kernel_body<lvkv::kBurstStamps, 8, 5>(a, lds, a.ngroups);
}
extern "C" __global__ void __launch_bounds__(512, 2)
    lvkv_engine_uniform_half_late_stamps(lvkv::UniformArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[lvkv::kCompactLdsBytes / 4];
  lvkv::burst_kernel_body<lvkv::kBurstStamps | lvkv::kBurstLate, 8, 5>(a, lds, a.ngroups);
}
