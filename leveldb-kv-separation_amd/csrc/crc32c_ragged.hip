// General-layout batch CRC32C (per-block offsets and lengths, any alignment,
// every KernelArgs mode) on the compact 64 KiB LDS image, so two 512-thread
// workgroups share a CU (crc32c_kernel.hip's 160 KiB image allows one). The
// walk itself is ragged_run (crc32c_ragged_body.h), shared with the fused
// whole-SSTable verify.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_compact_common.h"
#include "crc32c_device_common.h"
#include "crc32c_ragged_body.h"
#include "lvkv_crc32c.h"
#include "lvkv_kernel_args.h"

namespace lvkv {
namespace {

template <int W, int NCH, int R>
__global__ void __launch_bounds__(64 * W, 2)
    crc32c_ragged_kernel(KernelArgs a, const uint32_t* zpow, const uint32_t* lane_cols) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[RagLds<W>::kDwords];
  const uint32_t total = a.count != nullptr ? min(a.nblocks, sload_u32(a.count, 0)) : a.nblocks;
  ragged_run<W, NCH, R>(a, zpow, lane_cols, lds, blockIdx.x, gridDim.x, total, false);
}

}  // namespace

// cfg: shape = cfg & 3, or cfg >> 3 for the small-record shapes (1: 8 waves
// x 4 chains x 8 rows; 2: 8 x 6 x 8; 3: 8 x 8 x 4); the large-record shapes
// (cfg < 8) are 0: 8 x 2 x 24; 1: 8 x 3 x 16; 2: 8 x 2 x 32; 3: 8 x 3 x 24,
// and cfg & 4 asks for one round per workgroup (grid sized to the batch)
// instead of at most two workgroups per CU.
int ragged_blocks_per_round(int cfg) {
  switch (cfg >> 3) {
    case 1: return 8 * 4;
    case 2: return 8 * 6;
    case 3: return 8 * 8;
  }
  return ((cfg & 3) == 1 || (cfg & 3) == 3) ? 8 * 3 : 8 * 2;
}

hipError_t launch_crc32c_ragged(const KernelArgs& a, const uint32_t* zpow,
                                const uint32_t* lane_cols, int cfg, int num_groups,
                                hipStream_t stream) {
  const int shape = cfg >= 8 ? 4 + (cfg >> 3) : (cfg & 3);
  switch (shape) {
#define LVKV_RAG_CASE(c, w, nch, r)                                                            \
  case c:                                                                                      \
    hipLaunchKernelGGL((crc32c_ragged_kernel<w, nch, r>), dim3(num_groups), dim3(64 * w), 0,   \
                       stream, a, zpow, lane_cols);                                            \
    break;
    LVKV_RAG_CASE(0, 8, 2, 24)
    LVKV_RAG_CASE(1, 8, 3, 16)
    LVKV_RAG_CASE(2, 8, 2, 32)
    LVKV_RAG_CASE(3, 8, 3, 24)
    LVKV_RAG_CASE(5, 8, 4, 8)
    LVKV_RAG_CASE(6, 8, 6, 8)
    LVKV_RAG_CASE(7, 8, 8, 4)
#undef LVKV_RAG_CASE
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_crc32c_batch(const KernelArgs& args, bool uniform_aligned, int num_groups,
                               hipStream_t stream);

hipError_t launch_crc32c_long(const KernelArgs& args, const uint32_t* zpow,
                              const uint32_t* lane_cols, int num_groups, hipStream_t stream);

// General-layout batch (a.offsets set, a.row_tab = the device tables) on
// `cus` CUs; a.nblocks is the launch's capacity when a.count is set. Blocks
// over kLongBytes are included when a.long_split is set.
hipError_t launch_crc32c_general(const KernelArgs& a, int cus, hipStream_t stream) {
  const uint32_t n = a.nblocks;
  if (n == 0) return hipSuccess;
  // (kModeSstTable exists in this kernel only)
  const bool log = a.mode == kModeLogVerify || a.mode == kModeLogFill;
  // a.general_cfg: a ragged cfg (>= 0) or -1 for crc32c_kernel.hip's
  // persistent kernel; a.log_cfg: the shape for WAL records (the device
  // context's choices, lvkv_capi.cpp)
  int cfg = log && a.general_cfg >= 0 ? a.log_cfg : a.general_cfg;
  if (a.mode == kModeSstTable && cfg < 0) cfg = 0;
  if (cfg < 0) {  // the persistent kernel and, for long blocks, a second launch
    KernelArgs b = a;
    if (log) b.long_split = 0;  // crc32c_long_kernel has no WAL modes
    const uint32_t want = (n + kWavesPerGroup - 1) / kWavesPerGroup;
    hipError_t e = launch_crc32c_batch(
        b, false, static_cast<int>(min(static_cast<uint32_t>(cus), want)), stream);
    if (e == hipSuccess && b.long_split)
      e = launch_crc32c_long(b, b.row_tab + kZPowOffset,
                             b.row_tab + kRowTabDwords + kLaneTabDwords, cus, stream);
    return e;
  }
  const uint32_t per = static_cast<uint32_t>(ragged_blocks_per_round(cfg));
  const uint32_t rounds1 = (n + per - 1) / per;
  const uint32_t groups =
      (cfg & 4) ? min(rounds1, 1u << 20) : min(2u * static_cast<uint32_t>(cus), rounds1);
  return launch_crc32c_ragged(a, a.row_tab + kZPowOffset, a.row_tab + kRowTabDwords + kLaneTabDwords,
                              cfg, static_cast<int>(groups), stream);
}

}  // namespace lvkv
