// Helpers shared by the uniform-layout kernels (crc32c_uniform.hip,
// crc32c_stream.hip): block geometry on the end-aligned word grid, bounded
// buffer resources per block, row loads and the row-0 fix-ups.
#ifndef LVKV_CRC32C_UNIFORM_COMMON_H_
#define LVKV_CRC32C_UNIFORM_COMMON_H_

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_device_common.h"
#include "lvkv_kernel_args.h"

namespace lvkv {
namespace {

constexpr int kUniCachePolicy = 2;  // nt: block bytes are read once

enum : int {
  kUniProbeStamps = 64,
  kUniFillFirst = 128,  // probe: generate the row tables before any load
  kUniNoCompute = 1,    // probe: xor the words instead of the table walk
  kUniNoLoads = 2,      // probe: synthetic words instead of block loads
};

struct UniGeo {  // wave-uniform, loop-invariant
  uint32_t rows, nchunks, delta, s0l, s0, spill, nrec;
  int32_t vb0;
};


__device__ __forceinline__ UniGeo uni_geo(const UniformArgs& a) {
  UniGeo g;
  const uint32_t q = (a.length + 3u) >> 2;
  g.rows = (q + 63u) >> 6;
  g.nchunks = (g.rows + kRowsPerChunk - 1) / kRowsPerChunk;
  g.delta = 4u * q - a.length;
  g.s0l = 64u * g.rows - q;
  g.s0 = a.init ^ 0xffffffffu;
  g.spill = g.delta ? (g.s0 >> (32u - 8u * g.delta)) : 0u;
  g.nrec = 4u * q;
  g.vb0 = -4 * static_cast<int32_t>(g.s0l);
  return g;
}

// Row-0 fix-ups of a block's first chunk (see prep_chunk in crc32c_kernel.hip).
__device__ __forceinline__ void fix_first_chunk(uint32_t (&buf)[kRowsPerChunk],
                                                const UniGeo& g) {
  const uint32_t lane = lane_id();
  const uint32_t sh = 8u * g.delta;
  uint32_t w = buf[0];
  w = (lane < g.s0l) ? 0u : w;
  w = (lane == g.s0l) ? ((w & (0xffffffffu << sh)) ^ (g.s0 << sh)) : w;
  w = (lane == g.s0l + 1u) ? (w ^ g.spill) : w;
  buf[0] = w;
  if (g.s0l == 63u) buf[1] = (lane == 0) ? (buf[1] ^ g.spill) : buf[1];
}

template <int P>
__device__ __forceinline__ void stamp_uni(const UniformArgs& a, uint32_t gw, int slot) {
  if (P & kUniProbeStamps) {
    const uint64_t t = __builtin_amdgcn_s_memrealtime();
    if (lane_id() == 0) a.stamps[gw * 8u + slot] = t;
  }
}

template <int P>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t block_rsrc(
    const UniformArgs& a, const UniGeo& g, uint32_t block, bool valid) {
  const uint64_t ptr = reinterpret_cast<uint64_t>(a.base) +
                       static_cast<uint64_t>(valid ? block : 0u) * a.stride -
                       g.delta;
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(ptr));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(ptr >> 32));
  const uint32_t n = __builtin_amdgcn_readfirstlane(valid ? g.nrec : 0u);
  return __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<void*>((static_cast<uint64_t>(hi) << 32) | lo), 0,
      static_cast<int>(n), kBufferDword3);
}

// Row j of a block, j >= 0. Only row 0 can start before the block (vo < 0:
// those lanes read zeros through the bounded window and are masked by
// fix_first_chunk); rows >= 1 are addressed from vo1 = vo + 256 >= 4, kept
// opaque so the compiler cannot re-fold it into a negative voffset with a
// positive immediate (the range check would then reject the whole load).
__device__ __forceinline__ uint32_t load_word(__amdgpu_buffer_rsrc_t r,
                                              int32_t vo, int32_t vo1, int j) {
  if (j == 0) return __builtin_amdgcn_raw_buffer_load_b32(r, vo, 0, kUniCachePolicy);
  return __builtin_amdgcn_raw_buffer_load_b32(r, vo1 + 256 * (j - 1), 0, kUniCachePolicy);
}

}  // namespace
}  // namespace lvkv

#endif  // LVKV_CRC32C_UNIFORM_COMMON_H_
