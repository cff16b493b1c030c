// Uniform-layout batch CRC32C for gfx950, "burst" schedule: every wave issues
// ALL of its row loads (every chain, every row, row-interleaved) before the
// workgroup builds its LDS image, so the whole batch is requested from HBM in
// the first few hundred cycles of the launch and the table build hides under
// the first HBM round trip. Arithmetic and LDS image are those of
// crc32c_compact_common.h (end-aligned word grid, Horner over 256-byte rows
// with Z_256 byte tables, lane end shift Z_{256-4s}, DPP xor-reduce).
//
// Reference: util/crc32c.cc:276-377 (Extend), util/crc32c.h:20-32 (Value,
// Mask); the batch is what benchmarks/db_bench_new.cc:782-799 loops over.
//
// Work map: the batch is split into gridDim.x contiguous runs of equal length
// (+1 for the first nblocks % G); run element i goes to wave i % W, chain
// i / W, so a wave's valid chains are a prefix. Blocks are <= 16 rows
// (4 KiB + 252 B); the host checks n <= G * W * NCH.
//
// vmcnt discipline: the lane-column load is issued first, then the rows in
// walk order, all unconditionally (rows past a short block are outside its
// buffer window and return zeros without a memory access), so every wait the
// compiler places is a counted vmcnt(N) on exactly the loads it consumes.
#ifndef LVKV_CRC32C_BURST_H_
#define LVKV_CRC32C_BURST_H_

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_compact_common.h"
#include "crc32c_device_common.h"
#include "crc32c_uniform_common.h"
#include "lvkv_kernel_args.h"

namespace lvkv {

// Probe flags (tools/probe only; the product instantiates 0).
enum : int {
  kBurstBare = 1,      // loads + xor: no tables, no walk
  kBurstNoBuild = 2,   // walk an unbuilt image (timing only)
  kBurstNoWalk = 4,    // build the image, xor the rows instead of walking
  kBurstLate = 8,      // chain 0 before the build, the others after the barrier
  kBurstRowsHbm = 16,  // row tables copied from HBM instead of generated
  kBurstDefaultPolicy = 32,  // default cache policy instead of nt
  kBurstStamps = 64,   // per-wave s_memrealtime stamps (UniformArgs::stamps)
  kBurstSplit2 = 128,  // full blocks walked as 2 independent 8-row groups
  kBurstSplit4 = 256,  // ... as 4 independent 4-row groups
  kBurstPipe1 = 512,   // chain-pipelined: walk chain c, then issue chain c + 1
  kBurstPipe2 = 1024,  // ... two chains ahead: walk c, then issue c + 2
};

namespace {

// Row tables generated from the 32 columns of Z_256 (kernel arguments):
// 2048 16-byte slots q -> row b = q >> 3, table t = (q >> 1) & 3, copies
// 4h..4h+3 with h = q & 1 (address b*256 + 32t + 16h). Eight consecutive
// lanes cover one row's 128 B: conflict-free ds_write_b128.
template <int W>
__device__ __forceinline__ void burst_fill_rows(uint32_t* lds, const UniformArgs& a,
                                                uint32_t tid) {
  constexpr int kThreads = 64 * W;
  constexpr int kIters = 2048 / kThreads;
  const uint32_t t = (tid >> 1) & 3u;
  uint32_t col[8];
#pragma unroll
  for (int bit = 0; bit < 8; ++bit) {
    const uint32_t c01 = (t & 1u) ? a.zcol[8 + bit] : a.zcol[bit];
    const uint32_t c23 = (t & 1u) ? a.zcol[24 + bit] : a.zcol[16 + bit];
    col[bit] = (t & 2u) ? c23 : c01;
  }
#pragma unroll
  for (int it = 0; it < kIters; ++it) {
    const uint32_t q = tid + static_cast<uint32_t>(kThreads * it);
    const uint32_t b = q >> 3;
    uint32_t e = 0;
#pragma unroll
    for (int bit = 0; bit < 8; ++bit) e ^= (0u - ((b >> bit) & 1u)) & col[bit];
    *reinterpret_cast<uint4*>(reinterpret_cast<char*>(lds) + b * 256u + (q & 7u) * 16u) =
        make_uint4(e, e, e, e);
  }
}

template <int F>
__device__ __forceinline__ void burst_stamp(const UniformArgs& a, uint32_t gw, int slot) {
  if (F & kBurstStamps) {
    const uint64_t t = __builtin_amdgcn_s_memrealtime();
    if (lane_id() == 0) a.stamps[gw * 8u + slot] = t;
  }
}

template <int F>
__device__ __forceinline__ uint32_t burst_load(__amdgpu_buffer_rsrc_t r, int32_t vo, int32_t vo1,
                                               int j) {
  constexpr int kPol = (F & kBurstDefaultPolicy) ? 0 : kUniCachePolicy;
  if (j == 0) return __builtin_amdgcn_raw_buffer_load_b32(r, vo, 0, kPol);
  return __builtin_amdgcn_raw_buffer_load_b32(r, vo1 + 256 * (j - 1), 0, kPol);
}

// Wave-uniform v -> Z_{2^j}(v): four scalar loads from the zpow set j.
__device__ __forceinline__ uint32_t zpow_uniform(const uint32_t* zpow, uint32_t j, uint32_t v) {
  const uint32_t* t = zpow + j * 1024u;
  return sload_u32(t, v & 255u) ^ sload_u32(t, 256u + ((v >> 8) & 255u)) ^
         sload_u32(t, 512u + ((v >> 16) & 255u)) ^ sload_u32(t, 768u + (v >> 24));
}

// One wave with NV valid chains (blocks blk[0..NV)); `live` false: a wave
// past the batch (tiny batches) walks an empty window and stores nothing.
template <int F, int W, int NV, bool FULL>
__device__ __forceinline__ void burst_body(const UniformArgs& a, const UniGeo& g, uint32_t* lds,
                                           uint32_t tid, uint32_t lane, const uint32_t* blk,
                                           bool live) {
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t gw = blockIdx.x * W + wave;
  // The image is built by the first kBuild waves (all of them when W is a
  // power of two; the first 8 of a 10- or 12-wave workgroup).
  constexpr int kBuild = (W & (W - 1)) == 0 ? W : 8;
  const bool builder = wave < static_cast<uint32_t>(kBuild);
  burst_stamp<F>(a, gw, 0);
  __amdgpu_buffer_rsrc_t r[NV];
#pragma unroll
  for (int c = 0; c < NV; ++c) r[c] = block_rsrc<0>(a, g, blk[c], live);
  const int32_t vo = g.vb0 + 4 * static_cast<int32_t>(lane);
  int32_t vo1 = vo + kRowBytes;
  asm volatile("" : "+v"(vo1));
  uint32_t w[NV][kRowsPerChunk];
  // Split walk (full blocks only): G groups of R rows each, group k = rows
  // [kR, kR + R); loads issued in consumption order (step-major).
  constexpr int G = !FULL ? 1 : (F & kBurstSplit4) ? 4 : (F & kBurstSplit2) ? 2 : 1;
  constexpr int R = kRowsPerChunk / G;
  auto load_rows = [&](int c_lo, int c_hi) {
#pragma unroll
    for (int t = 0; t < R; ++t)
#pragma unroll
      for (int k = 0; k < G; ++k)
#pragma unroll
        for (int c = 0; c < NV; ++c) {
          const int j = k * R + t;
          if (c >= c_lo && c < c_hi && (FULL || static_cast<uint32_t>(j) < g.rows))
            w[c][j] = burst_load<F>(r[c], vo, vo1, j);
        }
  };

  if (F & kBurstBare) {
    load_rows(0, NV);
    uint32_t x = 0;
#pragma unroll
    for (int j = 0; j < kRowsPerChunk; ++j)
#pragma unroll
      for (int c = 0; c < NV; ++c)
        if (FULL || static_cast<uint32_t>(j) < g.rows) x ^= w[c][j];
    x = wave_xor_dpp(x);
    if (lane == 0 && live)
#pragma unroll
      for (int c = 0; c < NV; ++c) a.out[blk[c]] = x;
    return;
  }

  if (F & (kBurstPipe1 | kBurstPipe2)) {
    // Chain pipeline: the first D chains' rows go out before the image; then
    // each chain is walked, reduced and stored as soon as its rows land, and
    // the chain D ahead is issued after it, so a wave's row loads never sit
    // between it and the walk of data that has already arrived.
    constexpr int D = (F & kBurstPipe2) ? 2 : 1;
    LaneTabGen<kBuild> lg;
    if (builder) lg.load(a.lane_cols, wave, lane);
    __builtin_amdgcn_sched_barrier(0);
    load_rows(0, D < NV ? D : NV);
    __builtin_amdgcn_sched_barrier(0);
    burst_stamp<F>(a, gw, 1);
    if (builder) burst_fill_rows<kBuild>(lds, a, tid);
    burst_stamp<F>(a, gw, 3);
    if (builder) lg.store(lds, wave, lane);
    burst_stamp<F>(a, gw, 5);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    burst_stamp<F>(a, gw, 2);
    const LaneKeys keys = lane_keys(lane);
    const uint32_t lane_base = compact_lane_base(lane);
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      fix_first_chunk(w[c], g);
      uint32_t crc;
      if (G > 1) {
        // G independent R-row groups (ILP within the chain), Horner-combined
        uint32_t sg[G];
#pragma unroll
        for (int k = 0; k < G; ++k) sg[k] = w[c][k * R];
#pragma unroll
        for (int t = 1; t < R; ++t)
#pragma unroll
          for (int k = 0; k < G; ++k) sg[k] = row_step_c(lds, sg[k], w[c][k * R + t], keys);
        constexpr uint32_t kJ = (R == 8) ? 11u : (R == 4) ? 10u : 0u;  // log2(R * 256)
        uint32_t v = wave_xor_dpp(lane_end_shift_c(lds, sg[0], lane_base));
#pragma unroll
        for (int k = 1; k < G; ++k)
          v = zpow_uniform(a.zpow, kJ, v) ^ wave_xor_dpp(lane_end_shift_c(lds, sg[k], lane_base));
        crc = v ^ 0xffffffffu;
      } else {
        uint32_t st = w[c][0];
#pragma unroll
        for (int j = 1; j < kRowsPerChunk; ++j)
          if (FULL || static_cast<uint32_t>(j) < g.rows) st = row_step_c(lds, st, w[c][j], keys);
        crc = wave_xor_dpp(lane_end_shift_c(lds, st, lane_base)) ^ 0xffffffffu;
      }
      if (lane == 0 && live) a.out[blk[c]] = a.mask ? crc_mask(crc) : crc;
      if (c < 2) burst_stamp<F>(a, gw, 6 + c);
      __builtin_amdgcn_sched_barrier(0);
      if (c + D < NV) load_rows(c + D, c + D + 1);
      __builtin_amdgcn_sched_barrier(0);
    }
    burst_stamp<F>(a, gw, 4);
    return;
  }

  // 1. Lane columns, then every row of every chain (or only chain 0).
  LaneTabGen<kBuild> lg;
  RowTabStage<64 * kBuild> rt;
  if (!(F & kBurstNoBuild) && builder) {
    lg.load(a.lane_cols, wave, lane);
    if (F & kBurstRowsHbm) rt.load(a.zpow, tid);
  }
  __builtin_amdgcn_sched_barrier(0);
  load_rows(0, (F & kBurstLate) ? 1 : NV);
  __builtin_amdgcn_sched_barrier(0);
  burst_stamp<F>(a, gw, 1);
  // 2. The LDS image, one barrier.
  if (!(F & kBurstNoBuild) && builder) {
    if (F & kBurstRowsHbm)
      rt.store(lds, tid);
    else
      burst_fill_rows<kBuild>(lds, a, tid);
    lg.store(lds, wave, lane);
  }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  burst_stamp<F>(a, gw, 2);
  if (F & kBurstLate) load_rows(1, NV);

  // 3. Rows, chains interleaved; row-0 fix-ups first.
  uint32_t st[NV];
  if (F & kBurstNoWalk) {
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      fix_first_chunk(w[c], g);
      st[c] = w[c][0];
    }
#pragma unroll
    for (int j = 1; j < kRowsPerChunk; ++j)
      if (FULL || static_cast<uint32_t>(j) < g.rows)
#pragma unroll
        for (int c = 0; c < NV; ++c) st[c] ^= w[c][j];
  } else if (G > 1) {
    const LaneKeys keys = lane_keys(lane);
    uint32_t sg[NV][G];
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      fix_first_chunk(w[c], g);
#pragma unroll
      for (int k = 0; k < G; ++k) sg[c][k] = w[c][k * R];
    }
#pragma unroll
    for (int t = 1; t < R; ++t)
#pragma unroll
      for (int k = 0; k < G; ++k)
#pragma unroll
        for (int c = 0; c < NV; ++c) sg[c][k] = row_step_c(lds, sg[c][k], w[c][k * R + t], keys);
    burst_stamp<F>(a, gw, 3);
    const uint32_t lane_base = compact_lane_base(lane);
    uint32_t red[NV][G];
#pragma unroll
    for (int k = 0; k < G; ++k)
#pragma unroll
      for (int c = 0; c < NV; ++c) red[c][k] = wave_xor_dpp(lane_end_shift_c(lds, sg[c][k], lane_base));
    // Horner over the groups: each group ends R * 256 bytes before the next.
    constexpr uint32_t kJ = (R == 8) ? 11u : (R == 4) ? 10u : 0u;  // log2(R * 256)
    uint32_t crc[NV];
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      uint32_t v = red[c][0];
#pragma unroll
      for (int k = 1; k < G; ++k) v = zpow_uniform(a.zpow, kJ, v) ^ red[c][k];
      crc[c] = v ^ 0xffffffffu;
    }
    if (lane == 0 && live) {
#pragma unroll
      for (int c = 0; c < NV; ++c) a.out[blk[c]] = a.mask ? crc_mask(crc[c]) : crc[c];
    }
    burst_stamp<F>(a, gw, 4);
    return;
  } else {
    const LaneKeys keys = lane_keys(lane);
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      fix_first_chunk(w[c], g);
      st[c] = w[c][0];
    }
#pragma unroll
    for (int j = 1; j < kRowsPerChunk; ++j) {
      if (FULL || static_cast<uint32_t>(j) < g.rows) {
#pragma unroll
        for (int c = 0; c < NV; ++c) st[c] = row_step_c(lds, st[c], w[c][j], keys);
      }
    }
  }
  burst_stamp<F>(a, gw, 3);

  // 4. End shift, reduction, store.
  const uint32_t lane_base = compact_lane_base(lane);
  uint32_t crc[NV];
#pragma unroll
  for (int c = 0; c < NV; ++c)
    crc[c] = wave_xor_dpp(lane_end_shift_c(lds, st[c], lane_base)) ^ 0xffffffffu;
  if (lane == 0 && live) {
#pragma unroll
    for (int c = 0; c < NV; ++c) a.out[blk[c]] = a.mask ? crc_mask(crc[c]) : crc[c];
  }
  burst_stamp<F>(a, gw, 4);
}

// The kernel body for workgroup blockIdx.x of G (G passed explicitly so the
// AQL engine's dispatches need no hidden kernel arguments).
template <int F, int W, int NCH>
__device__ __forceinline__ void burst_kernel_body(const UniformArgs& a, uint32_t* lds, uint32_t G) {
  static_assert(NCH >= 1 && NCH <= 5, "chains per wave");
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = lane_id();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const UniGeo g = uni_geo(a);
  const uint32_t per = a.nblocks / G, extra = a.nblocks % G;
  const uint32_t n = per + (blockIdx.x < extra ? 1u : 0u);
  const uint32_t start = blockIdx.x * per + min(blockIdx.x, extra);
  uint32_t blk[NCH];
  uint32_t nv = 0;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const uint32_t i = static_cast<uint32_t>(c) * W + wave;
    blk[c] = start + i;
    nv += i < n ? 1u : 0u;
  }
  const bool full = g.rows == static_cast<uint32_t>(kRowsPerChunk);
  // Every body runs the same single barrier.
#define LVKV_BURST_BODY(NV)                                                   \
  if (full)                                                                   \
    burst_body<F, W, NV, true>(a, g, lds, tid, lane, blk, NV > 1 || nv != 0); \
  else                                                                        \
    burst_body<F, W, NV, false>(a, g, lds, tid, lane, blk, NV > 1 || nv != 0);
  if (NCH >= 5 && nv >= 5) {
    LVKV_BURST_BODY((NCH >= 5 ? 5 : 1))
  } else if (NCH >= 4 && nv >= 4) {
    LVKV_BURST_BODY((NCH >= 4 ? 4 : 1))
  } else if (NCH >= 3 && nv >= 3) {
    LVKV_BURST_BODY((NCH >= 3 ? 3 : 1))
  } else if (NCH >= 2 && nv >= 2) {
    LVKV_BURST_BODY((NCH >= 2 ? 2 : 1))
  } else {
    LVKV_BURST_BODY(1)
  }
#undef LVKV_BURST_BODY
}

}  // namespace

// W waves per workgroup, up to NCH chains per wave, OCC workgroups per CU.
template <int F, int W, int NCH, int OCC>
__global__ void __launch_bounds__(64 * W, OCC) crc32c_burst_kernel(UniformArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kCompactLdsBytes / 4];
  burst_kernel_body<F, W, NCH>(a, lds, gridDim.x);
}

}  // namespace lvkv

#endif  // LVKV_CRC32C_BURST_H_
