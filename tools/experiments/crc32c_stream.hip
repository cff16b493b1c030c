// Streamed uniform-batch CRC32C for gfx950: nblocks blocks of 16 rows
// (3841..4096 bytes, the leveldb block size) at base + i*stride, every block
// END 4-byte aligned, at most 3 blocks per wave of the grid (the 10k x 4 KiB
// headline and the 1k x 4 KiB config).
//
// Same arithmetic as crc32c_kernel.hip / crc32c_uniform.hip (end-aligned word
// grid, Horner over 256-byte rows with the Z_256 LDS tables, per-lane end
// shift Z_{256-4s}, wave xor-reduce). What differs is the schedule:
//
//  * Software pipeline per wave. A wave's blocks (A = gw, B = gw + W, C from
//    the balanced third round) form one stream of 16..48 row loads; the wave
//    keeps a window of `L` row loads in flight and consumes row r (one Horner
//    step) right after issuing row r + L. A block is finished (end shift,
//    reduction, store) as soon as its last row is consumed. Compute therefore
//    tracks the arrival of the bytes instead of starting after the last load
//    is issued (the one-round kernel's waves sat blocked on load issue for
//    most of the launch and walked all rows at the end).
//  * Cheap row-table fill: T_t is linear, so T_t[base ^ 8k] = T_t[base] ^
//    T_t[8k]. Each lane builds T_t[base] from five Z_256 columns once and its
//    eight entries with one xor each against wave-uniform values (scalar
//    unit), instead of eight 8-term selections.
//  * Lane tables (32 KiB, L2-resident) are loaded before any block load and
//    written to LDS with the row tables: one barrier per launch.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_device_common.h"
#include "crc32c_uniform_common.h"
#include "lvkv_kernel_args.h"

namespace lvkv {
namespace {

enum : int {
  kStreamNoLaneTab = 1024,    // probe: no lane tables (end shifts read garbage)
  kStreamCounterSync = 2048,  // fill completion by an LDS arrival counter
                              // instead of a workgroup barrier after it
  kStreamInterleave = 4096,   // stream order row-major over the chains
                              // (A0 B0 C0 A1 ...): independent steps back to back
};

// The arrival counter lives in lane-table slot (k = 0, nib = 0, s = 0): every
// nib = 0 entry is Z(0) = 0, and the k = 0 lookup masks nib = 0 instead of
// reading it.
constexpr uint32_t kLdsSyncCounter = kLdsLaneTabBase;

template <int P>
__device__ __forceinline__ uint32_t end_shift(const uint32_t* lds, uint32_t s,
                                              uint32_t lane_base) {
  if (!(P & kStreamCounterSync)) return lane_end_shift(lds, s, lane_base);
  uint32_t r = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint32_t nib = (s >> (4 * k)) & 15u;
    const uint32_t v = lds_ld(lds, (lane_base | (nib << 8)) + 4096u * k);
    r ^= (k == 0 && nib == 0) ? 0u : v;
  }
  return r;
}

// Spin (with s_sleep) until all 16 waves of the workgroup have published
// their share of the LDS tables.
__device__ __forceinline__ void wait_tables(uint32_t* lds) {
  volatile uint32_t* c = lds + kLdsSyncCounter / 4;
  while (__builtin_amdgcn_readfirstlane(*c) < static_cast<uint32_t>(kWavesPerGroup))
    __builtin_amdgcn_s_sleep(1);
}

// Row tables (LDS image of lvkv_kernel_args.h) from the 32 columns of Z_256.
// Wave w fills table t = w / 4, 16-byte slots v = (w % 4) * 512 + k * 64 +
// lane (k = 0..7): entry i = v >> 3 = base + 8k with base = (w % 4) * 64 +
// (lane >> 3), copies 4 * (lane & 7) .. +3.
__device__ __forceinline__ void fill_row_tables_linear(uint32_t* lds,
                                                       const UniformArgs& a,
                                                       uint32_t wave,
                                                       uint32_t lane) {
  const uint32_t t = wave >> 2;
  const uint32_t* col = a.zcol + 8u * t;
  const uint32_t base = (wave & 3u) * 64u + (lane >> 3);
  uint32_t e0 = 0;
  e0 ^= (0u - (base & 1u)) & col[0];
  e0 ^= (0u - ((base >> 1) & 1u)) & col[1];
  e0 ^= (0u - ((base >> 2) & 1u)) & col[2];
  e0 ^= (0u - ((base >> 6) & 1u)) & col[6];
  e0 ^= (0u - ((base >> 7) & 1u)) & col[7];
  const uint32_t c3 = col[3], c4 = col[4], c5 = col[5];
  char* dst = reinterpret_cast<char*>(lds) + (t >> 1) * kLdsRowRegionBytes +
              (t & 1u) * 128u + base * 256u + (lane & 7u) * 16u;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint32_t kv = ((k & 1) ? c3 : 0u) ^ ((k & 2) ? c4 : 0u) ^ ((k & 4) ? c5 : 0u);
    const uint32_t e = e0 ^ kv;
    *reinterpret_cast<uint4*>(dst + k * 8 * 256) = make_uint4(e, e, e, e);
  }
}

__device__ __forceinline__ uint32_t fix_row0(uint32_t w, const UniGeo& g, uint32_t lane) {
  const uint32_t sh = 8u * g.delta;
  w = (lane < g.s0l) ? 0u : w;
  w = (lane == g.s0l) ? ((w & (0xffffffffu << sh)) ^ (g.s0 << sh)) : w;
  return (lane == g.s0l + 1u) ? (w ^ g.spill) : w;
}

__device__ __forceinline__ uint32_t fix_row1(uint32_t w, const UniGeo& g, uint32_t lane) {
  return (g.s0l == 63u && lane == 0) ? (w ^ g.spill) : w;
}

// One wave's stream over NSEG blocks (NSEG = 1..3). valid0 = false only for a
// wave past the end of the batch (it runs over an empty window and stores
// nothing, but still takes part in the workgroup's fill and barrier).
template <int P, int NSEG, int L, int PRE>
__device__ __forceinline__ void stream_body(const UniformArgs& a, const UniGeo& g,
                                            uint32_t* lds, uint32_t tid, uint32_t lane,
                                            uint32_t wave, uint32_t gw,
                                            const uint32_t (&blk)[3], bool valid0) {
  constexpr int R = kRowsPerChunk * NSEG;
  constexpr int kLaneIters = (kLaneTabDwords / 4) / kGroupThreads;  // 2

  static_assert(kLaneIters == 2, "lane tables: two 16-byte slots per thread");
  constexpr bool kSync = (P & kStreamCounterSync) != 0;
  const uint4* lsrc = reinterpret_cast<const uint4*>(a.lane_tab) + tid;
  uint4 lt0 = {}, lt1 = {};
  if (!(P & kStreamNoLaneTab)) {
    lt0 = lsrc[0];
    lt1 = lsrc[kGroupThreads];
  }

  // (three named resources, not an array: an array of resources is kept in
  // scratch by the compiler)
  const __amdgpu_buffer_rsrc_t r0 = block_rsrc<P>(a, g, blk[0], valid0);
  const __amdgpu_buffer_rsrc_t r1 = block_rsrc<P>(a, g, NSEG > 1 ? blk[1] : 0u, NSEG > 1);
  const __amdgpu_buffer_rsrc_t r2 = block_rsrc<P>(a, g, NSEG > 2 ? blk[2] : 0u, NSEG > 2);
  const int32_t vo = g.vb0 + 4 * static_cast<int32_t>(lane);
  int32_t vo1 = vo + kRowBytes;
  asm volatile("" : "+v"(vo1));

  uint32_t w[R];
  constexpr bool kIlv = (P & kStreamInterleave) != 0;
  // stream position i -> (chain, row)
  auto chain_of = [](int i) { return kIlv ? i % NSEG : i / kRowsPerChunk; };
  auto row_of = [](int i) { return kIlv ? i / NSEG : i % kRowsPerChunk; };
  auto issue = [&](int i) {
    if (i < R) {
      const int c = chain_of(i);
      w[i] = load_word(c == 0 ? r0 : (c == 1 ? r1 : r2), vo, vo1, row_of(i));
    }
  };
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < PRE && i < L; ++i) issue(i);
  __builtin_amdgcn_sched_barrier(0);
  stamp_uni<P>(a, gw, 3);
  fill_row_tables_linear(lds, a, wave, lane);
  if (!(P & kStreamNoLaneTab)) {
    uint4* ldst = reinterpret_cast<uint4*>(lds + kLdsLaneTabBase / 4) + tid;
    if (!kSync || tid != 0) ldst[0] = lt0;  // slot 0 holds the counter
    ldst[kGroupThreads] = lt1;
  }
  if (kSync) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_fetch_add(lds + kLdsSyncCounter / 4, 1u, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_WORKGROUP);
  } else {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  __builtin_amdgcn_sched_barrier(0);
  stamp_uni<P>(a, gw, 1);
#pragma unroll
  for (int i = PRE; i < L; ++i) issue(i);
  if (kSync) {
    __builtin_amdgcn_sched_barrier(0);
    wait_tables(lds);
    __builtin_amdgcn_sched_barrier(0);
  }

  const uint32_t k0 = (lane & 31u) * 4u;
  const uint32_t k1 = k0 | 0x10000u;
  const uint32_t lane_base = kLdsLaneTabBase + lane * 4u;
  uint32_t st[NSEG];
#pragma unroll
  for (int rr = 0; rr < R; ++rr) {
    const int c = chain_of(rr), j = row_of(rr);
    issue(rr + L);
    uint32_t x = w[rr];
    if (j == 0) x = fix_row0(x, g, lane);
    if (j == 1) x = fix_row1(x, g, lane);
    st[c] = (j == 0) ? x : row_step(lds, st[c], x, k0, k1);
    if (j == kRowsPerChunk - 1) {
      const uint32_t crc = wave_xor_dpp(end_shift<P>(lds, st[c], lane_base)) ^ 0xffffffffu;
      if (lane == 0 && (c > 0 || valid0)) a.out[blk[c]] = a.mask ? crc_mask(crc) : crc;
    }
  }
  stamp_uni<P>(a, gw, 2);
}

}  // namespace

template <int P, int L, int PRE>
__global__ void __launch_bounds__(kGroupThreads, 1)
    crc32c_stream_kernel(UniformArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsBytes / 4];
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = lane_id();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t nwaves = gridDim.x * kWavesPerGroup;
  const uint32_t gw = blockIdx.x * kWavesPerGroup + wave;
  stamp_uni<P>(a, gw, 0);
  if (P & kStreamCounterSync) {  // zero the arrival counter before any arrives
    if (tid == 0) lds[kLdsSyncCounter / 4] = 0;
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  const UniGeo g = uni_geo(a);
  // Third round (nc = nblocks - 2W blocks) in equal contiguous runs per
  // workgroup, so every CU streams the same number of bytes. A wave's valid
  // blocks are a prefix (C valid => B valid => A valid).
  const uint32_t nc = a.nblocks > 2u * nwaves ? a.nblocks - 2u * nwaves : 0u;
  const uint32_t per = nc / gridDim.x, extra = nc % gridDim.x;
  const uint32_t run_len = per + (blockIdx.x < extra ? 1u : 0u);
  const uint32_t run_start = blockIdx.x * per + min(blockIdx.x, extra);
  const uint32_t blk_c = wave < run_len ? 2u * nwaves + run_start + wave : 0xffffffffu;
  const uint32_t blk[3] = {gw, gw + nwaves, blk_c};
  if (blk[2] < a.nblocks)
    stream_body<P, 3, L, PRE>(a, g, lds, tid, lane, wave, gw, blk, true);
  else if (blk[1] < a.nblocks)
    stream_body<P, 2, L, PRE>(a, g, lds, tid, lane, wave, gw, blk, true);
  else
    stream_body<P, 1, L, PRE>(a, g, lds, tid, lane, wave, gw, blk, blk[0] < a.nblocks);
  stamp_uni<P>(a, gw, 7);
}

// cfg selects the pipeline shape (window L, loads issued before the fill);
// bit 64 adds per-wave timestamps (probe builds). cfg 0 is production.
hipError_t launch_crc32c_stream(const UniformArgs& args, int cfg, int num_groups,
                                hipStream_t stream) {
  switch (cfg) {
#define LVKV_STREAM_CASE(c, l, pre)                                              \
  case c:                                                                        \
    hipLaunchKernelGGL((crc32c_stream_kernel<0, l, pre>), dim3(num_groups),      \
                       dim3(kGroupThreads), 0, stream, args);                    \
    break;                                                                       \
  case c + 64:                                                                   \
    hipLaunchKernelGGL((crc32c_stream_kernel<kUniProbeStamps, l, pre>),          \
                       dim3(num_groups), dim3(kGroupThreads), 0, stream, args);  \
    break;
    LVKV_STREAM_CASE(0, 24, 16)
    LVKV_STREAM_CASE(1, 16, 16)
    LVKV_STREAM_CASE(2, 32, 16)
    LVKV_STREAM_CASE(3, 40, 16)
    LVKV_STREAM_CASE(4, 48, 16)
    LVKV_STREAM_CASE(5, 16, 0)
    LVKV_STREAM_CASE(6, 24, 8)
    LVKV_STREAM_CASE(7, 12, 12)
    LVKV_STREAM_CASE(8, 32, 32)
#undef LVKV_STREAM_CASE
#define LVKV_STREAM_PROBE(c, p, l, pre)                                          \
  case c:                                                                        \
    hipLaunchKernelGGL((crc32c_stream_kernel<p, l, pre>), dim3(num_groups),      \
                       dim3(kGroupThreads), 0, stream, args);                    \
    break;                                                                       \
  case c + 64:                                                                   \
    hipLaunchKernelGGL((crc32c_stream_kernel<p | kUniProbeStamps, l, pre>),      \
                       dim3(num_groups), dim3(kGroupThreads), 0, stream, args);  \
    break;
    LVKV_STREAM_PROBE(20, kStreamNoLaneTab, 48, 0)   // fill, barrier, loads
    LVKV_STREAM_PROBE(21, kStreamNoLaneTab, 24, 0)
    LVKV_STREAM_PROBE(22, kStreamNoLaneTab, 48, 16)
    LVKV_STREAM_PROBE(23, kStreamNoLaneTab, 48, 48)  // all loads, fill, barrier
    LVKV_STREAM_PROBE(30, kStreamCounterSync, 24, 4)
    LVKV_STREAM_PROBE(31, kStreamCounterSync, 24, 8)
    LVKV_STREAM_PROBE(32, kStreamCounterSync, 32, 8)
    LVKV_STREAM_PROBE(33, kStreamCounterSync, 24, 16)
    LVKV_STREAM_PROBE(34, kStreamCounterSync, 48, 8)
    LVKV_STREAM_PROBE(35, kStreamCounterSync, 16, 4)
    LVKV_STREAM_PROBE(36, kStreamCounterSync, 48, 16)
    LVKV_STREAM_PROBE(37, kStreamCounterSync, 32, 0)
    LVKV_STREAM_PROBE(40, kStreamInterleave, 24, 16)
    LVKV_STREAM_PROBE(41, kStreamInterleave, 12, 12)
    LVKV_STREAM_PROBE(42, kStreamInterleave, 16, 16)
    LVKV_STREAM_PROBE(43, kStreamInterleave, 32, 16)
    LVKV_STREAM_PROBE(44, kStreamInterleave | kStreamCounterSync, 12, 4)
    LVKV_STREAM_PROBE(45, kStreamInterleave | kStreamCounterSync, 16, 8)
    LVKV_STREAM_PROBE(46, kStreamInterleave | kStreamCounterSync, 24, 8)
    LVKV_STREAM_PROBE(47, kStreamInterleave, 9, 9)
#undef LVKV_STREAM_PROBE
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace lvkv
