// Uniform-layout batch CRC32C for gfx950 with a 64 KiB LDS image, so two
// workgroups fit on one CU (the 160 KiB image of crc32c_uniform.hip allows
// one). Same arithmetic as the other kernels (end-aligned word grid, Horner
// over 256-byte rows with Z_256 byte tables, per-lane end shift Z_{256-4s},
// wave xor-reduce); what changes is how the row tables avoid bank conflicts.
//
// Row tables and lane tables: the compact image of crc32c_compact_common.h.
//
// Work map: the batch is split into `gridDim.x` contiguous runs of equal
// length (+1 for the first nblocks % G). Run element i goes to wave i % W,
// chain i / W, so a wave's valid chains are a prefix and every CU gets the
// same number of blocks. Chain 0's loads are issued before the LDS fill, the
// other chains' after the barrier (row-interleaved), then all chains are
// walked interleaved (crc32c_uniform.hip's measured schedule).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_device_common.h"
#include "crc32c_compact_common.h"
#include "crc32c_uniform_common.h"
#include "lvkv_crc32c.h"
#include "lvkv_kernel_args.h"

namespace lvkv {

namespace {

enum : int {
  kCmpBare = 1,     // probe: loads + xor only (no tables, no walk)
  kCmpGenLane = 2,  // lane tables generated from 4 columns per lane and
                    // nibble position (8 KiB of loads per workgroup, not 32)
};

// Row tables: 2048 16-byte slots q -> row b = q >> 3, table t = (q >> 1) & 3,
// copies 4h..4h+3 with h = q & 1 (address b*256 + 32t + 16h). Eight
// consecutive lanes cover one row's 128 B: conflict-free ds_write_b128.
template <int W>
__device__ __forceinline__ void fill_rows_c(uint32_t* lds, const UniformArgs& a, uint32_t tid) {
  constexpr int kThreads = 64 * W;
  constexpr int kIters = 2048 / kThreads;
  const uint32_t t = (tid >> 1) & 3u;  // the same for every iteration
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

// Lane tables from HBM (lane_tab[(k*16 + nib)*64 + s], kLaneTabDwords) into
// the upper halves of the bank rows.
template <int W>
struct LaneTabStage {
  static constexpr int kThreads = 64 * W;
  static constexpr int kIters = (kLaneTabDwords / 4) / kThreads;
  uint32_t v[kIters][4];

  __device__ __forceinline__ void load(const UniformArgs& a, uint32_t tid) {
#pragma unroll
    for (int it = 0; it < kIters; ++it) {
      const uint32_t* src = a.lane_tab + 4u * (tid + kThreads * it);
#pragma unroll
      for (int x = 0; x < 4; ++x) v[it][x] = src[x];
    }
  }
  __device__ __forceinline__ void store(uint32_t* lds, uint32_t tid) const {
#pragma unroll
    for (int it = 0; it < kIters; ++it) {
      const uint32_t d = 4u * (tid + kThreads * it);
      const uint32_t r = d >> 6, s = d & 63u;
      *reinterpret_cast<uint4*>(reinterpret_cast<char*>(lds) + (2u * r + (s >> 5)) * 256u +
                                128u + (s & 31u) * 4u) =
          make_uint4(v[it][0], v[it][1], v[it][2], v[it][3]);
    }
  }
};

// One wave with NV (1..NCH) valid chains; blocks blk[0..NV).
// `live` false: a wave past the batch (tiny batches only) runs chain 0 over an
// empty window (loads return zeros, no memory traffic) and stores nothing.
template <int P, int W, int NV, bool FULL>
__device__ __forceinline__ void compact_body(const UniformArgs& a, const UniGeo& g,
                                             uint32_t* lds, uint32_t tid, uint32_t lane,
                                             const uint32_t* blk, bool live) {
  LaneTabStage<W> lt;
  LaneTabGen<W> lg;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  __amdgpu_buffer_rsrc_t r[NV];
#pragma unroll
  for (int c = 0; c < NV; ++c) r[c] = block_rsrc<0>(a, g, blk[c], live);
  const int32_t vo = g.vb0 + 4 * static_cast<int32_t>(lane);
  int32_t vo1 = vo + kRowBytes;
  asm volatile("" : "+v"(vo1));
  uint32_t w[NV][kRowsPerChunk];
  auto load_rows = [&](int c_lo, int c_hi) {
#pragma unroll
    for (int j = 0; j < kRowsPerChunk; ++j)
#pragma unroll
      for (int c = 0; c < NV; ++c)
        if (c >= c_lo && c < c_hi && (FULL || static_cast<uint32_t>(j) < g.rows))
          w[c][j] = load_word(r[c], vo, vo1, j);
  };

  if (P & kCmpBare) {
    load_rows(0, NV);
    uint32_t x = 0;
#pragma unroll
    for (int j = 0; j < kRowsPerChunk; ++j)
#pragma unroll
      for (int c = 0; c < NV; ++c)
        if (FULL || static_cast<uint32_t>(j) < g.rows) x ^= w[c][j];
    asm volatile("s_barrier" ::: "memory");
    lds[tid] = x;
    if (lane == 0 && live)
#pragma unroll
      for (int c = 0; c < NV; ++c) a.out[blk[c]] = x;
    return;
  }

  // 1. Lane tables, chain 0, the LDS image, one barrier, the other chains.
  if (P & kCmpGenLane)
    lg.load(a.lane_cols, wave, lane);
  else
    lt.load(a, tid);
  __builtin_amdgcn_sched_barrier(0);
  load_rows(0, 1);
  __builtin_amdgcn_sched_barrier(0);
  fill_rows_c<W>(lds, a, tid);
  if (P & kCmpGenLane)
    lg.store(lds, wave, lane);
  else
    lt.store(lds, tid);
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  load_rows(1, NV);

  // 2. Rows, chains interleaved; row-0 fix-ups first.
  const LaneKeys keys = lane_keys(lane);
  uint32_t st[NV];
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

  // 3. End shift, reduction, store.
  const uint32_t lane_base = (lane >> 5) * 256u + 128u + (lane & 31u) * 4u;
  uint32_t crc[NV];
#pragma unroll
  for (int c = 0; c < NV; ++c)
    crc[c] = wave_xor_dpp(lane_end_shift_c(lds, st[c], lane_base)) ^ 0xffffffffu;
  if (lane == 0 && live) {
#pragma unroll
    for (int c = 0; c < NV; ++c) a.out[blk[c]] = a.mask ? crc_mask(crc[c]) : crc[c];
  }
}

}  // namespace

template <int P, int W, int NCH, int OCC>
__global__ void __launch_bounds__(64 * W, OCC) crc32c_compact_kernel(UniformArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kCompactLdsBytes / 4];
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = lane_id();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const UniGeo g = uni_geo(a);
  // Equal contiguous runs per workgroup.
  const uint32_t G = gridDim.x;
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
  if (NCH >= 3 && nv >= 3) {
    if (full) compact_body<P, W, (NCH >= 3 ? 3 : 1), true>(a, g, lds, tid, lane, blk, true);
    else compact_body<P, W, (NCH >= 3 ? 3 : 1), false>(a, g, lds, tid, lane, blk, true);
  } else if (NCH >= 2 && nv >= 2) {
    if (full) compact_body<P, W, (NCH >= 2 ? 2 : 1), true>(a, g, lds, tid, lane, blk, true);
    else compact_body<P, W, (NCH >= 2 ? 2 : 1), false>(a, g, lds, tid, lane, blk, true);
  } else {
    if (full) compact_body<P, W, 1, true>(a, g, lds, tid, lane, blk, nv != 0);
    else compact_body<P, W, 1, false>(a, g, lds, tid, lane, blk, nv != 0);
  }
}

// ---------------------------------------------------------------------------
// Long blocks of the general batch (covered length > kLongBytes), one
// workgroup per block instead of one wave: the bytes up to the last 4-byte
// boundary are cut at absolute 4-byte-aligned points into kLongSeg segments;
// wave w checksums segments w, w + 16, ... (segment 0 from init ^ ~0, the
// others from register 0), shifts each register to that boundary with Z_n =
// the product of the Z_{2^j} byte tables (zpow, HBM), and xors it into its
// accumulator. Wave 0 combines the 16 accumulators, feeds the 0-3 tail bytes
// through the byte table (Z_1) and stores in the batch's mode (compute, SST
// verify, SST fill). The main batch kernel skips exactly these blocks
// (KernelArgs::long_split). Bytes read per block: its covered length once.

namespace {

constexpr int kLongWaves = 16;

__device__ __forceinline__ uint32_t ld_le32_g(const uint8_t* t) {
  return static_cast<uint32_t>(t[0]) | (static_cast<uint32_t>(t[1]) << 8) |
         (static_cast<uint32_t>(t[2]) << 16) | (static_cast<uint32_t>(t[3]) << 24);
}

}  // namespace

__global__ void __launch_bounds__(1024, 1)
    crc32c_long_kernel(KernelArgs a, const uint32_t* zpow, const uint32_t* lane_cols) {
  constexpr int W = kLongWaves;
  // LDS: the compact image, one accumulator per wave, the slice's long-block
  // list and its length.
  constexpr uint32_t kAcc = kCompactLdsBytes / 4, kList = kAcc + W, kCount = kList + 1024;
  __shared__ __attribute__((aligned(16))) uint32_t lds[kCount + 1];
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = lane_id();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t n = a.count != nullptr ? min(a.nblocks, sload_u32(a.count, 0)) : a.nblocks;
  const uint64_t base = reinterpret_cast<uint64_t>(a.base);
  const bool sst = a.mode == kModeSstVerify || a.mode == kModeSstFill;
  const uint32_t extra = sst ? 1u : 0u;
  bool built = false;
  const LaneKeys keys = lane_keys(lane);
  const uint32_t lane_base = (lane >> 5) * 256u + 128u + (lane & 31u) * 4u;
  // Workgroup g scans blocks [g*per, (g+1)*per), 1024 lengths at a time
  // (coalesced), and walks the long ones it finds.
  const uint32_t per = (n + gridDim.x - 1) / gridDim.x;
  const uint32_t first = min(n, blockIdx.x * per), last = min(n, first + per);
  for (uint32_t slice = first; slice < last; slice += 1024) {
    if (tid == 0) lds[kCount] = 0;
    __syncthreads();
    const uint32_t i = slice + tid;
    if (i < last && a.lengths[i] + extra > kLongBytes) lds[kList + atomicAdd(&lds[kCount], 1u)] = i;
    __syncthreads();
    const uint32_t cnt = __builtin_amdgcn_readfirstlane(lds[kCount]);
    for (uint32_t li = 0; li < cnt; ++li) {
      const uint32_t b = __builtin_amdgcn_readfirstlane(lds[kList + li]);
      const uint64_t off = sload_u64(a.offsets, b);
      const uint64_t len = static_cast<uint64_t>(sload_u32(a.lengths, b)) + extra;
      const uint32_t init = sst ? 0u : (a.inits != nullptr ? sload_u32(a.inits, b) : a.init);
      if (!built) {  // the compact LDS image, once per workgroup
        build_compact_image<kLongWaves>(lds, zpow, lane_cols, tid, wave, lane);
        built = true;
      }
      const uint64_t start = base + off, end = start + len;
      const uint32_t crc =
          workgroup_crc<kLongWaves>(lds, lds + kAcc, start, end, init, keys, tid, wave, lane, lane_base, zpow);
      if (tid == 0) {
        if (a.mode == kModeSstFill) {
          uint8_t* dst = reinterpret_cast<uint8_t*>(end);
          const uint32_t mcrc = crc_mask(crc);
          for (int k = 0; k < 4; ++k) dst[k] = static_cast<uint8_t>(mcrc >> (8 * k));
          if (a.out_crc != nullptr) a.out_crc[b] = crc;
        } else if (a.mode == kModeSstVerify) {
          a.out_crc[b] = crc;
          if (a.out_status != nullptr)
            a.out_status[b] = crc != crc_unmask(ld_le32_g(reinterpret_cast<const uint8_t*>(end)));
        } else {
          a.out_crc[b] = a.mask ? crc_mask(crc) : crc;
        }
      }
    }
    __syncthreads();
  }
}

hipError_t launch_crc32c_long(const KernelArgs& args, const uint32_t* zpow,
                              const uint32_t* lane_cols, int num_groups, hipStream_t stream) {
  hipLaunchKernelGGL(crc32c_long_kernel, dim3(num_groups), dim3(1024), 0, stream, args, zpow,
                     lane_cols);
  return hipGetLastError();
}

// cfg: bits 0-1 = shape (0: 16 waves x 3 chains, 1 WG/CU; 1: 8 waves x 3
// chains, 2 WGs/CU; 2: 16 waves x 2 chains, 2 WGs/CU); bit 2 = bare probe;
// bit 3 = generated lane tables.
int compact_capacity(int cfg) {
  switch (cfg & 3) {
    case 0: return 16 * 3;
    case 1: return 8 * 3;
    case 2: return 16 * 2;
  }
  return 0;
}
int compact_occupancy(int cfg) { return (cfg & 3) == 0 ? 1 : 2; }

hipError_t launch_crc32c_compact(const UniformArgs& args, int cfg, int num_groups,
                                 hipStream_t stream) {
  switch (cfg & 15) {
#define LVKV_CMP_CASE(c, p, w, nch, occ)                                        \
  case c:                                                                       \
    hipLaunchKernelGGL((crc32c_compact_kernel<p, w, nch, occ>), dim3(num_groups), \
                       dim3(64 * w), 0, stream, args);                          \
    break;
    LVKV_CMP_CASE(9, kCmpGenLane, 8, 3, 2)  // production (kCompactProductionCfg)
#ifdef LVKV_PROBE_BUILD
    LVKV_CMP_CASE(0, 0, 16, 3, 1)
    LVKV_CMP_CASE(1, 0, 8, 3, 2)
    LVKV_CMP_CASE(2, 0, 16, 2, 2)
    LVKV_CMP_CASE(4, kCmpBare, 16, 3, 1)
    LVKV_CMP_CASE(5, kCmpBare, 8, 3, 2)
    LVKV_CMP_CASE(6, kCmpBare, 16, 2, 2)
    LVKV_CMP_CASE(8, kCmpGenLane, 16, 3, 1)
#endif
#undef LVKV_CMP_CASE
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace lvkv
