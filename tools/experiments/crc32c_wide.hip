// Wide-load uniform-batch CRC32C for gfx950: the production kernel for
// nblocks blocks of 16 rows (the leveldb 4 KiB block size) at base + i*stride,
// every block END 4-byte aligned and its word grid 16-byte aligned
// (s0l % 4 == 0, e.g. 4093..4096 bytes), at most 3 blocks per wave of the
// grid (the 10k x 4 KiB headline and the 1k x 4 KiB config).
//
// Same arithmetic as the other kernels (end-aligned word grid, Horner over
// 256-byte rows with the Z_256 LDS tables, per-lane end shift, wave reduce).
// What differs is how the bytes come in, chosen from measurements of the bare
// memory side (tools/order_probe.hip, 10k x 4 KiB cold):
//
//  * 16 bytes per lane per load (buffer_load_dwordx4, 1 KiB per wave
//    instruction): 7.5 us per launch against 8.0 us with one dword per lane.
//  * Each wave owns a contiguous run of 2-3 blocks of its CU's contiguous
//    range and reads it in address order; row-interleaving the blocks costs
//    0.5 us (DRAM locality).
//  * A 1 KiB chunk lands as lane l = bytes [16l, 16l+16); one ds_write_b128
//    into the wave's LDS slot and four ds_read_b32 turn it into four 256-byte
//    rows with lane s = word s, the layout the Horner walk needs.
//  * The 1 KiB per wave comes from halving the lane tables: lane s applies
//    Z_{4(32-(s&31))} (32 slots, one per bank, shared by lanes s and s+32 of
//    the other half-wave), and the lower half's extra Z_128 is applied once
//    to its reduced value (slot 0's op is Z_128).
//  * Software pipeline: `L` chunks in flight per wave; a block is finished as
//    soon as its last row is consumed.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_device_common.h"
#include "crc32c_uniform_common.h"
#include "lvkv_kernel_args.h"

namespace lvkv {
namespace {

constexpr int kChunksPerBlock = kRowsPerChunk / 4;  // 1 KiB chunks per 16-row block

// Row tables from the 32 columns of Z_256 by linearity, by F filler waves.
// Filler f writes table t = f / (F/4), entries [e0, e0 + 1024/F) with
// e0 = (f % (F/4)) * (1024/F); lane l covers entries e0 + (l >> 3) + 8k and
// copies 4 * (l & 7) .. +3 (one 16-byte store per entry). T_t is linear and
// the three index fields have disjoint bits, so
// T_t[e0 + (l >> 3) + 8k] = T_t[e0] ^ T_t[l >> 3] ^ T_t[8k]: the first and
// last terms are wave-uniform (scalar unit), the middle one three selects.
template <int F>
__device__ __forceinline__ void wide_fill_rows(uint32_t* lds, const UniformArgs& a,
                                               uint32_t f, uint32_t lane) {
  static_assert(F == 4 || F == 8 || F == 16, "filler count");
  constexpr uint32_t kPerTable = F / 4;           // fillers per table
  constexpr uint32_t kEntries = 256 / kPerTable;  // entries per filler
  constexpr int kK = kEntries / 8;                // 16-byte stores per lane
  const uint32_t t = f / kPerTable;
  const uint32_t e0 = (f % kPerTable) * kEntries;
  const uint32_t* col = a.zcol + 8u * t;
  auto tab = [&](uint32_t i) {  // uniform i: scalar selects
    uint32_t r = 0;
#pragma unroll
    for (int b = 0; b < 8; ++b) r ^= ((i >> b) & 1u) ? col[b] : 0u;
    return r;
  };
  const uint32_t lo = lane >> 3;
  const uint32_t e_lane = tab(e0) ^ ((0u - (lo & 1u)) & col[0]) ^
                          ((0u - ((lo >> 1) & 1u)) & col[1]) ^ ((0u - ((lo >> 2) & 1u)) & col[2]);
  char* dst = reinterpret_cast<char*>(lds) + (t >> 1) * kLdsRowRegionBytes +
              (t & 1u) * 128u + (e0 + lo) * 256u + (lane & 7u) * 16u;
#pragma unroll
  for (int k = 0; k < kK; ++k) {
    const uint32_t e = e_lane ^ tab(8u * k);
    *reinterpret_cast<uint4*>(dst + k * 8 * 256) = make_uint4(e, e, e, e);
  }
}

// Z_{4(32-v)} for this lane's slot v = lane & 31: eight nibble lookups.
__device__ __forceinline__ uint32_t end_shift32(const uint32_t* lds, uint32_t s,
                                                uint32_t lane_base) {
  uint32_t r = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint32_t nib = (s >> (4 * k)) & 15u;
    r ^= lds_ld(lds, lane_base + nib * 128u + 2048u * k);
  }
  return r;
}

// raw CRC of a finished block from the lanes' Horner states:
// XOR_s Z_{256-4s}(S_s) = Z_128(XOR_{s<32} Y_s) ^ XOR_{s>=32} Y_s with
// Y_s = Z_{4(32-(s&31))}(S_s).
__device__ __forceinline__ uint32_t finish32(const uint32_t* lds, uint32_t st,
                                             uint32_t lane_base) {
  uint32_t v = end_shift32(lds, st, lane_base);
  v ^= static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(v), 0xB1, 0xF, 0xF, false));
  v ^= static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(v), 0x4E, 0xF, 0xF, false));
  v ^= static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(v), 0x141, 0xF, 0xF, false));
  v ^= static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(v), 0x140, 0xF, 0xF, false));
  const uint32_t lo = __builtin_amdgcn_readlane(v, 0) ^ __builtin_amdgcn_readlane(v, 16);
  const uint32_t hi = __builtin_amdgcn_readlane(v, 32) ^ __builtin_amdgcn_readlane(v, 48);
  // Z_128(lo): slot 0's op, same address in every lane (broadcast reads)
  uint32_t z = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint32_t nib = (lo >> (4 * k)) & 15u;
    z ^= lds_ld(lds, kLdsLane32Base + nib * 128u + 2048u * k);
  }
  return __builtin_amdgcn_readfirstlane(z) ^ hi;
}

__device__ __forceinline__ uint32_t wide_fix_row0(uint32_t w, const UniGeo& g, uint32_t lane) {
  const uint32_t sh = 8u * g.delta;
  w = (lane < g.s0l) ? 0u : w;
  w = (lane == g.s0l) ? ((w & (0xffffffffu << sh)) ^ (g.s0 << sh)) : w;
  return (lane == g.s0l + 1u) ? (w ^ g.spill) : w;
}

__device__ __forceinline__ uint32_t wide_fix_row1(uint32_t w, const UniGeo& g, uint32_t lane) {
  return (g.s0l == 63u && lane == 0) ? (w ^ g.spill) : w;
}

__device__ __forceinline__ uint4 load_chunk(__amdgpu_buffer_rsrc_t r, int32_t vo, int j) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, vo + 1024 * j, 0, kUniCachePolicy);
  return make_uint4(v[0], v[1], v[2], v[3]);
}

// One wave's run of NB consecutive blocks (first = b0). valid = false only for
// a wave with no block (empty window, no store; it still fills its share).
template <int P, int NB, int L, int PRE, int F>
__device__ __forceinline__ void wide_body(const UniformArgs& a, const UniGeo& g,
                                          uint32_t* lds, uint32_t tid, uint32_t lane,
                                          uint32_t wave, uint32_t gw, uint32_t b0,
                                          bool valid) {
  constexpr int R = kChunksPerBlock * NB;  // chunks in the run

  // Waves 0..F-1 fill the LDS tables before they load anything; waves F..15
  // issue their first PRE chunks first, so the memory pipe fills while the
  // tables are written. The lane tables (1024 x 16 B) are split over the
  // fillers' lanes.
  // F = 0: every wave issues PRE chunks, then fills 1/16 of the tables.
  constexpr int kF = F == 0 ? kWavesPerGroup : F;
  const bool filler = wave < static_cast<uint32_t>(kF);
  constexpr int kLtPer = kGroupThreads / 64 / kF;  // 16-byte slots per filler lane
  uint4 lt[kLtPer];
  if (filler) {
#pragma unroll
    for (int k = 0; k < kLtPer; ++k)
      lt[k] = reinterpret_cast<const uint4*>(a.lane_tab32)[(wave * kLtPer + k) * 64 + lane];
  }

  const __amdgpu_buffer_rsrc_t r0 = block_rsrc<P>(a, g, b0, valid);
  const __amdgpu_buffer_rsrc_t r1 = block_rsrc<P>(a, g, b0 + 1, NB > 1);
  const __amdgpu_buffer_rsrc_t r2 = block_rsrc<P>(a, g, b0 + 2, NB > 2);
  // grid word 4*lane of each chunk; vb0 = -4*s0l is a multiple of 16 here, so
  // a lane's 16 bytes are either all front padding (out of the window: zeros)
  // or all inside the block
  const int32_t vo = g.vb0 + 16 * static_cast<int32_t>(lane);

  uint4 w[R];
  auto issue = [&](int i) {
    if (i < R) {
      const int c = i / kChunksPerBlock;
      w[i] = load_chunk(c == 0 ? r0 : (c == 1 ? r1 : r2), vo, i % kChunksPerBlock);
    }
  };
  __builtin_amdgcn_sched_barrier(0);
  if (F == 0) {
#pragma unroll
    for (int i = 0; i < PRE && i < L; ++i) issue(i);
    __builtin_amdgcn_sched_barrier(0);
  }
  if (filler) {
    stamp_uni<P>(a, gw, 3);
    wide_fill_rows<kF>(lds, a, wave, lane);
#pragma unroll
    for (int k = 0; k < kLtPer; ++k)
      reinterpret_cast<uint4*>(lds + kLdsLane32Base / 4)[(wave * kLtPer + k) * 64 + lane] = lt[k];
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    stamp_uni<P>(a, gw, 1);
#pragma unroll
    for (int i = (F == 0 ? PRE : 0); i < L; ++i) issue(i);
  } else {
#pragma unroll
    for (int i = 0; i < PRE && i < L; ++i) issue(i);
    __builtin_amdgcn_sched_barrier(0);
    stamp_uni<P>(a, gw, 3);
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    stamp_uni<P>(a, gw, 1);
#pragma unroll
    for (int i = PRE; i < L; ++i) issue(i);
  }
  __builtin_amdgcn_sched_barrier(0);  // keep the window's loads here

  const uint32_t k0 = (lane & 31u) * 4u;
  const uint32_t k1 = k0 | 0x10000u;
  const uint32_t lane_base = kLdsLane32Base + (lane & 31u) * 4u;
  uint4* slot_w = reinterpret_cast<uint4*>(lds + (kLdsStageBase + wave * 1024u) / 4) + lane;
  const uint32_t* slot_r = lds + (kLdsStageBase + wave * 1024u) / 4 + lane;
  uint32_t st = 0;
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int c = i / kChunksPerBlock, j = i % kChunksPerBlock;
    issue(i + L);
    __builtin_amdgcn_sched_barrier(0);  // the refill is not sunk below the walk
    *slot_w = w[i];
    uint32_t x[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) x[q] = slot_r[64 * q];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = 4 * j + q;
      uint32_t y = x[q];
      if (row == 0) y = wide_fix_row0(y, g, lane);
      if (row == 1) y = wide_fix_row1(y, g, lane);
      st = (row == 0) ? y : row_step(lds, st, y, k0, k1);
    }
    if (j == kChunksPerBlock - 1) {
      const uint32_t crc = finish32(lds, st, lane_base) ^ 0xffffffffu;
      if (lane == 0 && valid) a.out[b0 + c] = a.mask ? crc_mask(crc) : crc;
    }
  }
  stamp_uni<P>(a, gw, 2);
}

}  // namespace

template <int P, int L, int PRE, int F>
__global__ void __launch_bounds__(kGroupThreads, 1)
    crc32c_wide_kernel(UniformArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsBytes / 4];
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = lane_id();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t gw = blockIdx.x * kWavesPerGroup + wave;
  stamp_uni<P>(a, gw, 0);
  const UniGeo g = uni_geo(a);
  // Workgroup g owns a contiguous range of the batch (equal shares, the
  // remainder to the first groups); its waves own consecutive runs of it.
  const uint32_t per = a.nblocks / gridDim.x, extra = a.nblocks % gridDim.x;
  const uint32_t n_g = per + (blockIdx.x < extra ? 1u : 0u);
  const uint32_t start = blockIdx.x * per + min(blockIdx.x, extra);
  const uint32_t q = n_g / kWavesPerGroup, rem = n_g % kWavesPerGroup;
  const uint32_t cnt = q + (wave < rem ? 1u : 0u);
  const uint32_t b0 = start + wave * q + min(wave, rem);
  if (cnt >= 3)
    wide_body<P, 3, L, PRE, F>(a, g, lds, tid, lane, wave, gw, b0, true);
  else if (cnt == 2)
    wide_body<P, 2, L, PRE, F>(a, g, lds, tid, lane, wave, gw, b0, true);
  else
    wide_body<P, 1, L, PRE, F>(a, g, lds, tid, lane, wave, gw, b0, cnt == 1);
  stamp_uni<P>(a, gw, 7);
}

// ---------------------------------------------------------------------------
// Chunk-balanced variant for contiguous 4096-byte blocks (length == stride ==
// 4096): every wave of a workgroup streams the same number of 1 KiB chunks
// (+-1) of its CU's contiguous range, so no wave is left streaming alone at
// the end of the launch (with whole blocks, 7 of 16 waves own 3 blocks and the
// others 2). A block cut between waves w and w+1 is joined at the end: wave w
// finishes its prefix as if the block ended there and shifts the result by the
// missing m KiB (Z_{1024 m}, 32 columns in the kernel arguments, scalar unit);
// wave w+1 xors it into its suffix after one workgroup barrier.

namespace {

__device__ __forceinline__ uint32_t shift_kib(const UniformArgs& a, uint32_t x, uint32_t m) {
  uint32_t r = 0;
#pragma unroll
  for (int b = 0; b < 32; ++b) r ^= ((x >> b) & 1u) ? a.zchunk[m - 1][b] : 0u;
  return r;
}

}  // namespace

template <int P, int L>
__global__ void __launch_bounds__(kGroupThreads, 1)
    crc32c_wide_bal_kernel(UniformArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsBytes / 4];
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = lane_id();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t gw = blockIdx.x * kWavesPerGroup + wave;
  stamp_uni<P>(a, gw, 0);
  const uint32_t per = a.nblocks / gridDim.x, extra = a.nblocks % gridDim.x;
  const uint32_t n_g = per + (blockIdx.x < extra ? 1u : 0u);
  const uint32_t start = blockIdx.x * per + min(blockIdx.x, extra);
  uint32_t c0, nch;  // this wave's chunks, relative to the group's first chunk
  if (n_g <= static_cast<uint32_t>(kWavesPerGroup)) {
    c0 = 4u * wave;
    nch = wave < n_g ? 4u : 0u;
  } else {
    const uint32_t tot = 4u * n_g, q = tot / kWavesPerGroup, rem = tot % kWavesPerGroup;
    nch = q + (wave < rem ? 1u : 0u);
    c0 = wave * q + min(wave, rem);
  }
  c0 = __builtin_amdgcn_readfirstlane(c0);
  nch = __builtin_amdgcn_readfirstlane(nch);
  const uint64_t run = reinterpret_cast<uint64_t>(a.base) +
                       (static_cast<uint64_t>(start) * 4u + c0) * 1024u;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<void*>(run), 0, static_cast<int>(nch * 1024u), kBufferDword3);
  const int32_t vo = 16 * static_cast<int32_t>(lane);

  const uint4 lt = reinterpret_cast<const uint4*>(a.lane_tab32)[tid];
  uint4 ring[L];
#pragma unroll
  for (int u = 0; u < L; ++u) ring[u] = load_chunk(r, vo, u);
  __builtin_amdgcn_sched_barrier(0);
  stamp_uni<P>(a, gw, 3);
  wide_fill_rows<kWavesPerGroup>(lds, a, wave, lane);
  reinterpret_cast<uint4*>(lds + kLdsLane32Base / 4)[tid] = lt;
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  stamp_uni<P>(a, gw, 1);

  const uint32_t k0 = (lane & 31u) * 4u;
  const uint32_t k1 = k0 | 0x10000u;
  const uint32_t lane_base = kLdsLane32Base + (lane & 31u) * 4u;
  uint4* slot_w = reinterpret_cast<uint4*>(lds + (kLdsStageBase + wave * 1024u) / 4) + lane;
  const uint32_t* slot_r = lds + (kLdsStageBase + wave * 1024u) / 4 + lane;
  const uint32_t s0 = a.init ^ 0xffffffffu;
  const bool cut_head = (c0 & 3u) != 0u && nch != 0u;  // run starts mid-block
  uint32_t head_raw = 0;                               // raw CRC of that suffix
  uint32_t st = 0;
  for (uint32_t i = 0; i < nch; i += L) {
#pragma unroll
    for (int u = 0; u < L; ++u) {
      const uint32_t idx = i + u;
      if (idx < nch) {
        const uint4 x4 = ring[u];
        ring[u] = load_chunk(r, vo, static_cast<int>(idx) + L);
        __builtin_amdgcn_sched_barrier(0);
        const uint32_t ch = c0 + idx, j = ch & 3u;
        *slot_w = x4;
        uint32_t x[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) x[q] = slot_r[64 * q];
        if (j == 0u) x[0] ^= (lane == 0) ? s0 : 0u;  // init injection, row 0
        const bool fresh = j == 0u || idx == 0u;
        st = fresh ? x[0] : row_step(lds, st, x[0], k0, k1);
#pragma unroll
        for (int q = 1; q < 4; ++q) st = row_step(lds, st, x[q], k0, k1);
        if (j == 3u) {
          const uint32_t raw = finish32(lds, st, lane_base);
          if (cut_head && idx < 4u) {
            head_raw = raw;
          } else {
            const uint32_t crc = raw ^ 0xffffffffu;
            if (lane == 0) a.out[start + (ch >> 2)] = a.mask ? crc_mask(crc) : crc;
          }
        }
      }
    }
  }
  stamp_uni<P>(a, gw, 2);
  // A block cut at the end of this run: hand its shifted prefix to wave + 1.
  const uint32_t tail = (c0 + nch) & 3u;
  if (nch != 0u && tail != 0u) {
    const uint32_t part = shift_kib(a, finish32(lds, st, lane_base), 4u - tail);
    if (lane == 0) lds[(kLdsStageBase + wave * 1024u) / 4] = part;
  }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  if (cut_head) {
    const uint32_t prev = lds[(kLdsStageBase + (wave - 1u) * 1024u) / 4];
    const uint32_t crc = __builtin_amdgcn_readfirstlane(prev) ^ head_raw ^ 0xffffffffu;
    if (lane == 0) a.out[start + (c0 >> 2)] = a.mask ? crc_mask(crc) : crc;
  }
  stamp_uni<P>(a, gw, 7);
}

hipError_t launch_crc32c_wide_bal(const UniformArgs& args, int cfg, int num_groups,
                                  hipStream_t stream) {
  switch (cfg) {
#define LVKV_BAL_CASE(c, l)                                                      \
  case c:                                                                        \
    hipLaunchKernelGGL((crc32c_wide_bal_kernel<0, l>), dim3(num_groups),         \
                       dim3(kGroupThreads), 0, stream, args);                    \
    break;                                                                       \
  case c + 64:                                                                   \
    hipLaunchKernelGGL((crc32c_wide_bal_kernel<kUniProbeStamps, l>),             \
                       dim3(num_groups), dim3(kGroupThreads), 0, stream, args);  \
    break;
    LVKV_BAL_CASE(0, 3)
    LVKV_BAL_CASE(1, 2)
    LVKV_BAL_CASE(2, 4)
#undef LVKV_BAL_CASE
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Transposed-lane variant: the same wide loads and per-wave block runs as
// crc32c_wide_kernel, but the 1 KiB chunk is turned into four rows in
// registers instead of through LDS. Lane L's 16 bytes are the words 4L..4L+3,
// i.e. row L >> 4 at positions 4(L & 15) + i. Swapping lane bit 5 with
// register bit 1 (v_permlane32_swap on register pairs (0,2), (1,3)) and lane
// bit 4 with register bit 0 (v_permlane16_swap on (0,1), (2,3)) leaves row q in
// register q with lane L at position p(L) = 4(L & 15) + (L >> 4) in every row.
// The Horner walk does not care which lane owns which position; the end shift
// does: position p needs Z_{4(64 - p)} (a word's bytes are shifted through the
// register too), lane L applies op v = L & 31 = Z_{4(62 - p(v))}, exact for
// lane v + 32 (position p(v) + 2) and short by Z_8 for lane v, applied once to
// the reduced lower half (uniform Z_8 nibble table). Four VALU swaps per 1 KiB
// replace the LDS round trip (ds_write_b128 + 4 ds_read_b32) of the staging
// variant, and there is no staging area.

namespace {

// Probe builds: 16 timestamps per wave (0 entry, 1 after the barrier,
// 2 + i after chunk i (i < 12), 15 exit).
template <int P>
__device__ __forceinline__ void stamp16(const UniformArgs& a, uint32_t gw, int slot) {
  if (P & kUniProbeStamps) {
    const uint64_t t = __builtin_amdgcn_s_memrealtime();
    if (lane_id() == 0) a.stamps[gw * 16u + slot] = t;
  }
}

__device__ __forceinline__ void xpose_rows(const uint4& v, uint32_t (&x)[4]) {
  const auto a = __builtin_amdgcn_permlane32_swap(v.x, v.z, false, false);
  const auto b = __builtin_amdgcn_permlane32_swap(v.y, v.w, false, false);
  const auto c = __builtin_amdgcn_permlane16_swap(a[0], b[0], false, false);
  const auto d = __builtin_amdgcn_permlane16_swap(a[1], b[1], false, false);
  x[0] = c[0];
  x[1] = c[1];
  x[2] = d[0];
  x[3] = d[1];
}

__device__ __forceinline__ uint32_t finish_x(const uint32_t* lds, uint32_t st,
                                             uint32_t lane_base) {
  uint32_t v = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint32_t nib = (st >> (4 * k)) & 15u;
    v ^= lds_ld(lds, lane_base + nib * 128u + 2048u * k);
  }
  v ^= static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(v), 0xB1, 0xF, 0xF, false));
  v ^= static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(v), 0x4E, 0xF, 0xF, false));
  v ^= static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(v), 0x141, 0xF, 0xF, false));
  v ^= static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(v), 0x140, 0xF, 0xF, false));
  const uint32_t lo = __builtin_amdgcn_readlane(v, 0) ^ __builtin_amdgcn_readlane(v, 16);
  const uint32_t hi = __builtin_amdgcn_readlane(v, 32) ^ __builtin_amdgcn_readlane(v, 48);
  uint32_t z = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint32_t nib = (lo >> (4 * k)) & 15u;
    z ^= lds_ld(lds, kLdsZ8Base + (k * 16u + nib) * 4u);
  }
  return __builtin_amdgcn_readfirstlane(z) ^ hi;
}

template <int P, int NB, int L, int PRE>
__device__ __forceinline__ void xpose_body(const UniformArgs& a, const UniGeo& g,
                                           uint32_t* lds, uint32_t tid, uint32_t lane,
                                           uint32_t wave, uint32_t gw, uint32_t b0,
                                           bool valid) {
  constexpr int R = kChunksPerBlock * NB;
  const uint4* lsrc = reinterpret_cast<const uint4*>(a.lane_tab_x);
  const uint4 lt0 = lsrc[tid];
  uint4 lt1 = {};
  if (tid < 32) lt1 = lsrc[kGroupThreads + tid];  // the Z_8 table

  const __amdgpu_buffer_rsrc_t r0 = block_rsrc<P>(a, g, b0, valid);
  const __amdgpu_buffer_rsrc_t r1 = block_rsrc<P>(a, g, b0 + 1, NB > 1);
  const __amdgpu_buffer_rsrc_t r2 = block_rsrc<P>(a, g, b0 + 2, NB > 2);
  const int32_t vo = g.vb0 + 16 * static_cast<int32_t>(lane);

  uint4 w[R];
  auto issue = [&](int i) {
    if (i < R) {
      const int c = i / kChunksPerBlock;
      w[i] = load_chunk(c == 0 ? r0 : (c == 1 ? r1 : r2), vo, i % kChunksPerBlock);
    }
  };
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < PRE && i < L; ++i) issue(i);
  __builtin_amdgcn_sched_barrier(0);
  wide_fill_rows<kWavesPerGroup>(lds, a, wave, lane);
  uint4* ldst = reinterpret_cast<uint4*>(lds + kLdsLaneXBase / 4);
  ldst[tid] = lt0;
  if (tid < 32) ldst[kGroupThreads + tid] = lt1;
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  stamp16<P>(a, gw, 1);
#pragma unroll
  for (int i = PRE; i < L; ++i) issue(i);
  __builtin_amdgcn_sched_barrier(0);

  const uint32_t k0 = (lane & 31u) * 4u;
  const uint32_t k1 = k0 | 0x10000u;
  const uint32_t lane_base = kLdsLaneXBase + (lane & 31u) * 4u;
  const uint32_t pos = 4u * (lane & 15u) + (lane >> 4);
  uint32_t st = 0;
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int c = i / kChunksPerBlock, j = i % kChunksPerBlock;
    issue(i + L);
    __builtin_amdgcn_sched_barrier(0);
    uint32_t x[4];
    xpose_rows(w[i], x);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = 4 * j + q;
      uint32_t y = x[q];
      if (row == 0) y = wide_fix_row0(y, g, pos);
      if (row == 1) y = wide_fix_row1(y, g, pos);
      st = (row == 0) ? y : row_step(lds, st, y, k0, k1);
    }
    if (j == kChunksPerBlock - 1) {
      const uint32_t crc = finish_x(lds, st, lane_base) ^ 0xffffffffu;
      if (lane == 0 && valid) a.out[b0 + c] = a.mask ? crc_mask(crc) : crc;
    }
    if (i < 12) stamp16<P>(a, gw, 2 + i);
  }
}

}  // namespace

template <int P, int L, int PRE>
__global__ void __launch_bounds__(kGroupThreads, 1)
    crc32c_xpose_kernel(UniformArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsXposeBytes / 4];
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = lane_id();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t gw = blockIdx.x * kWavesPerGroup + wave;
  stamp16<P>(a, gw, 0);
  const UniGeo g = uni_geo(a);
  const uint32_t per = a.nblocks / gridDim.x, extra = a.nblocks % gridDim.x;
  const uint32_t n_g = per + (blockIdx.x < extra ? 1u : 0u);
  const uint32_t start = blockIdx.x * per + min(blockIdx.x, extra);
  const uint32_t q = n_g / kWavesPerGroup, rem = n_g % kWavesPerGroup;
  const uint32_t cnt = q + (wave < rem ? 1u : 0u);
  const uint32_t b0 = start + wave * q + min(wave, rem);
  if (cnt >= 3)
    xpose_body<P, 3, L, PRE>(a, g, lds, tid, lane, wave, gw, b0, true);
  else if (cnt == 2)
    xpose_body<P, 2, L, PRE>(a, g, lds, tid, lane, wave, gw, b0, true);
  else
    xpose_body<P, 1, L, PRE>(a, g, lds, tid, lane, wave, gw, b0, cnt == 1);
  stamp16<P>(a, gw, 15);
}

hipError_t launch_crc32c_xpose(const UniformArgs& args, int cfg, int num_groups,
                               hipStream_t stream) {
  switch (cfg) {
#define LVKV_XP_CASE(c, l, pre)                                                  \
  case c:                                                                        \
    hipLaunchKernelGGL((crc32c_xpose_kernel<0, l, pre>), dim3(num_groups),       \
                       dim3(kGroupThreads), 0, stream, args);                    \
    break;                                                                       \
  case c + 64:                                                                   \
    hipLaunchKernelGGL((crc32c_xpose_kernel<kUniProbeStamps, l, pre>),           \
                       dim3(num_groups), dim3(kGroupThreads), 0, stream, args);  \
    break;
    LVKV_XP_CASE(0, 3, 3)
    LVKV_XP_CASE(1, 2, 2)
    LVKV_XP_CASE(2, 4, 4)
    LVKV_XP_CASE(3, 4, 2)
    LVKV_XP_CASE(4, 6, 4)
    LVKV_XP_CASE(5, 8, 4)
    LVKV_XP_CASE(6, 12, 4)
#undef LVKV_XP_CASE
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// cfg selects the pipeline shape (chunks in flight, chunks issued before the
// table fill); bit 64 adds per-wave timestamps. cfg 0 is production.
hipError_t launch_crc32c_wide(const UniformArgs& args, int cfg, int num_groups,
                              hipStream_t stream) {
  switch (cfg) {
#define LVKV_WIDE_CASE(c, l, pre, f)                                             \
  case c:                                                                        \
    hipLaunchKernelGGL((crc32c_wide_kernel<0, l, pre, f>), dim3(num_groups),     \
                       dim3(kGroupThreads), 0, stream, args);                    \
    break;                                                                       \
  case c + 64:                                                                   \
    hipLaunchKernelGGL((crc32c_wide_kernel<kUniProbeStamps, l, pre, f>),         \
                       dim3(num_groups), dim3(kGroupThreads), 0, stream, args);  \
    break;
    LVKV_WIDE_CASE(0, 3, 3, 0)
    LVKV_WIDE_CASE(1, 2, 2, 0)
    LVKV_WIDE_CASE(2, 3, 3, 16)
    LVKV_WIDE_CASE(3, 4, 2, 0)
    LVKV_WIDE_CASE(4, 3, 2, 0)
    LVKV_WIDE_CASE(5, 3, 3, 8)
    LVKV_WIDE_CASE(6, 8, 8, 8)
    LVKV_WIDE_CASE(7, 6, 4, 8)
    LVKV_WIDE_CASE(8, 8, 6, 4)
#undef LVKV_WIDE_CASE
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace lvkv
