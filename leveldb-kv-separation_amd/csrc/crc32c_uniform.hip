// Uniform-layout batch CRC32C for gfx950: nblocks blocks of `length` bytes at
// base + i*stride, every block END 4-byte aligned (the benchmark's 10k x 4 KiB
// batch, an SST region of equal-size blocks, 32 KiB WAL blocks at +6).
//
// Same arithmetic as crc32c_kernel.hip (see its header): end-aligned word
// grid, Horner over 256-byte rows with the Z_256 LDS tables, per-lane end
// shift Z_{256-4s}, wave xor-reduce. What differs is the schedule, built from
// measurements (tools/timeline.py, tools/probe.py):
//
//  * The row tables are GENERATED in-kernel from the 32 columns of Z_256
//    passed as kernel arguments: loading them from memory at kernel start put
//    them behind the whole batch's block stream (fill done at ~6 us).
//  * The lane tables (32 KiB) are loaded after the first round's block loads
//    and written to LDS only when the first finished blocks are flushed (one
//    barrier per wave, at its first flush or at exit).
//  * Finished blocks are queued (up to 4) and flushed together, so their
//    lane-shift lookups and reductions interleave.
//  * Loads: 16 dword loads per 4 KiB chunk (no re-alignment slot), chunks of
//    the next round issued unconditionally (out-of-range chunks read nothing)
//    so the compiler's vmcnt bookkeeping stays exact; at most 2 rounds = 64
//    loads in flight per wave.
//  * Two block streams per wave (A: gw, gw+2W, ...; B: gw+W, gw+3W, ...), their
//    row chains interleaved, as in the general kernel.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_device_common.h"
#include "crc32c_uniform_common.h"
#include "lvkv_kernel_args.h"

namespace lvkv {
namespace {

struct Cursor {  // one block stream: current block and chunk
  uint32_t block;
  uint32_t chunk;
};

__device__ __forceinline__ Cursor advance(const Cursor& c, const UniGeo& g,
                                          uint32_t block_stride) {
  Cursor n;
  const bool same = c.chunk + 1 < g.nchunks;
  n.block = same ? c.block : c.block + block_stride;
  n.chunk = same ? c.chunk + 1 : 0u;
  return n;
}

// 16 row loads of one chunk; a chunk past the batch gets an empty window so
// its loads return zeros without touching memory (keeps the issue count, and
// so the compiler's vmcnt accounting, the same on every path).
template <int P>
__device__ __forceinline__ void issue16(uint32_t (&buf)[kRowsPerChunk],
                                        const UniformArgs& a, const UniGeo& g,
                                        const Cursor& c) {
  if (P & kUniNoLoads) {
#pragma unroll
    for (int j = 0; j < kRowsPerChunk; ++j)
      buf[j] = (lane_id() * 0x9E3779B1u) ^ (static_cast<uint32_t>(j) * 0x85EBCA6Bu) ^ c.block;
    return;
  }
  const bool valid = c.block < a.nblocks;
  const uint64_t ptr = reinterpret_cast<uint64_t>(a.base) +
                       static_cast<uint64_t>(valid ? c.block : 0u) * a.stride -
                       g.delta;
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(ptr));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(ptr >> 32));
  const uint32_t n = __builtin_amdgcn_readfirstlane(valid ? g.nrec : 0u);
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<void*>((static_cast<uint64_t>(hi) << 32) | lo), 0,
      static_cast<int>(n), kBufferDword3);
  const int32_t row0 = g.vb0 + kRowBytes * kRowsPerChunk * static_cast<int32_t>(c.chunk);
  const int32_t vo = row0 + 4 * static_cast<int32_t>(lane_id());
  if (row0 >= 0) {
#pragma unroll
    for (int j = 0; j < kRowsPerChunk; ++j)
      buf[j] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, vo + 256 * j, 0,
                                                    kUniCachePolicy);
  } else {
#pragma unroll
    for (int j = 0; j < kRowsPerChunk; ++j) {
      int32_t o = vo + 256 * j;
      asm volatile("" : "+v"(o));
      buf[j] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, o, 0, kUniCachePolicy);
    }
  }
}

// Horner rows of the current chunks of streams A and B, interleaved.
__device__ __forceinline__ void rows2(const uint32_t* lds,
                                      uint32_t (&ba)[kRowsPerChunk], uint32_t na,
                                      bool first_a, uint32_t& sa,
                                      uint32_t (&bb)[kRowsPerChunk], uint32_t nb,
                                      bool first_b, uint32_t& sb,
                                      uint32_t k0, uint32_t k1) {
  if (na != 0) sa = first_a ? ba[0] : row_step(lds, sa, ba[0], k0, k1);
  if (nb != 0) sb = first_b ? bb[0] : row_step(lds, sb, bb[0], k0, k1);
  if (na == kRowsPerChunk && nb == kRowsPerChunk) {
#pragma unroll
    for (int j = 1; j < kRowsPerChunk; ++j) {
      sa = row_step(lds, sa, ba[j], k0, k1);
      sb = row_step(lds, sb, bb[j], k0, k1);
    }
  } else {
    const uint32_t nab = min(na, nb);
#pragma unroll
    for (int j = 1; j < kRowsPerChunk; ++j) {
      if (static_cast<uint32_t>(j) < nab) {
        sa = row_step(lds, sa, ba[j], k0, k1);
        sb = row_step(lds, sb, bb[j], k0, k1);
      }
    }
#pragma unroll
    for (int j = 1; j < kRowsPerChunk; ++j) {
      const uint32_t u = static_cast<uint32_t>(j);
      if (u >= nab && u < na) sa = row_step(lds, sa, ba[j], k0, k1);
    }
#pragma unroll
    for (int j = 1; j < kRowsPerChunk; ++j) {
      const uint32_t u = static_cast<uint32_t>(j);
      if (u >= nab && u < nb) sb = row_step(lds, sb, bb[j], k0, k1);
    }
  }
}

// Finished-block queue (static register slots, shifted on push).
struct Pending {
  uint32_t s0, s1, s2, s3;  // per-lane Horner states
  uint32_t b0, b1, b2, b3;  // block indices (uniform)
  uint32_t count;
};

}  // namespace

template <int P>
__global__ void __launch_bounds__(kGroupThreads, 1)
    crc32c_uniform_kernel(UniformArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsBytes / 4];

  const uint32_t tid = threadIdx.x;
  const uint32_t lane = lane_id();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t nwaves = gridDim.x * kWavesPerGroup;
  const uint32_t gw = blockIdx.x * kWavesPerGroup + wave;
  const uint32_t sstride = 2u * nwaves;
  stamp_uni<P>(a, gw, 0);
  const UniGeo g = uni_geo(a);

  // Round counts of the two streams (chunks of their blocks).
  const uint32_t nblk_a = gw < a.nblocks ? (a.nblocks - gw + sstride - 1) / sstride : 0u;
  const uint32_t gwb = gw + nwaves;
  const uint32_t nblk_b = gwb < a.nblocks ? (a.nblocks - gwb + sstride - 1) / sstride : 0u;
  const uint32_t nrounds = max(nblk_a, nblk_b) * g.nchunks;

  // 1. First round in flight.
  uint32_t a0[kRowsPerChunk], b0[kRowsPerChunk], a1[kRowsPerChunk], b1[kRowsPerChunk];
  Cursor ca0 = {gw, 0u}, cb0 = {gwb, 0u};
  if (!(P & kUniFillFirst)) {
    issue16<P>(a0, a, g, ca0);
    issue16<P>(b0, a, g, cb0);
  }
  __builtin_amdgcn_sched_barrier(0);

  // 2. Row tables from the Z_256 columns: wave w fills table t = w / 4,
  //    uint4 slots [(w % 4) * 512, +512) of that table's 2048 (8 per lane).
  {
    const uint32_t t = wave >> 2;
    const uint32_t region = (t >> 1) * kLdsRowRegionBytes + (t & 1u) * 128u;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint32_t v = (wave & 3u) * 512u + static_cast<uint32_t>(k) * 64u + lane;
      const uint32_t i = v >> 3;          // table index (8 slots of 4 copies)
      const uint32_t c4 = v & 7u;         // copies 4*c4 .. 4*c4+3
      uint32_t e = 0;
#pragma unroll
      for (int bit = 0; bit < 8; ++bit) {
        const uint32_t m = 0u - ((i >> bit) & 1u);
        e ^= m & a.zcol[8u * t + bit];
      }
      *reinterpret_cast<uint4*>(reinterpret_cast<char*>(lds) + region + i * 256u + c4 * 16u) =
          make_uint4(e, e, e, e);
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  stamp_uni<P>(a, gw, 1);
  if (P & kUniFillFirst) {
    issue16<P>(a0, a, g, ca0);
    issue16<P>(b0, a, g, cb0);
  }

  // 3. Lane tables (needed at the first flush), then the second round.
  constexpr int kLaneIters = (kLaneTabDwords / 4) / kGroupThreads;  // 2
  uint32_t lt[kLaneIters][4];
#pragma unroll
  for (int k = 0; k < kLaneIters; ++k) {
    const uint32_t* src = a.lane_tab + 4u * (tid + kGroupThreads * k);
#pragma unroll
    for (int x = 0; x < 4; ++x) lt[k][x] = src[x];
  }
  Cursor ca1 = advance(ca0, g, sstride), cb1 = advance(cb0, g, sstride);
  issue16<P>(a1, a, g, ca1);
  issue16<P>(b1, a, g, cb1);

  const uint32_t k0 = (lane & 31u) * 4u;
  const uint32_t k1 = k0 | 0x10000u;
  const uint32_t lane_base = kLdsLaneTabBase + lane * 4u;
  bool lane_ready = false;
  Pending pq = {0, 0, 0, 0, 0, 0, 0, 0, 0};

  auto flush = [&]() {
    if (!lane_ready) {
#pragma unroll
      for (int k = 0; k < kLaneIters; ++k)
        reinterpret_cast<uint4*>(lds + kLdsLaneTabBase / 4)[tid + kGroupThreads * k] =
            make_uint4(lt[k][0], lt[k][1], lt[k][2], lt[k][3]);
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      lane_ready = true;
    }
    // Up to four finishes; their lookups and reductions interleave.
    const uint32_t c0 = wave_xor_dpp(lane_end_shift(lds, pq.s0, lane_base)) ^ 0xffffffffu;
    uint32_t c1 = 0, c2 = 0, c3 = 0;
    if (pq.count > 1) c1 = wave_xor_dpp(lane_end_shift(lds, pq.s1, lane_base)) ^ 0xffffffffu;
    if (pq.count > 2) c2 = wave_xor_dpp(lane_end_shift(lds, pq.s2, lane_base)) ^ 0xffffffffu;
    if (pq.count > 3) c3 = wave_xor_dpp(lane_end_shift(lds, pq.s3, lane_base)) ^ 0xffffffffu;
    if (lane == 0) {
      a.out[pq.b0] = a.mask ? crc_mask(c0) : c0;
      if (pq.count > 1) a.out[pq.b1] = a.mask ? crc_mask(c1) : c1;
      if (pq.count > 2) a.out[pq.b2] = a.mask ? crc_mask(c2) : c2;
      if (pq.count > 3) a.out[pq.b3] = a.mask ? crc_mask(c3) : c3;
    }
    pq.count = 0;
  };
  auto push = [&](uint32_t s, uint32_t b) {
    pq.s3 = pq.s2; pq.b3 = pq.b2;
    pq.s2 = pq.s1; pq.b2 = pq.b1;
    pq.s1 = pq.s0; pq.b1 = pq.b0;
    pq.s0 = s; pq.b0 = b;
    pq.count += 1;
    if (pq.count == 4) flush();
  };

  uint32_t sa = 0, sb = 0;
  auto consume = [&](uint32_t (&ba)[kRowsPerChunk], const Cursor& ca,
                     uint32_t (&bb)[kRowsPerChunk], const Cursor& cb) {
    const bool va = ca.block < a.nblocks, vb = cb.block < a.nblocks;
    if (va && ca.chunk == 0) fix_first_chunk(ba, g);
    if (vb && cb.chunk == 0) fix_first_chunk(bb, g);
    const uint32_t na = va ? min(static_cast<uint32_t>(kRowsPerChunk),
                                 g.rows - kRowsPerChunk * ca.chunk) : 0u;
    const uint32_t nb = vb ? min(static_cast<uint32_t>(kRowsPerChunk),
                                 g.rows - kRowsPerChunk * cb.chunk) : 0u;
    if (P & kUniNoCompute) {
#pragma unroll
      for (int j = 0; j < kRowsPerChunk; ++j) {
        sa ^= ba[j];
        sb ^= bb[j];
      }
    } else {
      rows2(lds, ba, na, ca.chunk == 0, sa, bb, nb, cb.chunk == 0, sb, k0, k1);
    }
    if (va && ca.chunk + 1 == g.nchunks) push(sa, ca.block);
    if (vb && cb.chunk + 1 == g.nchunks) push(sb, cb.block);
  };

  // 4. Steady state: consume round k, issue round k+2 unconditionally.
  uint32_t k = 0;
  while (k + 2 < nrounds) {
    consume(a0, ca0, b0, cb0);
    ca0 = advance(ca1, g, sstride);
    cb0 = advance(cb1, g, sstride);
    issue16<P>(a0, a, g, ca0);
    issue16<P>(b0, a, g, cb0);
    ++k;
    if (!(k + 2 < nrounds)) {
      // Tail with the buffers swapped: rounds k (in a1/b1) and k+1 (a0/b0).
      consume(a1, ca1, b1, cb1);
      if (k + 1 < nrounds) consume(a0, ca0, b0, cb0);
      k = nrounds;
      break;
    }
    consume(a1, ca1, b1, cb1);
    ca1 = advance(ca0, g, sstride);
    cb1 = advance(cb0, g, sstride);
    issue16<P>(a1, a, g, ca1);
    issue16<P>(b1, a, g, cb1);
    ++k;
  }
  // 5. Tail: the last (up to) two rounds, nothing more to issue.
  if (k < nrounds) {
    consume(a0, ca0, b0, cb0);
    if (k + 1 < nrounds) consume(a1, ca1, b1, cb1);
  }
  stamp_uni<P>(a, gw, 2);
  if (pq.count != 0 || !lane_ready) {
    if (pq.count != 0) {
      flush();
    } else {
      // No block to finish: still write this wave's share of the lane
      // tables and pass the barrier every wave executes once.
#pragma unroll
      for (int k2 = 0; k2 < kLaneIters; ++k2)
        reinterpret_cast<uint4*>(lds + kLdsLaneTabBase / 4)[tid + kGroupThreads * k2] =
            make_uint4(lt[k2][0], lt[k2][1], lt[k2][2], lt[k2][3]);
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
  }
  stamp_uni<P>(a, gw, 7);
}

// ---------------------------------------------------------------------------
// Small batches (nblocks <= 3 x waves in the grid, blocks of <= 16 rows =
// <= 4 KiB + 252 B): ONE round per wave. Wave gw owns blocks gw, gw+W, gw+2W
// (W = waves in the grid) as three interleaved Horner chains; its 48 loads
// are issued row-interleaved (A_j, B_j, C_j) so row j can be processed as
// soon as its three words land, and everything a wave needs is in flight at
// once (48 block loads + 2 lane-table loads <= 63).

namespace {

template <int P>
__device__ __forceinline__ void row_tables_from_columns(uint32_t* lds,
                                                        const UniformArgs& a,
                                                        uint32_t wave,
                                                        uint32_t lane) {
  const uint32_t t = wave >> 2;
  const uint32_t region = (t >> 1) * kLdsRowRegionBytes + (t & 1u) * 128u;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint32_t v = (wave & 3u) * 512u + static_cast<uint32_t>(k) * 64u + lane;
    const uint32_t i = v >> 3;
    const uint32_t c4 = v & 7u;
    uint32_t e = 0;
#pragma unroll
    for (int bit = 0; bit < 8; ++bit) {
      const uint32_t m = 0u - ((i >> bit) & 1u);
      e ^= m & a.zcol[8u * t + bit];
    }
    *reinterpret_cast<uint4*>(reinterpret_cast<char*>(lds) + region + i * 256u + c4 * 16u) =
        make_uint4(e, e, e, e);
  }
}

}  // namespace

enum : int {
  kSmallLaneEarly = 4,  // lane tables loaded first, written with the row
                        // tables (one barrier; none at the end)
  kSmallEarlyA = 8,     // chain A's loads issued before the row-table fill
  kSmallOneBarrier = 16,  // lane tables first, chain A, fill, chains B/C,
                          // write lane tables, then the only barrier
  kSmallSkipFill = 32,    // probe: no row-table fill (CRCs wrong)
  kSmallHalfA = 256,      // with kSmallEarlyA: only waves 0-7 load chain A
                          // before the fill
  kSmallBare = 4096,      // probe: loads + xor only (no tables, no walk)
};

// Body of the small kernel for a wave with NCH valid chains (1..3). Every
// value a body loads is consumed unconditionally, so the compiler cannot sink
// a load into the branch that uses it; FULL = 16-row (4 KiB-class) blocks,
// no per-row guards. Every body executes the same barriers.
template <int P, int NCH, bool FULL>
__device__ __forceinline__ void small_body(const UniformArgs& a, const UniGeo& g,
                                           uint32_t* lds, uint32_t tid,
                                           uint32_t lane, uint32_t wave,
                                           uint32_t gw, const uint32_t (&blk)[3]) {
  constexpr bool kLaneEarly = (P & kSmallLaneEarly) != 0;
  constexpr bool kEarlyA = (P & kSmallEarlyA) != 0;
  constexpr bool kFillBeforeBC = (P & (kUniFillFirst | kSmallEarlyA)) != 0;
  constexpr int kLaneIters = (kLaneTabDwords / 4) / kGroupThreads;  // 2

  uint32_t lt[kLaneIters][4];
  auto load_lane_tables = [&]() {
#pragma unroll
    for (int k = 0; k < kLaneIters; ++k) {
      const uint32_t* src = a.lane_tab + 4u * (tid + kGroupThreads * k);
#pragma unroll
      for (int x = 0; x < 4; ++x) lt[k][x] = src[x];
    }
  };
  auto write_lane_tables = [&]() {
#pragma unroll
    for (int k = 0; k < kLaneIters; ++k)
      reinterpret_cast<uint4*>(lds + kLdsLaneTabBase / 4)[tid + kGroupThreads * k] =
          make_uint4(lt[k][0], lt[k][1], lt[k][2], lt[k][3]);
  };

  __amdgpu_buffer_rsrc_t r[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c)  // invalid only for NCH == 1 past the batch
    r[c] = block_rsrc<P>(a, g, blk[c], NCH > 1 || blk[c] < a.nblocks);
  const int32_t vo = g.vb0 + 4 * static_cast<int32_t>(lane);
  int32_t vo1 = vo + kRowBytes;
  asm volatile("" : "+v"(vo1));
  uint32_t w[NCH][kRowsPerChunk];
  auto load_rows = [&](int c_lo, int c_hi) {  // row-interleaved over chains
#pragma unroll
    for (int j = 0; j < kRowsPerChunk; ++j)
#pragma unroll
      for (int c = 0; c < NCH; ++c)
        if (c >= c_lo && c < c_hi)
          w[c][j] = (P & kUniNoLoads)
                        ? (lane * 0x9E3779B1u) ^ (static_cast<uint32_t>(j) * 0x85EBCA6Bu) ^ blk[c]
                        : load_word(r[c], vo, vo1, j);
  };
  auto fill = [&]() {
    stamp_uni<P>(a, gw, 3);
    if (!(P & kSmallSkipFill)) row_tables_from_columns<P>(lds, a, wave, lane);
    if (kLaneEarly) write_lane_tables();
    stamp_uni<P>(a, gw, 4);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);  // nothing that waits on loads moves up
    stamp_uni<P>(a, gw, 1);
  };

  // 1. Loads and the LDS image, in the order the variant asks for.
  if (P & kSmallOneBarrier) {
    load_lane_tables();
    __builtin_amdgcn_sched_barrier(0);
    load_rows(0, 1);
    __builtin_amdgcn_sched_barrier(0);
    row_tables_from_columns<P>(lds, a, wave, lane);
    __builtin_amdgcn_sched_barrier(0);
    load_rows(1, NCH);
    __builtin_amdgcn_sched_barrier(0);
    write_lane_tables();
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    stamp_uni<P>(a, gw, 1);
  } else if (kFillBeforeBC) {
    if (kLaneEarly) {
      load_lane_tables();
      __builtin_amdgcn_sched_barrier(0);  // keep them ahead of the block loads
    }
    // kSmallHalfA: waves 8-15 leave chain A until after the fill
    const bool early_a = kEarlyA && (!(P & kSmallHalfA) || wave < kWavesPerGroup / 2);
    if (early_a) {
      load_rows(0, 1);
      __builtin_amdgcn_sched_barrier(0);
    }
    fill();
    if (early_a) load_rows(1, NCH); else load_rows(0, NCH);
    stamp_uni<P>(a, gw, 5);
    if (!kLaneEarly) load_lane_tables();
  } else {
    if (kLaneEarly) {
      load_lane_tables();
      __builtin_amdgcn_sched_barrier(0);
    }
    load_rows(0, NCH);
    if (!kLaneEarly) load_lane_tables();
    fill();
  }

  // 2. Rows: the chains interleaved; row-0 fix-ups first.
  const uint32_t k0 = (lane & 31u) * 4u;
  const uint32_t k1 = k0 | 0x10000u;
  uint32_t st[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    fix_first_chunk(w[c], g);
    st[c] = w[c][0];
  }
  auto walk = [&](int c_lo, int c_hi) {  // rows 1.., chains [c_lo, c_hi) interleaved
#pragma unroll
    for (int j = 1; j < kRowsPerChunk; ++j) {
      if (FULL || static_cast<uint32_t>(j) < g.rows) {
#pragma unroll
        for (int c = 0; c < NCH; ++c)
          if (c >= c_lo && c < c_hi)
            st[c] = (P & kUniNoCompute) ? (st[c] * 0x01000193u) ^ w[c][j]
                                        : row_step(lds, st[c], w[c][j], k0, k1);
      }
    }
  };
  const uint32_t lane_base = kLdsLaneTabBase + lane * 4u;
  uint32_t crc[NCH];
  auto reduce = [&](int c_lo, int c_hi) {  // end shift + reduction
#pragma unroll
    for (int c = 0; c < NCH; ++c)
      if (c >= c_lo && c < c_hi)
        crc[c] = wave_xor_dpp(lane_end_shift(lds, st[c], lane_base)) ^ 0xffffffffu;
  };
  // One store pass at the very end: a global store between the chains'
  // waits would make the compiler's vmcnt accounting conservative.
  auto store = [&]() {
    if (lane == 0) {
#pragma unroll
      for (int c = 0; c < NCH; ++c)
        if (NCH > 1 || blk[c] < a.nblocks) a.out[blk[c]] = a.mask ? crc_mask(crc[c]) : crc[c];
    }
  };
  walk(0, NCH);
  stamp_uni<P>(a, gw, 2);

  // 3. Lane tables (unless already in LDS), end shift + reduction, store.
  if (!kLaneEarly && !(P & kSmallOneBarrier)) {
    write_lane_tables();
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  reduce(0, NCH);
  store();
}

// Probe: the memory side alone (same loads, mapping and LDS footprint).
template <int P, int NCH>
__device__ __forceinline__ void small_body_bare(const UniformArgs& a, const UniGeo& g,
                                                uint32_t* lds, uint32_t lane,
                                                const uint32_t (&blk)[3]) {
  __amdgpu_buffer_rsrc_t r[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c)
    r[c] = block_rsrc<P>(a, g, blk[c], NCH > 1 || blk[c] < a.nblocks);
  const int32_t vo = g.vb0 + 4 * static_cast<int32_t>(lane);
  int32_t vo1 = vo + kRowBytes;
  asm volatile("" : "+v"(vo1));
  uint32_t w[NCH][kRowsPerChunk];
#pragma unroll
  for (int j = 0; j < kRowsPerChunk; ++j)
#pragma unroll
    for (int c = 0; c < NCH; ++c) w[c][j] = load_word(r[c], vo, vo1, j);
  uint32_t x = 0;
#pragma unroll
  for (int j = 0; j < kRowsPerChunk; ++j)
#pragma unroll
    for (int c = 0; c < NCH; ++c) x ^= w[c][j];
  lds[lane] = x;  // keeps the LDS allocation live
  if (lane == 0)
#pragma unroll
    for (int c = 0; c < NCH; ++c)
      if (NCH > 1 || blk[c] < a.nblocks) a.out[blk[c]] = x;
}

template <int P, int NCH, bool FULL>
__device__ __forceinline__ void small_dispatch(const UniformArgs& a, const UniGeo& g,
                                               uint32_t* lds, uint32_t tid, uint32_t lane,
                                               uint32_t wave, uint32_t gw,
                                               const uint32_t (&blk)[3]) {
  if (P & kSmallBare)
    small_body_bare<P, NCH>(a, g, lds, lane, blk);
  else
    small_body<P, NCH, FULL>(a, g, lds, tid, lane, wave, gw, blk);
}

template <int P>
__global__ void __launch_bounds__(kGroupThreads, 1)
    crc32c_uniform_small_kernel(UniformArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsBytes / 4];
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = lane_id();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t nwaves = gridDim.x * kWavesPerGroup;
  const uint32_t gw = blockIdx.x * kWavesPerGroup + wave;
  stamp_uni<P>(a, gw, 0);
  const UniGeo g = uni_geo(a);
  // Chains A and B: 16 contiguous blocks per workgroup each. Chain C (the
  // partial third round, nc = nblocks - 2W blocks) is split into equal
  // contiguous runs per workgroup (waves 0.. of group g take run g), so every
  // CU gets the same share and each CU's CRC stores stay in one run. A
  // wave's valid chains are a prefix (C valid => B valid => A valid).
  const uint32_t nc = a.nblocks > 2u * nwaves ? a.nblocks - 2u * nwaves : 0u;
  const uint32_t per = nc / gridDim.x, extra = nc % gridDim.x;
  const uint32_t run_len = per + (blockIdx.x < extra ? 1u : 0u);
  const uint32_t run_start = blockIdx.x * per + min(blockIdx.x, extra);
  const uint32_t blk_c = wave < run_len ? 2u * nwaves + run_start + wave : 0xffffffffu;
  const uint32_t blk[3] = {gw, gw + nwaves, blk_c};
  const bool full = g.rows == static_cast<uint32_t>(kRowsPerChunk);
  if (blk[2] < a.nblocks) {
    if (full) small_dispatch<P, 3, true>(a, g, lds, tid, lane, wave, gw, blk);
    else small_dispatch<P, 3, false>(a, g, lds, tid, lane, wave, gw, blk);
  } else if (blk[1] < a.nblocks) {
    if (full) small_dispatch<P, 2, true>(a, g, lds, tid, lane, wave, gw, blk);
    else small_dispatch<P, 2, false>(a, g, lds, tid, lane, wave, gw, blk);
  } else {
    // One chain; a wave past the batch (only in the last workgroup) runs it
    // over an empty window and stores nothing, keeping the barrier count.
    const uint32_t one[3] = {blk[0] < a.nblocks ? blk[0] : 0xffffffffu, 0, 0};
    if (full) small_dispatch<P, 1, true>(a, g, lds, tid, lane, wave, gw, one);
    else small_dispatch<P, 1, false>(a, g, lds, tid, lane, wave, gw, one);
  }
  stamp_uni<P>(a, gw, 7);
}

hipError_t launch_crc32c_uniform_small(const UniformArgs& args, int variant,
                                       int num_groups, hipStream_t stream) {
  switch (variant & (kUniProbeStamps | kUniFillFirst | kSmallLaneEarly | kSmallEarlyA |
                     kSmallOneBarrier | kSmallSkipFill | kUniNoCompute | kUniNoLoads |
                     kSmallHalfA | kSmallBare)) {
#define LVKV_UNI_SMALL_CASE(v)                                               \
  case v:                                                                    \
    hipLaunchKernelGGL(crc32c_uniform_small_kernel<v>, dim3(num_groups),     \
                       dim3(kGroupThreads), 0, stream, args);                \
    break;
#define LVKV_UNI_SMALL_PAIR(v) LVKV_UNI_SMALL_CASE(v) LVKV_UNI_SMALL_CASE(v + 64)
    LVKV_UNI_SMALL_CASE(12)   // production: lane tables first, chain A before the fill
#ifdef LVKV_PROBE_BUILD
    LVKV_UNI_SMALL_CASE(76)   // 12 with stamps
    LVKV_UNI_SMALL_PAIR(0)    // all loads, then the fill
    LVKV_UNI_SMALL_PAIR(4)    // + lane tables first
    LVKV_UNI_SMALL_PAIR(8)    // chain A before the fill
    LVKV_UNI_SMALL_PAIR(16)   // one barrier after chains B/C
    LVKV_UNI_SMALL_PAIR(128)  // fill first
    LVKV_UNI_SMALL_PAIR(132)
    LVKV_UNI_SMALL_PAIR(268)  // 12, chain A early in waves 0-7 only
    LVKV_UNI_SMALL_PAIR(13)   // probes: 12 without the table walk,
    LVKV_UNI_SMALL_PAIR(14)   //   without block loads,
    LVKV_UNI_SMALL_PAIR(44)   //   without the row-table fill,
    LVKV_UNI_SMALL_PAIR(15)   //   loads and walk both off
    LVKV_UNI_SMALL_PAIR(4096)  // memory side only
#endif
#undef LVKV_UNI_SMALL_PAIR
#undef LVKV_UNI_SMALL_CASE
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_crc32c_uniform(const UniformArgs& args, int variant,
                                 int num_groups, hipStream_t stream) {
  switch (variant & (kUniProbeStamps | kUniFillFirst | kUniNoCompute | kUniNoLoads)) {
#define LVKV_UNI_CASE(v)                                                     \
  case v:                                                                    \
    hipLaunchKernelGGL(crc32c_uniform_kernel<v>, dim3(num_groups),           \
                       dim3(kGroupThreads), 0, stream, args);                \
    break;
    LVKV_UNI_CASE(0)  // production
#ifdef LVKV_PROBE_BUILD
    LVKV_UNI_CASE(1)
    LVKV_UNI_CASE(2)
    LVKV_UNI_CASE(3)
    LVKV_UNI_CASE(64)
    LVKV_UNI_CASE(65)
    LVKV_UNI_CASE(66)
    LVKV_UNI_CASE(67)
    LVKV_UNI_CASE(128)
    LVKV_UNI_CASE(129)
    LVKV_UNI_CASE(130)
    LVKV_UNI_CASE(131)
    LVKV_UNI_CASE(192)
    LVKV_UNI_CASE(193)
    LVKV_UNI_CASE(194)
    LVKV_UNI_CASE(195)
#endif
#undef LVKV_UNI_CASE
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace lvkv
