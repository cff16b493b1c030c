// The general-layout batch walk of crc32c_ragged.hip as a device function
// (ragged_run), shared by crc32c_ragged_kernel and the fused whole-SSTable
// verify (lvkv_sst_table.hip), whose CRC workgroups run it once the table
// heads of the same launch have published their block lists.
//
// Arithmetic as in the other kernels: the block is laid on a grid of 4-byte
// words aligned to its END, lane s of row r holds grid word 64r + s, Horner
// over rows with Z_256 (row_step_c), per-lane end shift Z_{256-4s}, wave
// xor-reduce.
//
// A block whose end is not 4-byte aligned (e = end & 3) is read as aligned
// dwords D and each grid word rebuilt as v_alignbyte(D_next, D, e), where
// D_next (lane s + 1's dword; lane 63: lane 0 of the next row) comes from a
// DPP wave_rol:1 of the row, a VALU op (crc32c_kernel.hip uses ds_bpermute,
// an LDS instruction beside the walk's own). Unaligned dword loads measured
// 40% slower on 4271-byte blocks. The window is [floor4(ptr), ceil4(end)), so
// no dword outside the block's own is read; dwords before it come back as
// zeros and the front padding is masked.
//
// Layout: per-block offsets and lengths, or (offsets == nullptr, compute
// mode) block b at base + b * stride of `length` bytes.
//
// Work map: G contiguous runs of equal length. A run is walked in rounds of
// W * NCH blocks: wave w, chain c takes block c * W + w of the round. Each
// chain's block is read in chunks of R rows, all chains' loads in flight
// together, chains walked interleaved. Blocks over 64 KiB (long_split) are
// walked at the end of the run by the whole workgroup, blocks under 4 bytes
// bitwise by lane 0.
#ifndef LVKV_CRC32C_RAGGED_BODY_H_
#define LVKV_CRC32C_RAGGED_BODY_H_

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_compact_common.h"
#include "crc32c_device_common.h"
#include "lvkv_crc32c.h"
#include "lvkv_kernel_args.h"

namespace lvkv {
namespace {

constexpr int kRagCachePolicy = 2;  // nt: block bytes are read once

enum : uint32_t { kRagNone = 0, kRagRows = 1, kRagTiny = 2, kRagSkip = 3 };

// One chain's block, wave-uniform. Only what the mode parse produces is
// kept; the grid geometry is recomputed where it is used (scalar ALU is
// cheaper than the SGPRs: three chains of a wider struct spill).
struct RagBlock {
  uint32_t ptr_lo, ptr_hi;  // first covered byte
  uint32_t len;             // covered bytes
  uint32_t s0;              // init ^ ~0, xored into the first 4 data bytes
  uint32_t expected;        // verify modes: unmasked stored CRC
  uint32_t kind;
  __device__ __forceinline__ uint64_t ptr() const {
    return (static_cast<uint64_t>(ptr_hi) << 32) | ptr_lo;
  }
  __device__ __forceinline__ uint32_t q() const { return (len + 3u) >> 2; }  // grid words
  __device__ __forceinline__ uint32_t rows() const { return (q() + 63u) >> 6; }
  __device__ __forceinline__ uint32_t delta() const { return 4u * q() - len; }
  __device__ __forceinline__ uint32_t s0l() const { return 64u * rows() - q(); }
  __device__ __forceinline__ uint32_t spill() const {
    return delta() ? (s0 >> (32u - 8u * delta())) : 0u;
  }
  __device__ __forceinline__ uint32_t e() const { return (ptr_lo + len) & 3u; }  // end misalignment
  // window [floor4(ptr), ceil4(end)): the aligned dwords holding the block
  __device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc() const {
    const uint64_t b4 = ptr() & ~uint64_t{3};
    const uint64_t e4 = (ptr() + len + 3u) & ~uint64_t{3};
    const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(b4));
    const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(b4 >> 32));
    const uint32_t n = __builtin_amdgcn_readfirstlane(kind == kRagRows ? static_cast<uint32_t>(e4 - b4) : 0u);
    return __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void*>((static_cast<uint64_t>(hi) << 32) | lo), 0, static_cast<int>(n),
        kBufferDword3);
  }
  // window offset of the aligned dword holding grid word 0: floor4(end) - 4q
  // - floor4(ptr), which is -4 or 0
  __device__ __forceinline__ int32_t base_off() const {
    const uint32_t end4 = (ptr_lo + len) & ~3u;
    return static_cast<int32_t>(end4 - 4u * q() - (ptr_lo & ~3u));
  }
};

// Descriptor b. Written by an earlier launch: through the scalar cache.
// Written by workgroups of this same launch (a.fresh_desc, the fused SST
// verify): vector loads after the caller's acquire, never a scalar-cache line
// that could predate the write.
__device__ __forceinline__ uint64_t desc_u64(const KernelArgs& a, uint32_t b) {
  if (!a.fresh_desc) return sload_u64(a.offsets, b);
  const uint64_t v = __hip_atomic_load(a.offsets + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v >> 32));
  return (static_cast<uint64_t>(hi) << 32) | lo;
}
__device__ __forceinline__ uint32_t desc_u32(const KernelArgs& a, uint32_t b) {
  if (!a.fresh_desc) return sload_u32(a.lengths, b);
  return __builtin_amdgcn_readfirstlane(
      __hip_atomic_load(a.lengths + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// Block b's covered range and verdict inputs by mode (crc32c_kernel.hip
// make_geo: log headers, SST trailers, per-block inits).
// With `defer`, an SST mode's stored trailer is not loaded here: the walk
// loads it with a vector load when the block's round starts (RagRound::adopt)
// and reads it at the store, so no scalar load is outstanding while the walk
// waits on its LDS reads (one lgkmcnt counts both).
__device__ __forceinline__ RagBlock rag_block(const KernelArgs& a, uint32_t b, bool live,
                                              bool defer = false) {
  RagBlock g;
  g.ptr_lo = g.ptr_hi = g.len = g.s0 = g.expected = 0;
  g.kind = kRagNone;
  if (!live) return g;
  const uint64_t base = reinterpret_cast<uint64_t>(a.base);
  uint64_t off;
  uint32_t len, init = a.init, expected = 0;
  if (a.mode == kModeLogVerify || a.mode == kModeLogFill || a.mode == kModeLogStaged) {
    // [masked crc u32][len u16][type u8]; the CRC covers type + payload
    // (db/log_reader.cc:217-221, 243-247).
    const uint64_t hoff = desc_u64(a, b);
    const uint32_t len_type = sload_le(base + hoff + 4, 3);
    if (a.mode != kModeLogFill) expected = crc_unmask(sload_le(base + hoff, 4));
    off = hoff + 6;
    len = 1u + (len_type & 0xffffu);
    init = 0;
  } else {
    if (a.offsets == nullptr) {  // uniform layout: block b at base + b * stride
      off = static_cast<uint64_t>(b) * a.stride;
      len = a.length;
    } else {
      off = desc_u64(a, b);
      len = desc_u32(a, b);
    }
    if (a.inits != nullptr) init = sload_u32(a.inits, b);
  }
  if (a.mode == kModeSstVerify || a.mode == kModeSstFill || a.mode == kModeSstTable) {
    // contents n bytes + type byte; the masked CRC follows
    // (table/format.cc:92-94, table/table_builder.cc:199-203)
    len += 1;
    init = 0;
    if (a.mode != kModeSstFill && !defer) expected = crc_unmask(sload_le(base + off + len, 4));
  }
  const uint64_t ptr = base + off;
  g.ptr_lo = static_cast<uint32_t>(ptr);
  g.ptr_hi = static_cast<uint32_t>(ptr >> 32);
  g.len = len;
  g.s0 = init ^ 0xffffffffu;
  g.expected = expected;
  if (a.long_split && len > a.long_split) {
    g.kind = kRagSkip;
    return g;
  }
  if (len < 4) {
    g.kind = kRagTiny;
    return g;
  }
  g.kind = kRagRows;
  return g;
}

__device__ __forceinline__ uint32_t rag_tiny(const RagBlock& g) {
  uint32_t reg = g.s0;
  if (g.len > 0) {
    const uint32_t bytes = sload_le(g.ptr(), g.len);
    for (uint32_t i = 0; i < g.len; ++i) {
      reg ^= (bytes >> (8u * i)) & 0xffu;
#pragma unroll
      for (int k = 0; k < 8; ++k) reg = (reg >> 1) ^ (kCastagnoliReflected & (0u - (reg & 1u)));
    }
  }
  return reg ^ 0xffffffffu;
}

// A value written by this launch's other workgroups (a.fresh_desc) or by an
// earlier launch: agent-scope atomic load or a plain one.
template <typename T>
__device__ __forceinline__ T fresh_ld(const KernelArgs& a, const T* p) {
  return a.fresh_desc ? __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : *p;
}

// Table of entry e in kModeSstTable: the last report whose first <= e.
__device__ __forceinline__ uint32_t sst_table_of(const KernelArgs& a,
                                                 const lvkv_sst_report* reports, uint32_t ntables,
                                                 uint32_t e) {
  uint32_t lo = 0, hi = ntables;  // answer in [lo, hi)
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (fresh_ld(a, &reports[mid].first) <= e) lo = mid; else hi = mid;
  }
  return lo;
}

// Lane 0 stores block b's result in the batch's mode.
__device__ __forceinline__ void rag_store(const KernelArgs& a, uint32_t b, const RagBlock& g,
                                          uint32_t crc) {
  if (lane_id() != 0) return;
  if (a.mode == kModeSstTable) {
    // ReadBlock's order (format.cc:92-97, :104-158): the index parse status
    // first, then the checksum, then the type byte
    uint8_t st = fresh_ld(a, a.out_status + b);
    a.out_crc[b] = st == LVKV_BLOCK_OK ? crc : 0u;  // no CRC of an unreadable block
    if (st == LVKV_BLOCK_OK) {
      const uint8_t type = *reinterpret_cast<const uint8_t*>(g.ptr() + g.len - 1);
      if (crc != g.expected)
        st = LVKV_BLOCK_CHECKSUM;
      else if (type == 1 || type == 2)  // snappy / zstd: absent in the as-built
        st = LVKV_BLOCK_COMPRESSED;     // reference (port_stdcxx.h:108-118)
      else if (type > 2)
        st = LVKV_BLOCK_BAD_TYPE;
      if (st != LVKV_BLOCK_OK) a.out_status[b] = st;
    }
    if (st != LVKV_BLOCK_OK) {
      lvkv_sst_report* reps = static_cast<lvkv_sst_report*>(a.sst_reports);
      lvkv_sst_report* r = reps + sst_table_of(a, reps, a.sst_ntables, b);
      atomicAdd(&r->nbad, 1u);
      atomicMin(&r->first_bad, b - fresh_ld(a, &r->first));
    }
  } else if (a.mode == kModeCompute) {
    a.out_crc[b] = a.mask ? crc_mask(crc) : crc;
  } else if (a.mode == kModeSstFill || a.mode == kModeLogFill) {
    // the stored form (Mask, little-endian) into the trailer / header hole
    uint8_t* dst = reinterpret_cast<uint8_t*>(a.mode == kModeSstFill ? g.ptr() + g.len
                                                                     : g.ptr() - 6);
    const uint32_t m = crc_mask(crc);
#pragma unroll
    for (int k = 0; k < 4; ++k) dst[k] = static_cast<uint8_t>(m >> (8 * k));
    if (a.out_crc != nullptr) a.out_crc[b] = crc;
  } else {
    a.out_crc[b] = crc;
    if (a.out_status != nullptr) a.out_status[b] = crc != g.expected ? 1 : 0;
    if (a.mode == kModeLogStaged && crc != g.expected) {
      // the block's first mismatch (its records are staged in file order)
      const uint64_t hoff = g.ptr() - 6u - reinterpret_cast<uint64_t>(a.base);
      atomicMin(a.log_first_bad + (hoff >> 15), b);
    }
  }
}

// Where a walk's blocks come from and where its results go: the batch's
// descriptor arrays and rag_store (ArgsSrc), or a caller's own list (the
// whole-SSTable verify's entries decoded into LDS, lvkv_sst_table.hip).
struct ArgsSrc {
  // the stored CRC follows the covered bytes (SST verify modes): loaded by
  // the walk (RagRound::adopt), not by block()
  __device__ __forceinline__ bool trailer(const KernelArgs& a) const {
    return a.mode == kModeSstVerify || a.mode == kModeSstTable;
  }
  __device__ __forceinline__ RagBlock block(const KernelArgs& a, uint32_t b, bool live) const {
    return rag_block(a, b, live, trailer(a));
  }
  __device__ __forceinline__ void store(const KernelArgs& a, uint32_t b, const RagBlock& g,
                                        uint32_t crc) const {
    rag_store(a, b, g, crc);
  }
  // covered length of block b, as rag_block computes it (the long-block scan)
  __device__ __forceinline__ uint32_t covered(const KernelArgs& a, uint32_t b) const {
    const bool sst = a.mode == kModeSstVerify || a.mode == kModeSstFill || a.mode == kModeSstTable;
    const bool log = a.mode == kModeLogVerify || a.mode == kModeLogFill || a.mode == kModeLogStaged;
    if (log) {
      const uint8_t* h = a.base + fresh_ld(a, a.offsets + b);
      return 1u + (static_cast<uint32_t>(h[4]) | (static_cast<uint32_t>(h[5]) << 8));
    }
    return (a.offsets == nullptr ? a.length : fresh_ld(a, a.lengths + b)) + (sst ? 1u : 0u);
  }
};

// One round of one wave: NCH chains (blocks), chunk k of each in flight.
template <int NCH, int R>
struct RagRound {
  RagBlock g[NCH];
  uint32_t blk[NCH];
  uint32_t nchunks;  // max over the chains, >= 1
  uint32_t w[NCH][R + 1];  // row R: the neighbour dwords of row R - 1
  uint32_t x[NCH];  // the stored trailer's aligned dwords (Src::trailer): lanes 0, 1

  // Chain c of round r0 is block start + r0 + c * W + wave.
  template <class Src>
  __device__ static __forceinline__ void fetch(RagBlock (&out)[NCH], const KernelArgs& a,
                                               const Src& src, uint32_t start, uint32_t n,
                                               uint32_t r0, uint32_t wave, uint32_t W) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const uint32_t i = r0 + static_cast<uint32_t>(c) * W + wave;
      out[c] = src.block(a, start + i, i < n);
    }
  }
  // `trailer`: load each block's stored CRC (the 4 bytes after it) now, as
  // vector loads issued before the round's rows; expected() reads them.
  __device__ __forceinline__ void adopt(const RagBlock (&in)[NCH], uint32_t start, uint32_t r0,
                                        uint32_t wave, uint32_t W, bool trailer) {
    nchunks = 1;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      g[c] = in[c];
      blk[c] = start + r0 + static_cast<uint32_t>(c) * W + wave;
      if (g[c].kind == kRagRows) nchunks = max(nchunks, (g[c].rows() + R - 1) / R);
      x[c] = 0;
      if (trailer && (g[c].kind == kRagRows || g[c].kind == kRagTiny)) {
        // lane 0 the dword holding the trailer's first byte, lane 1 the next
        // (when the trailer straddles two)
        const uint64_t t = g[c].ptr() + g[c].len;
        const uint32_t lane = lane_id();
        if (lane == 0 || (lane == 1 && (t & 3u)))
          x[c] = gload32((t & ~uint64_t{3}) + 4u * lane);
      }
    }
  }
  __device__ __forceinline__ uint32_t expected(int c) const {
    const uint32_t sh = static_cast<uint32_t>(g[c].ptr_lo + g[c].len) & 3u;
    const uint32_t lo = __builtin_amdgcn_readlane(x[c], 0), hi = __builtin_amdgcn_readlane(x[c], 1);
    return crc_unmask(__builtin_amdgcn_alignbyte(hi, lo, sh));
  }

  // R + 1 loads per chain, unconditional: rows past the block (and every
  // row of an idle chain) are outside the window and come back as zeros
  // without a memory access, and branch-free issue keeps the vmcnt waits
  // exact.
  __device__ __forceinline__ void issue(uint32_t k, uint32_t lane) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const __amdgpu_buffer_rsrc_t rs = g[c].rsrc();
      const int32_t vo = g[c].base_off() + 4 * static_cast<int32_t>(lane) -
                         4 * static_cast<int32_t>(g[c].s0l()) +
                         kRowBytes * R * static_cast<int32_t>(k);
      // row 0 of chunk 0: lanes before s0l (and the dword before the block)
      // read zeros through a negative offset; rows >= 1 start at vo1 >= 0
      int32_t o0 = vo;
      asm volatile("" : "+v"(o0));
      w[c][0] = __builtin_amdgcn_raw_buffer_load_b32(rs, o0, 0, kRagCachePolicy);
      int32_t vo1 = vo + kRowBytes;
      asm volatile("" : "+v"(vo1));
#pragma unroll
      for (int j = 1; j <= R; ++j)
        w[c][j] = __builtin_amdgcn_raw_buffer_load_b32(rs, vo1 + kRowBytes * (j - 1), 0,
                                                       kRagCachePolicy);
    }
  }

  // Grid words of chain c from its aligned dwords (end misalignment e != 0).
  __device__ __forceinline__ void realign(int c, uint32_t lane) {
    const uint32_t e = g[c].e();
    uint32_t r0 = static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(w[c][0]), 0x134,
                                                                 0xF, 0xF, false));
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const uint32_t r1 = static_cast<uint32_t>(
          __builtin_amdgcn_mov_dpp(static_cast<int>(w[c][j + 1]), 0x134, 0xF, 0xF, false));
      const uint32_t hi = lane == 63u ? r1 : r0;  // wave_rol:1 = lane s + 1's dword
      w[c][j] = __builtin_amdgcn_alignbyte(hi, w[c][j], e);
      r0 = r1;
    }
  }
};

// LDS dwords of a W-wave ragged workgroup: the compact image, then (long
// blocks only) one accumulator per wave, a flag, a list of 64 * W block ids
// and its length.
template <int W>
struct RagLds {
  static constexpr uint32_t kAcc = kCompactLdsBytes / 4, kFlag = kAcc + W, kList = kFlag + 1,
                            kCount = kList + 64 * W, kDwords = kCount + 1;
};

// Blocks over kLongBytes in the run [start, start + n) (rare): the whole
// workgroup walks each one, 16 KiB segments over the waves (workgroup_crc),
// instead of a second kernel launch per batch. The run's lengths are scanned
// 64 * W at a time only when a wave met one (lds[kFlag], set by the walk).
// Every thread of the workgroup calls it.
template <int W, class Src = ArgsSrc>
__device__ __forceinline__ void ragged_long_pass(const KernelArgs& a, const uint32_t* zpow,
                                                 uint32_t* lds, uint32_t start, uint32_t n,
                                                 const LaneKeys& keys, uint32_t lane_base,
                                                 const Src& src = Src()) {
  constexpr uint32_t kAcc = RagLds<W>::kAcc, kFlag = RagLds<W>::kFlag,
                     kList = RagLds<W>::kList, kCount = RagLds<W>::kCount;
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = lane_id();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  __syncthreads();
  if (lds[kFlag] == 0) return;
  for (uint32_t slice = 0; slice < n; slice += 64 * W) {
    if (tid == 0) lds[kCount] = 0;
    __syncthreads();
    const uint32_t i = slice + tid;
    if (i < n && src.covered(a, start + i) > a.long_split)
      lds[kList + atomicAdd(&lds[kCount], 1u)] = start + i;
    __syncthreads();
    const uint32_t cnt = __builtin_amdgcn_readfirstlane(lds[kCount]);
    for (uint32_t li = 0; li < cnt; ++li) {
      const uint32_t b = __builtin_amdgcn_readfirstlane(lds[kList + li]);
      RagBlock g = src.block(a, b, true);
      if (src.trailer(a)) g.expected = crc_unmask(sload_le(g.ptr() + g.len, 4));
      // WAL fragments (<= 32 KiB): 4 KiB segments, one per wave; longer
      // blocks: 16 KiB segments
      const uint32_t crc =
          g.len <= 32768u
              ? workgroup_crc<W, 4096>(lds, lds + kAcc, g.ptr(), g.ptr() + g.len,
                                       g.s0 ^ 0xffffffffu, keys, tid, wave, lane, lane_base, zpow)
              : workgroup_crc<W>(lds, lds + kAcc, g.ptr(), g.ptr() + g.len, g.s0 ^ 0xffffffffu,
                                 keys, tid, wave, lane, lane_base, zpow);
      if (tid == 0) src.store(a, b, g, crc);
    }
    __syncthreads();
  }
}

// Workgroup `grp` of G walks its run of blocks [0, total). `image_ready`:
// the caller built the compact image in `lds` (and zeroed lds[kFlag]) before
// a barrier; otherwise it is built here, overlapped with the first loads.
// Every thread of the workgroup calls it; it returns workgroup-uniformly.
template <int W, int NCH, int R, class Src = ArgsSrc>
__device__ __forceinline__ void ragged_run(const KernelArgs& a, const uint32_t* zpow,
                                           const uint32_t* lane_cols, uint32_t* lds,
                                           uint32_t grp, uint32_t G, uint32_t total,
                                           bool image_ready, const Src& src = Src()) {
  constexpr uint32_t kFlag = RagLds<W>::kFlag;
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = lane_id();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  uint32_t start, n;
  if (a.run_base != nullptr) {  // runs of whole units (bytes balanced)
    const uint32_t U = a.run_units;
    const uint32_t u0 = static_cast<uint32_t>(static_cast<uint64_t>(grp) * U / G);
    const uint32_t u1 = static_cast<uint32_t>(static_cast<uint64_t>(grp + 1) * U / G);
    start = min(total, sload_u32(a.run_base, u0));
    const uint32_t end = u1 < U ? min(total, sload_u32(a.run_base, u1)) : total;
    n = end > start ? end - start : 0u;
  } else {
    const uint32_t per = total / G, extra = total % G;
    n = per + (grp < extra ? 1u : 0u);
    start = grp * per + min(grp, extra);
  }
  if (n == 0) return;  // the whole workgroup: no barrier is left waiting

  // 1. table loads, round 0's first chunk in flight, the LDS image, barrier
  RagRound<NCH, R> rd;
  if (image_ready) {
    RagBlock g0[NCH];
    RagRound<NCH, R>::fetch(g0, a, src, start, n, 0, wave, W);
    rd.adopt(g0, start, 0, wave, W, src.trailer(a));
    rd.issue(0, lane);
  } else {
    RowTabStage<64 * W> rt;
    LaneTabGen<W> lg;
    rt.load(zpow, tid);
    lg.load(lane_cols, wave, lane);
    {
      RagBlock g0[NCH];
      RagRound<NCH, R>::fetch(g0, a, src, start, n, 0, wave, W);
      rd.adopt(g0, start, 0, wave, W, src.trailer(a));
    }
    __builtin_amdgcn_sched_barrier(0);
    rd.issue(0, lane);
    __builtin_amdgcn_sched_barrier(0);
    rt.store(lds, tid);
    lg.store(lds, wave, lane);
    if (tid == 0) lds[kFlag] = 0;
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  }
  const LaneKeys keys = lane_keys(lane);
  const uint32_t lane_base = compact_lane_base(lane);

  uint32_t r0 = 0, k = 0;
  uint32_t st[NCH];
  RagBlock gn[NCH];  // the next round's chains
  while (true) {
    // 2. the next round's descriptors (offsets, lengths, headers, trailers:
    //    dependent scalar loads) fetched while this round's rows are in
    //    flight. Row 0: start every chain (fix-ups) or continue it. Idle
    //    chains walk zeros and store nothing.
    if (k == 0) RagRound<NCH, R>::fetch(gn, a, src, start, n, r0 + W * NCH, wave, W);
#pragma unroll
    for (int c = 0; c < NCH; ++c)
      if (rd.g[c].e() != 0) rd.realign(c, lane);
    if (k == 0) {
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const uint32_t s0l = rd.g[c].s0l(), sh = 8u * rd.g[c].delta();
        uint32_t x = rd.w[c][0];
        x = lane < s0l ? 0u : x;
        x = lane == s0l ? (x & (0xffffffffu << sh)) ^ (rd.g[c].s0 << sh) : x;
        x = lane == s0l + 1u ? x ^ rd.g[c].spill() : x;
        st[c] = x;
        // the spill of a first word in lane 63 lands in row 1, lane 0
        rd.w[c][1] = (s0l == 63u && lane == 0) ? rd.w[c][1] ^ rd.g[c].spill() : rd.w[c][1];
      }
    } else {
#pragma unroll
      for (int c = 0; c < NCH; ++c) st[c] = row_step_c(lds, st[c], rd.w[c][0], keys);
    }
    // 3. rows 1.. : all chains interleaved up to the shortest, then the rest
    uint32_t nrow[NCH];
    uint32_t nab = R;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const uint32_t rows = rd.g[c].kind == kRagRows ? rd.g[c].rows() : 0u;
      nrow[c] = rows > k * R ? min(static_cast<uint32_t>(R), rows - k * R) : 0u;
      nab = min(nab, nrow[c]);
    }
#pragma unroll
    for (int j = 1; j < R; ++j) {
      if (static_cast<uint32_t>(j) < nab) {
#pragma unroll
        for (int c = 0; c < NCH; ++c) st[c] = row_step_c(lds, st[c], rd.w[c][j], keys);
      }
    }
    // (row-major: the chains still running stay interleaved)
#pragma unroll
    for (int j = 1; j < R; ++j) {
      const uint32_t u = static_cast<uint32_t>(j);
      if (u >= nab) {
#pragma unroll
        for (int c = 0; c < NCH; ++c)
          if (u < nrow[c]) st[c] = row_step_c(lds, st[c], rd.w[c][j], keys);
      }
    }
    // 4. chains whose last chunk this was; tiny blocks at the round's end
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      if (nrow[c] > 0 && rd.g[c].rows() <= (k + 1) * R) {
        const uint32_t crc = wave_xor_dpp(lane_end_shift_c(lds, st[c], lane_base)) ^ 0xffffffffu;
        if (src.trailer(a)) rd.g[c].expected = rd.expected(c);
        src.store(a, rd.blk[c], rd.g[c], crc);
      }
    }
    // 5. next chunk of this round, or the next round
    if (++k == rd.nchunks) {
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        if (rd.g[c].kind == kRagTiny) {
          if (src.trailer(a)) rd.g[c].expected = rd.expected(c);
          src.store(a, rd.blk[c], rd.g[c], rag_tiny(rd.g[c]));
        }
        if (rd.g[c].kind == kRagSkip && lane == 0) lds[kFlag] = 1;
      }
      r0 += W * NCH;
      if (r0 >= n) break;
      rd.adopt(gn, start, r0, wave, W, src.trailer(a));
      k = 0;
    }
    rd.issue(k, lane);
  }

  // 6. Blocks over kLongBytes in this run (rare)
  ragged_long_pass<W>(a, zpow, lds, start, n, keys, lane_base, src);
}

}  // namespace
}  // namespace lvkv

#endif  // LVKV_CRC32C_RAGGED_BODY_H_
