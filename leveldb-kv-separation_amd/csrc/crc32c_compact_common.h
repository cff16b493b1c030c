// The compact 64 KiB LDS image shared by crc32c_compact.hip (uniform layout,
// long blocks, SST index/metaindex) and crc32c_ragged.hip (general layout):
// layout, row step, lane end shift and the in-kernel builders.
//
// Row tables: ds_read_b32 banks are (addr/4) mod 32 per 32-lane half-wave.
// Instead of 32 copies of each table (lane l -> copy l), lane l looks up, in
// its p-th lookup of a row step, byte t = (l + p) & 3 of the state in table t,
// copy c = (l >> 2) & 7. Over one half-wave the pairs (t, c) are all 32
// distinct, and copy c of table t sits in bank 8t + c of every 256-byte bank
// row, so each lookup instruction is conflict-free with 8 copies per table:
//
//   LDS row b (256 B), bytes [0, 128):   T_t[b] copy c at 32t + 4c
//   LDS row r (256 B), bytes [128, 256): lane nibble table r>>1 = k*16 + nib,
//                                        lane s (r & 1 = s >> 5) at 128 + 4(s & 31)
//
// The address of a lookup is one v_perm_b32 with a per-lane selector:
// {kpack.byte[p], S.byte[t], 0, 0} = S.byte[t] * 256 + 32t + 4c, where kpack
// holds 32t_p + 4c for p = 0..3. XOR order does not matter, so lane l's four
// lookups still cover the four bytes of its state.
#ifndef LVKV_CRC32C_COMPACT_COMMON_H_
#define LVKV_CRC32C_COMPACT_COMMON_H_

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_device_common.h"
#include "crc32c_uniform_common.h"
#include "lvkv_kernel_args.h"

namespace lvkv {

constexpr uint32_t kCompactLdsBytes = 64 * 1024;
// Segment of a long block walked by one wave (workgroup_crc).
constexpr uint64_t kLongSeg = 16 * 1024;

namespace {

struct LaneKeys {
  uint32_t kpack;   // byte p = 32 * t_p + 4 * c
  uint32_t sel[4];  // v_perm selectors {kpack.byte[p], S.byte[t_p], 0, 0}
};

__device__ __forceinline__ LaneKeys lane_keys(uint32_t lane) {
  LaneKeys k;
  const uint32_t c = (lane >> 2) & 7u;
  k.kpack = 0;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const uint32_t t = (lane + static_cast<uint32_t>(p)) & 3u;
    k.kpack |= (32u * t + 4u * c) << (8 * p);
    k.sel[p] = 0x0C0C0000u | ((4u + t) << 8) | static_cast<uint32_t>(p);
  }
  return k;
}

// Byte offset of lane s's nibble-table column in the image.
__device__ __forceinline__ uint32_t compact_lane_base(uint32_t lane) {
  return (lane >> 5) * 256u + 128u + (lane & 31u) * 4u;
}

// S -> Z_256(S) ^ w on the compact image.
__device__ __forceinline__ uint32_t row_step_c(const uint32_t* lds, uint32_t s, uint32_t w,
                                               const LaneKeys& k) {
  const uint32_t a0 = __builtin_amdgcn_perm(s, k.kpack, k.sel[0]);
  const uint32_t a1 = __builtin_amdgcn_perm(s, k.kpack, k.sel[1]);
  const uint32_t a2 = __builtin_amdgcn_perm(s, k.kpack, k.sel[2]);
  const uint32_t a3 = __builtin_amdgcn_perm(s, k.kpack, k.sel[3]);
  const uint32_t x = xor3(lds_ld(lds, a0), lds_ld(lds, a1), w);
  return xor3(x, lds_ld(lds, a2), lds_ld(lds, a3));
}

// S -> Z_{256-4s}(S) for this lane s (eight lane-private nibble lookups).
__device__ __forceinline__ uint32_t lane_end_shift_c(const uint32_t* lds, uint32_t s,
                                                     uint32_t lane_base) {
  uint32_t r = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint32_t nib = (s >> (4 * k)) & 15u;
    r ^= lds_ld(lds, (lane_base | (nib << 9)) + 8192u * k);
  }
  return r;
}

// Row image entries from the Z_256 tables in HBM (zpow set j = 8): 2048
// 16-byte slots q -> row b = q >> 3, table t = (q >> 1) & 3, copies 4h..4h+3
// with h = q & 1. Loaded in load(), written in store() (the caller issues
// other loads in between).
template <int kThreads, int J = 8>
struct RowTabStage {
  static constexpr int kIters = 2048 / kThreads;
  uint32_t v[kIters];

  __device__ __forceinline__ void load(const uint32_t* zpow, uint32_t tid) {
    const uint32_t* z256 = zpow + static_cast<uint32_t>(J) * 1024u;  // Z_{2^J}
#pragma unroll
    for (int it = 0; it < kIters; ++it) {
      const uint32_t q = tid + static_cast<uint32_t>(kThreads * it);
      v[it] = z256[((q >> 1) & 3u) * 256u + (q >> 3)];
    }
  }
  __device__ __forceinline__ void store(uint32_t* lds, uint32_t tid) const {
#pragma unroll
    for (int it = 0; it < kIters; ++it) {
      const uint32_t q = tid + static_cast<uint32_t>(kThreads * it);
      *reinterpret_cast<uint4*>(reinterpret_cast<char*>(lds) + (q >> 3) * 256u + (q & 7u) * 16u) =
          make_uint4(v[it], v[it], v[it], v[it]);
    }
  }
};

// Lane tables generated in-kernel: wave w owns nibble position k = w % 8
// (and, with 16 waves, nibbles 8 (w / 8) .. +7), loads the 4 columns of
// Z_{256-4s} it needs (lane_cols[(k*64 + s)*4 + j], one 16-byte load per
// lane), and writes its entries in Gray-code order, one xor each. For a fixed
// (k, nib) the 64 lanes write two contiguous 128-byte half rows:
// conflict-free ds_write_b32.
template <int W>
struct LaneTabGen {
  static constexpr int kNibs = 16 * 8 / W;  // entries per lane
  uint32_t col[4];

  __device__ __forceinline__ void load(const uint32_t* lane_cols, uint32_t wave, uint32_t lane) {
    const uint32_t k = wave & 7u;
    const uint4 v = *reinterpret_cast<const uint4*>(lane_cols + (k * 64u + lane) * 4u);
    col[0] = v.x;
    col[1] = v.y;
    col[2] = v.z;
    col[3] = v.w;
  }
  __device__ __forceinline__ void store(uint32_t* lds, uint32_t wave, uint32_t lane) const {
    const uint32_t k = wave & 7u;
    const uint32_t nib0 = (W == 16) ? (wave >> 3) * 8u : 0u;
    char* base = reinterpret_cast<char*>(lds) + (lane >> 5) * 256u + 128u + (lane & 31u) * 4u +
                 (k * 16u + nib0) * 512u;
    uint32_t e = 0;
    if (W == 16 && nib0) e = col[3];  // entry nib0 = 8
#pragma unroll
    for (int i = 0; i < kNibs; ++i) {
      if (i) e ^= col[__builtin_ctz(i)];
      const int g = i ^ (i >> 1);  // Gray code: nib = nib0 + g
      *reinterpret_cast<uint32_t*>(base + g * 512) = e;
    }
  }
};

// The compact image for a workgroup of W waves: row tables from the Z_256
// set of zpow, lane tables generated from lane_cols; ends with a barrier.
template <int W>
__device__ __forceinline__ void build_compact_image(uint32_t* lds, const uint32_t* zpow,
                                                    const uint32_t* lane_cols, uint32_t tid,
                                                    uint32_t wave, uint32_t lane) {
  RowTabStage<64 * W> rt;
  LaneTabGen<W> lg;
  rt.load(zpow, tid);
  lg.load(lane_cols, wave, lane);
  rt.store(lds, tid);
  lg.store(lds, wave, lane);
  __syncthreads();
}

// ---- long blocks: one workgroup per block -------------------------------

__device__ __forceinline__ uint32_t zshift_g(const uint32_t* zpow, uint32_t v, uint64_t n) {
  while (n) {
    const uint32_t j = __builtin_ctzll(n);
    const uint32_t* t = zpow + j * 1024u;
    v = t[v & 255u] ^ t[256u + ((v >> 8) & 255u)] ^ t[512u + ((v >> 16) & 255u)] ^
        t[768u + (v >> 24)];
    n &= n - 1;
  }
  return v;
}

// Register after [s, e) (e 4-byte aligned, e - s <= kLongSeg) from state
// init ^ ~0: the end-aligned row walk of the uniform kernels, 16-row chunks,
// the next chunk's loads in flight while one is walked.
__device__ __forceinline__ uint32_t segment_register(const uint32_t* lds, uint64_t s, uint64_t e,
                                                    uint32_t init,
                                     const LaneKeys& keys, uint32_t lane, uint32_t lane_base) {
  const uint32_t len = static_cast<uint32_t>(e - s);
  UniGeo g;
  const uint32_t q = (len + 3u) >> 2;
  g.rows = (q + 63u) >> 6;
  g.delta = 4u * q - len;
  g.s0l = 64u * g.rows - q;
  g.s0 = init ^ 0xffffffffu;
  g.spill = g.delta ? (g.s0 >> (32u - 8u * g.delta)) : 0u;
  g.nrec = 4u * q;
  g.vb0 = -4 * static_cast<int32_t>(g.s0l);
  const uint64_t b4 = e - 4ull * q;
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(b4));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(b4 >> 32));
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<void*>((static_cast<uint64_t>(hi) << 32) | lo), 0,
      static_cast<int>(g.nrec), kBufferDword3);
  const int32_t vo = g.vb0 + 4 * static_cast<int32_t>(lane);
  int32_t vo1 = vo + kRowBytes;
  asm volatile("" : "+v"(vo1));
  const uint32_t nchunks = (g.rows + kRowsPerChunk - 1) / kRowsPerChunk;
  uint32_t buf[2][kRowsPerChunk];
  auto issue = [&](uint32_t (&b)[kRowsPerChunk], uint32_t c) {
#pragma unroll
    for (int j = 0; j < kRowsPerChunk; ++j) {
      const int32_t row = static_cast<int32_t>(c) * kRowsPerChunk + j;
      b[j] = row == 0 ? __builtin_amdgcn_raw_buffer_load_b32(r, vo, 0, kUniCachePolicy)
                      : __builtin_amdgcn_raw_buffer_load_b32(r, vo1 + 256 * (row - 1), 0,
                                                             kUniCachePolicy);
    }
  };
  uint32_t st = 0;
  issue(buf[0], 0);
  for (uint32_t c = 0; c < nchunks; c += 2) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint32_t cc = c + h;
      if (cc < nchunks) {
        if (cc + 1 < nchunks) issue(buf[h ^ 1], cc + 1);
        uint32_t(&b)[kRowsPerChunk] = buf[h];
        if (cc == 0) {
          fix_first_chunk(b, g);
          st = b[0];
        } else {
          st = row_step_c(lds, st, b[0], keys);
        }
        const uint32_t nrow = min(static_cast<uint32_t>(kRowsPerChunk), g.rows - cc * kRowsPerChunk);
#pragma unroll
        for (int j = 1; j < kRowsPerChunk; ++j)
          if (static_cast<uint32_t>(j) < nrow) st = row_step_c(lds, st, b[j], keys);
      }
    }
  }
  return wave_xor_dpp(lane_end_shift_c(lds, st, lane_base));
}

// v -> Z_{2^j}(v) with zpow set j (one step of four lookups).
__device__ __forceinline__ uint32_t zstep_g(const uint32_t* t, uint32_t v) {
  return t[v & 255u] ^ t[256u + ((v >> 8) & 255u)] ^ t[512u + ((v >> 16) & 255u)] ^
         t[768u + (v >> 24)];
}

// CRC32C of [start, end) from `init` by the whole workgroup: SEG-byte
// segments on 4-byte boundaries, wave w of W takes segments w, w + W, ... and
// folds them Horner-style, acc <- Z_{W * SEG}(acc) ^ reg (one zpow set, since
// W * SEG is a power of two; only the batch's last segment and the final
// shift to the last 4-byte boundary are variable, Z_n as a product of zpow
// sets). Thread 0 combines the waves' accumulators, feeds the 0-3 tail bytes
// through Z_1 and returns the CRC (other threads: undefined). Two barriers;
// every thread of the workgroup must call it.
template <int W, uint64_t SEG = kLongSeg>
__device__ uint32_t workgroup_crc(const uint32_t* lds, uint32_t* acc_slots, uint64_t start,
                                  uint64_t end, uint32_t init, const LaneKeys& keys,
                                  uint32_t tid, uint32_t wave, uint32_t lane, uint32_t lane_base,
                                  const uint32_t* zpow) {
  constexpr uint64_t kLongSeg = SEG;
  constexpr uint64_t kStride = W * kLongSeg;
  static_assert((kStride & (kStride - 1)) == 0 && kStride < (uint64_t{1} << kZPowCount),
                "W * SEG must be a power of two");
  const uint32_t* zstride = zpow + static_cast<uint32_t>(__builtin_ctzll(kStride)) * 1024u;
  const uint64_t e4 = end & ~uint64_t{3};
  const uint64_t a4 = start & ~uint64_t{3};
  const uint32_t m = e4 > start ? static_cast<uint32_t>((e4 - a4 + kLongSeg - 1) / kLongSeg) : 0u;
  uint32_t acc = 0;
  uint64_t at = 0;  // the boundary acc is the register at (0: nothing yet)
  for (uint32_t k = wave; k < m; k += W) {
    const uint64_t s = k == 0 ? start : a4 + k * kLongSeg;
    const uint64_t e = min(a4 + (k + 1) * kLongSeg, e4);
    const uint32_t reg =
        segment_register(lds, s, e, k == 0 ? init : 0xffffffffu, keys, lane, lane_base);
    if (at != 0) acc = e - at == kStride ? zstep_g(zstride, acc) : zshift_g(zpow, acc, e - at);
    acc ^= reg;
    at = e;
  }
  if (at != 0) acc = zshift_g(zpow, acc, e4 - at);
  if (lane == 0) acc_slots[wave] = acc;
  __syncthreads();
  uint32_t crc = 0;
  if (tid == 0) {
    // m == 0 (fewer than 4 bytes up to a boundary): the init state is the
    // register, the bytes all go through the tail step
    uint32_t reg = m ? 0u : init ^ 0xffffffffu;
#pragma unroll
    for (int w = 0; w < W; ++w) reg ^= acc_slots[w];
    for (uint64_t p = m ? e4 : start; p < end; ++p)  // tail bytes: Z_1 = the byte table
      reg = zpow[(reg ^ *reinterpret_cast<const uint8_t*>(p)) & 255u] ^ (reg >> 8);
    crc = reg ^ 0xffffffffu;
  }
  __syncthreads();
  return crc;
}

// ---- one block over a group of waves, constant shifts in registers ------

// Columns of Z_{c * 2^log2seg} (lvkv_tables.h build_zmul_columns; they
// follow zpow in the device tables).
__device__ __forceinline__ const uint32_t* zmul_cols(const uint32_t* zpow, uint32_t log2seg,
                                                     uint32_t c) {
  return zpow + kZPowDwords + ((log2seg - kZMulLog0) * kZMulMaxC + c - 1u) * 32u;
}

// Z(v) for a wave-uniform v and an operator given by its 32 columns: scalar
// loads of the (never written) columns and 32 conditional xors, no chain of
// dependent table lookups.
__device__ __forceinline__ uint32_t apply_cols(const uint32_t* cols, uint32_t v) {
  uint32_t r = 0;
#pragma unroll
  for (int b = 0; b < 32; ++b) r ^= ((v >> b) & 1u) ? sload_u32(cols, static_cast<uint32_t>(b)) : 0u;
  return r;
}

// The same with the columns held one per lane: lanes 32 h + b hold column b
// of operator h; v wave-uniform; one DPP xor-reduction.
__device__ __forceinline__ uint32_t apply_lane_cols(uint32_t colv, uint32_t v, uint32_t h,
                                                    uint32_t lane) {
  const bool on = (lane >> 5) == h && ((v >> (lane & 31u)) & 1u);
  return wave_xor_dpp(on ? colv : 0u);
}

// Bitwise register update over the n (< 4) little-endian bytes of `bytes`.
__device__ __forceinline__ uint32_t crc_bytes_bitwise(uint32_t reg, uint32_t bytes, uint32_t n) {
  for (uint32_t i = 0; i < n; ++i) {
    reg ^= (bytes >> (8u * i)) & 0xffu;
#pragma unroll
    for (int k = 0; k < 8; ++k) reg = (reg >> 1) ^ (kCastagnoliReflected & (0u - (reg & 1u)));
  }
  return reg;
}

// Smallest segment (log2, 2^10 .. 2^15 bytes) that gives each of GW waves at
// most one segment of a `len`-byte block, where that is possible.
__device__ __forceinline__ uint32_t group_log2seg(uint64_t len, uint32_t GW) {
  uint32_t l = 10;
  while (l < 15 && (uint64_t{GW} << l) < len) ++l;
  return l;
}

// This wave's share of the register of [start, end) from `init`, for wave gw
// of a group of GW waves. Segments of 2^log2seg bytes are cut back from
// e4 = floor4(end): segment j (j = 0 the last) is [max(start, e4 - (j+1)S),
// e4 - jS). Wave gw takes j = gw, gw + GW, ..., front to back, folding
// acc <- Z_{GW S}(acc) ^ reg, and finally shifts acc by Z_{gw S} to e4: every
// shift is a constant operator (apply_cols). The xor of the group's shares is
// the register at e4; group_crc_finish adds the 0-3 bytes after it.
__device__ inline uint32_t group_crc_part(const uint32_t* lds, uint64_t start, uint64_t end,
                                   uint32_t init, uint32_t gw, uint32_t GW, uint32_t log2seg,
                                   const LaneKeys& keys, uint32_t lane, uint32_t lane_base,
                                   const uint32_t* zpow) {
  const uint64_t seg = uint64_t{1} << log2seg;
  const uint64_t e4 = end & ~uint64_t{3};
  if (e4 <= start) return 0u;
  const uint32_t m = static_cast<uint32_t>((e4 - start + seg - 1) >> log2seg);
  if (gw >= m) return 0u;
  const uint32_t jmax = gw + ((m - 1u - gw) / GW) * GW;
  // both operators' columns, loaded before the walks: lanes [0, 32) hold
  // Z_{GW S}, lanes [32, 64) Z_{gw S}
  const uint32_t colv = lane < 32u ? zmul_cols(zpow, log2seg, GW)[lane]
                                   : (gw ? zmul_cols(zpow, log2seg, gw)[lane - 32u] : 0u);
  uint32_t acc = 0;
  for (uint32_t j = jmax;; j -= GW) {
    const uint64_t e = e4 - uint64_t{j} * seg;
    const bool front = j == m - 1u;
    const uint64_t s = front ? start : e - seg;
    const uint32_t reg =
        segment_register(lds, s, e, front ? init : 0xffffffffu, keys, lane, lane_base);
    acc = (j == jmax ? 0u : apply_lane_cols(colv, acc, 0, lane)) ^ reg;
    if (j < GW) break;
  }
  return gw ? apply_lane_cols(colv, acc, 1, lane) : acc;
}

// CRC of [start, end) from the xor of the group's shares and `tail`, the
// little-endian bytes from max(start, floor4(end)) to end (fewer than 4).
__device__ __forceinline__ uint32_t group_crc_finish(uint32_t parts, uint64_t start, uint64_t end,
                                                     uint32_t init, uint32_t tail) {
  const uint64_t e4 = end & ~uint64_t{3};
  const bool none = e4 <= start;  // fewer than 4 bytes up to a boundary
  const uint32_t reg = none ? init ^ 0xffffffffu : parts;
  return crc_bytes_bitwise(reg, tail, static_cast<uint32_t>(end - (none ? start : e4))) ^
         0xffffffffu;
}

// The little-endian bytes [max(start, floor4(end)), end) (the `tail` above).
__device__ __forceinline__ uint32_t group_crc_tail(uint64_t start, uint64_t end) {
  const uint64_t e4 = end & ~uint64_t{3};
  const uint64_t from = e4 <= start ? start : e4;
  uint32_t v = 0;
  for (uint64_t p = from; p < end; ++p)
    v |= static_cast<uint32_t>(*reinterpret_cast<const uint8_t*>(p)) << (8u * (p - from));
  return v;
}

}  // namespace
}  // namespace lvkv

#endif  // LVKV_CRC32C_COMPACT_COMMON_H_
