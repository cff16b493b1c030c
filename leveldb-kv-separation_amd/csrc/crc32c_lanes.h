// Lane-serial general-layout batch CRC32C for SHORT blocks (WAL records,
// small values: tens of bytes to a few KiB): every LANE checksums one block
// on its own, with the four-stream stride of the reference's Extend
// (util/crc32c.cc:293-366: four interleaved 4-byte streams over 16-byte
// swaths, each stream advanced by the 16-byte operator, combined at the end)
// instead of a whole wave walking one block row by row.
//
// Why: the row walk (crc32c_ragged_body.h) spends a wave's whole fixed cost
// per block — descriptor fetch, row-0 fix-ups, the eight-lookup lane end
// shift and a six-step reduction — and a 1 KiB record is only four rows, so
// 62,000 records of 0-2000 B reached 0.2-0.3 of 8 TB/s whatever the shape.
// Here 64 blocks of a wave cost 64 lanes' work in parallel, there is no
// reduction, and the fixed cost is one vector load of the descriptors.
//
// Per lane, for a block [p, p + n) from state l = init ^ ~0:
//   * the 0-3 bytes up to p's 4-byte boundary through the byte table Z_1;
//   * the 16-byte swaths: s_i (i = 0..3) start as the first swath's words
//     (s_0 ^= l) and advance s_i <- Z_16(s_i) ^ word_i; then
//     l = Z_16(s_0) ^ Z_12(s_1) ^ Z_8(s_2) ^ Z_4(s_3) (word i of the last
//     swath is followed by 12 - 4i more bytes);
//   * the 0-3 words left: l <- Z_4(l ^ w); the 0-3 bytes left: Z_1.
// Z_16 and Z_4 are the two halves of each 256-byte LDS row, eight copies per
// byte table, read conflict-free with the compact image's per-lane selectors
// (crc32c_compact_common.h lane_keys); Z_8 and Z_1 (a handful of lookups per
// block) one copy each.
//
// Loads: every swath is a 16-byte load at a 4-byte aligned address inside
// the block; a lane keeps kLanePf swaths in flight. All loads are issued
// unconditionally (a lane past its block re-reads its block's first swath),
// so the compiler's vmcnt waits stay counted. Nothing outside
// [floor4(p), ceil4(p + n)) is read.
//
// Blocks whose covered length exceeds a.long_split are left to the whole
// workgroup at the end of the run (ragged_long_pass on the compact image,
// built then).
#ifndef LVKV_CRC32C_LANES_H_
#define LVKV_CRC32C_LANES_H_

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_compact_common.h"
#include "crc32c_device_common.h"
#include "crc32c_ragged_body.h"
#include "lvkv_crc32c.h"
#include "lvkv_kernel_args.h"

namespace lvkv {

constexpr uint32_t kLaneZ8 = 64 * 1024;          // Z_8 byte tables (4 KiB)
constexpr uint32_t kLaneZ1 = kLaneZ8 + 4096;     // Z_1 byte table (1 KiB)
constexpr uint32_t kLaneFlag = kLaneZ1 + 1024;   // a block was left to the long pass
constexpr uint32_t kLaneImageBytes = kLaneFlag + 16;
constexpr int kLanePf = 8;                       // swaths in flight per lane
// Blocks longer than this leave the lane walk for the workgroup's: one lane
// walking 4 KiB is 256 dependent swath steps while its wave's other lanes
// idle.
constexpr uint32_t kLaneLongBytes = 4096;

// LDS bytes of a W-wave lane-serial workgroup: its image, or the ragged
// layout the long pass uses (whichever is larger).
template <int W>
constexpr uint32_t lanes_lds_bytes() {
  return kLaneImageBytes > RagLds<W>::kDwords * 4 ? kLaneImageBytes : RagLds<W>::kDwords * 4;
}

namespace {

typedef uint32_t LaneU32x4 __attribute__((ext_vector_type(4)));
// Global-address-space views: flat loads would count in lgkmcnt too and
// make every wait on an LDS lookup wait on them.
typedef __attribute__((address_space(1))) const LaneU32x4 GlobalU32x4;
typedef __attribute__((address_space(1))) const uint32_t GlobalU32;
typedef __attribute__((address_space(1))) const uint64_t GlobalU64;

__device__ __forceinline__ uint32_t gld32(uint64_t addr) {
  return *reinterpret_cast<GlobalU32*>(addr);
}

// The image: zpow sets j = 4 (Z_16) and 2 (Z_4) into the two row halves, 8
// copies each (2048 16-byte slots per half: row b = q >> 3, table
// t = (q >> 1) & 3, copies 4h .. 4h + 3 with h = q & 1), set 3 (Z_8) and
// set 0's first table (Z_1) once. Ends with a barrier.
template <int W>
__device__ __forceinline__ void build_lane_image(uint32_t* lds, const uint32_t* zpow,
                                                 uint32_t tid) {
  constexpr uint32_t kThreads = 64 * W;
  const uint32_t* z16 = zpow + 4u * 1024u;
  const uint32_t* z4 = zpow + 2u * 1024u;
  const uint32_t* z8 = zpow + 3u * 1024u;
  char* base = reinterpret_cast<char*>(lds);
  for (uint32_t q = tid; q < 2048u; q += kThreads) {
    const uint32_t src = ((q >> 1) & 3u) * 256u + (q >> 3);
    const uint32_t a = z16[src], b = z4[src];
    const uint32_t at = (q >> 3) * 256u + (q & 7u) * 16u;
    *reinterpret_cast<uint4*>(base + at) = make_uint4(a, a, a, a);
    *reinterpret_cast<uint4*>(base + at + 128u) = make_uint4(b, b, b, b);
  }
  for (uint32_t i = tid; i < 1024u; i += kThreads)
    *reinterpret_cast<uint32_t*>(base + kLaneZ8 + 4u * i) = z8[i];
  for (uint32_t i = tid; i < 256u; i += kThreads)
    *reinterpret_cast<uint32_t*>(base + kLaneZ1 + 4u * i) = zpow[i];
  if (tid == 0) *reinterpret_cast<uint32_t*>(base + kLaneFlag) = 0;
  __syncthreads();
}

// The Z_4 half's selectors: the Z_16 ones + 128 in every byte of kpack.
__device__ __forceinline__ LaneKeys lane_keys_hi(uint32_t lane) {
  LaneKeys k = lane_keys(lane);
  k.kpack += 0x80808080u;
  return k;
}

__device__ __forceinline__ uint32_t lz8(const uint32_t* lds, uint32_t v) {
  const char* t = reinterpret_cast<const char*>(lds) + kLaneZ8;
  return xor3(*reinterpret_cast<const uint32_t*>(t + 4u * (v & 255u)),
              *reinterpret_cast<const uint32_t*>(t + 1024u + 4u * ((v >> 8) & 255u)),
              *reinterpret_cast<const uint32_t*>(t + 2048u + 4u * ((v >> 16) & 255u))) ^
         *reinterpret_cast<const uint32_t*>(t + 3072u + 4u * (v >> 24));
}

// One byte b through the register: Z_1(l ^ b), the reference's byte step.
__device__ __forceinline__ uint32_t lz1(const uint32_t* lds, uint32_t l, uint32_t b) {
  const char* t = reinterpret_cast<const char*>(lds) + kLaneZ1;
  return *reinterpret_cast<const uint32_t*>(t + 4u * ((l ^ b) & 255u)) ^ (l >> 8);
}

// This lane's block: covered range, initial register, the stored CRC the
// verify modes compare with, and whether it is left to the long pass.
struct LaneBlock {
  uint64_t ptr;
  uint32_t len;
  uint32_t s0;        // init ^ ~0
  uint32_t expected;  // verify modes: unmasked stored CRC
  bool live, skip;
};

// Little-endian n (1..4) bytes at any address, from the aligned dwords that
// hold [addr, addr + n) and no others (higher bytes: whatever those dwords
// hold).
__device__ __forceinline__ uint32_t ld_le(uint64_t addr, uint32_t n) {
  const uint64_t d = addr & ~uint64_t{3};
  const uint32_t sh = static_cast<uint32_t>(addr & 3u);
  const uint32_t lo = gld32(d);
  const uint32_t hi = sh + n > 4u ? gld32(d + 4) : 0u;
  return __builtin_amdgcn_alignbyte(hi, lo, sh);
}

// Block b's descriptor by mode (rag_block's semantics, one lane).
__device__ __forceinline__ LaneBlock lane_block(const KernelArgs& a, uint32_t b, bool live) {
  LaneBlock g;
  g.ptr = 0;
  g.len = 0;
  g.s0 = 0xffffffffu;
  g.expected = 0;
  g.live = live;
  g.skip = false;
  if (!live) return g;
  const uint64_t base = reinterpret_cast<uint64_t>(a.base);
  uint64_t off;
  uint32_t len, init = a.init;
  const bool log = a.mode == kModeLogVerify || a.mode == kModeLogFill || a.mode == kModeLogStaged;
  if (log) {
    // [masked crc u32][len u16][type u8]; the CRC covers type + payload
    // (db/log_reader.cc:217-221, 243-247)
    const uint64_t hoff = reinterpret_cast<GlobalU64*>(reinterpret_cast<uint64_t>(a.offsets))[b];
    if (a.mode != kModeLogFill) g.expected = crc_unmask(ld_le(base + hoff, 4));
    len = 1u + (ld_le(base + hoff + 4, 2) & 0xffffu);
    off = hoff + 6;
    init = 0;
  } else {
    if (a.offsets == nullptr) {
      off = static_cast<uint64_t>(b) * a.stride;
      len = a.length;
    } else {
      off = reinterpret_cast<GlobalU64*>(reinterpret_cast<uint64_t>(a.offsets))[b];
      len = reinterpret_cast<GlobalU32*>(reinterpret_cast<uint64_t>(a.lengths))[b];
    }
    if (a.inits != nullptr) init = reinterpret_cast<GlobalU32*>(reinterpret_cast<uint64_t>(a.inits))[b];
  }
  if (a.mode == kModeSstVerify || a.mode == kModeSstFill) {
    // contents n bytes + type byte; the masked CRC follows
    // (table/format.cc:92-94, table/table_builder.cc:199-203)
    len += 1;
    init = 0;
    if (a.mode == kModeSstVerify) g.expected = crc_unmask(ld_le(base + off + len, 4));
  }
  g.ptr = base + off;
  g.len = len;
  g.s0 = init ^ 0xffffffffu;
  g.skip = a.long_split != 0 && len > a.long_split;
  return g;
}

// This lane stores its block's result in the batch's mode (rag_store's
// semantics; kModeSstTable is not served here).
__device__ __forceinline__ void lane_store(const KernelArgs& a, uint32_t b, const LaneBlock& g,
                                           uint32_t crc) {
  if (a.mode == kModeCompute) {
    a.out_crc[b] = a.mask ? crc_mask(crc) : crc;
  } else if (a.mode == kModeSstFill || a.mode == kModeLogFill) {
    uint8_t* dst = reinterpret_cast<uint8_t*>(a.mode == kModeSstFill ? g.ptr + g.len : g.ptr - 6);
    const uint32_t m = crc_mask(crc);
#pragma unroll
    for (int k = 0; k < 4; ++k) dst[k] = static_cast<uint8_t>(m >> (8 * k));
    if (a.out_crc != nullptr) a.out_crc[b] = crc;
  } else {
    a.out_crc[b] = crc;
    if (a.out_status != nullptr) a.out_status[b] = crc != g.expected ? 1 : 0;
    if (a.mode == kModeLogStaged && crc != g.expected) {
      const uint64_t hoff = g.ptr - 6u - reinterpret_cast<uint64_t>(a.base);
      atomicMin(a.log_first_bad + (hoff >> 15), b);
    }
  }
}

// The four-stream walk of one block per lane (all lanes of the wave call
// it; `m_max` = the wave's largest swath count).
__device__ __forceinline__ uint32_t lane_crc(const uint32_t* lds, const LaneKeys& k16,
                                             const LaneKeys& k4, uint64_t p, uint32_t n,
                                             uint32_t l, bool active, const LaneU32x4* safe_ptr) {
  // 1. bytes up to the 4-byte boundary
  const uint32_t mis = static_cast<uint32_t>(p & 3u);
  const uint32_t hb = active ? min(n, (4u - mis) & 3u) : 0u;
  if (__builtin_amdgcn_readfirstlane(__ballot(hb != 0) != 0)) {
    const uint32_t w = hb ? gld32(p & ~uint64_t{3}) : 0u;
    for (uint32_t i = 0; i < 3u; ++i)
      if (i < hb) l = lz1(lds, l, (w >> (8u * (mis + i))) & 255u);
  }
  p += hb;
  n = active ? n - hb : 0u;
  // 2. 16-byte swaths, kLanePf in flight
  const uint32_t m = n >> 4;  // swaths
  uint32_t mmax = m;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) mmax = max(mmax, static_cast<uint32_t>(__shfl_xor(static_cast<int>(mmax), d, 64)));
  mmax = __builtin_amdgcn_readfirstlane(mmax);
  if (mmax != 0) {
    GlobalU32x4* q = reinterpret_cast<GlobalU32x4*>(p);  // 4-byte aligned
    // a lane without swath i re-reads its block's first one, or (no swath
    // at all: a short block, an idle lane) the 16 bytes at `safe_ptr`
    GlobalU32x4* safe = m ? q : reinterpret_cast<GlobalU32x4*>(reinterpret_cast<uint64_t>(safe_ptr));
    LaneU32x4 buf[kLanePf];
#pragma unroll
    for (int i = 0; i < kLanePf; ++i) {
      GlobalU32x4* src = static_cast<uint32_t>(i) < m ? q + i : safe;
      buf[i] = *src;
    }
    uint32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
    for (uint32_t base = 0; base < mmax; base += kLanePf) {
#pragma unroll
      for (int i = 0; i < kLanePf; ++i) {
        const uint32_t k = base + static_cast<uint32_t>(i);
        const LaneU32x4 d = buf[i];
        const uint32_t kn = k + kLanePf;
        buf[i] = *(kn < m ? q + kn : safe);
        const bool v = k < m;
        if (k == 0) {
          s0 = v ? d.x ^ l : 0u;
          s1 = v ? d.y : 0u;
          s2 = v ? d.z : 0u;
          s3 = v ? d.w : 0u;
        } else {
          const uint32_t t0 = row_step_c(lds, s0, d.x, k16), t1 = row_step_c(lds, s1, d.y, k16);
          const uint32_t t2 = row_step_c(lds, s2, d.z, k16), t3 = row_step_c(lds, s3, d.w, k16);
          s0 = v ? t0 : s0;
          s1 = v ? t1 : s1;
          s2 = v ? t2 : s2;
          s3 = v ? t3 : s3;
        }
      }
    }
    if (m) {
      // Z_16(s0) ^ Z_12(s1) ^ Z_8(s2) ^ Z_4(s3), Z_12 = Z_8 Z_4
      const uint32_t a0 = row_step_c(lds, s0, 0u, k16);
      const uint32_t a1 = lz8(lds, row_step_c(lds, s1, 0u, k4));
      const uint32_t a2 = lz8(lds, s2);
      const uint32_t a3 = row_step_c(lds, s3, 0u, k4);
      l = xor3(a0, a1, a2) ^ a3;
    }
    p += uint64_t{m} << 4;
    n -= m << 4;
  }
  // 3. words, then bytes
  for (uint32_t i = 0; i < 3u; ++i) {
    if (n >= 4u) {
      l = row_step_c(lds, l ^ gld32(p), 0u, k4);
      p += 4;
      n -= 4;
    }
  }
  if (n) {
    const uint32_t w = gld32(p);
    for (uint32_t i = 0; i < 3u; ++i)
      if (i < n) l = lz1(lds, l, (w >> (8u * i)) & 255u);
  }
  return l ^ 0xffffffffu;
}

// Workgroup `grp` of G walks its run of [0, total): rounds of 64 W blocks,
// one per lane. Every thread of the workgroup calls it.
template <int W>
__device__ __forceinline__ void lanes_run(const KernelArgs& a, const uint32_t* zpow,
                                          const uint32_t* lane_cols, uint32_t* lds,
                                          uint32_t grp, uint32_t G, uint32_t total) {
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = lane_id();
  const uint32_t per = total / G, extra = total % G;
  const uint32_t n = per + (grp < extra ? 1u : 0u);
  const uint32_t start = grp * per + min(grp, extra);
  if (n == 0) return;  // the whole workgroup
  build_lane_image<W>(lds, zpow, tid);
  const LaneKeys k16 = lane_keys(lane), k4 = lane_keys_hi(lane);
  bool skipped = false;
  for (uint32_t r0 = 0; r0 < n; r0 += 64u * W) {
    const uint32_t i = r0 + tid;
    const LaneBlock g = lane_block(a, start + i, i < n);
    const bool active = g.live && !g.skip;
    skipped |= g.live && g.skip;
    const uint32_t crc = lane_crc(lds, k16, k4, g.ptr, g.len, g.s0, active,
                                  reinterpret_cast<const LaneU32x4*>(zpow));
    if (active) lane_store(a, start + i, g, crc);
  }
  // blocks over long_split: the whole workgroup walks each (ragged_long_pass
  // on the compact image, built over this image)
  if (__ballot(skipped)) reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(lds) + kLaneFlag)[0] = 1;
  __syncthreads();
  if (reinterpret_cast<volatile uint32_t*>(reinterpret_cast<char*>(lds) + kLaneFlag)[0] == 0) return;
  __syncthreads();
  build_compact_image<W>(lds, zpow, lane_cols, tid, __builtin_amdgcn_readfirstlane(tid >> 6), lane);
  if (tid == 0) lds[RagLds<W>::kFlag] = 1;
  const LaneKeys keys = lane_keys(lane);
  ragged_long_pass<W>(a, zpow, lds, start, n, keys, compact_lane_base(lane));
}

}  // namespace
}  // namespace lvkv

#endif  // LVKV_CRC32C_LANES_H_
