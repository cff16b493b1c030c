// The grouped small-record walk (group_run): four records per wave at once,
// one per 16-lane row, for batches of short blocks (WAL records, small
// values) where the 64-lane walk (crc32c_ragged_body.h) spends a whole wave's
// end shift, reduction, store and scalar descriptor work on each ~1 KB
// record.
//
// Arithmetic as everywhere here, on 64-byte rows: record g of
// a chain is laid on its own grid of 4-byte words aligned to its END (q
// words, rows_g = ceil(q / 16) rows, s0l = 16 rows_g - q words of front
// padding), lane t of the group's 16-lane row holds grid word 16 r + t - s0l
// of row r, Horner over rows with Z_64 (row_step_c on the group image of
// crc32c_compact_common.h: Z_64 byte tables), lane end shift Z_{64-4t},
// xor over the 16 lanes (four DPP row ops: every lane of the row then holds
// the register). The four records of a chain start together at row 0 and
// each group's state is frozen once its own rows are done, so the row-0
// fix-ups (front padding, the initial state's injection and its spill) are
// at fixed places and the walk runs to the chain's longest record.
//
// Descriptors are loaded by one lane per record, lane 16 g + c for chain c
// of the wave's round (vector loads, the dependent header / trailer loads a
// round ahead), sorted by length so a chain's four records are alike, and
// reach the group's lanes by DPP row_newbcast:c. A chunk's rows come through
// one buffer resource per chain whose window is the chain's records cut to
// the chunk's rows, so a row past a record's end reads other bytes of the
// batch or zeros, never memory outside it (the state is frozen there); row
// 0's lanes before a record read through an offset past the window (zeros,
// no access). Records of any length are walked this way; records under 4
// bytes bit by bit in their desc lanes; chains whose records lie more than a
// buffer window apart walk one group per pass.
//
// Reference: util/crc32c.cc:276-377 (Extend), util/crc32c.h:20-38;
// db/log_reader.cc:243-247 and table/format.cc:92-99 (the verify modes),
// db/log_writer.cc:94-96 and table/table_builder.cc:199-203 (the fills).
#ifndef LVKV_CRC32C_GROUP_BODY_H_
#define LVKV_CRC32C_GROUP_BODY_H_

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_compact_common.h"
#include "crc32c_device_common.h"
#include "crc32c_ragged_body.h"
#include "lvkv_crc32c.h"
#include "lvkv_kernel_args.h"

namespace lvkv {
namespace {

constexpr uint32_t kGrpRowBytes = 64;     // one group row: 16 lanes x 4 B
constexpr uint32_t kGrpBad = 0x80000000u; // a buffer offset past every window
constexpr uint32_t kGrpSpanMax = 0x7fff0000u;  // a chain's window, bytes

enum : uint32_t { kGrpNone = 0, kGrpRows = 1, kGrpTiny = 2 };

template <int C>
__device__ __forceinline__ uint32_t row_bcast(uint32_t v) {  // row_newbcast:C
  return static_cast<uint32_t>(
      __builtin_amdgcn_mov_dpp(static_cast<int>(v), 0x150 + C, 0xF, 0xF, false));
}
__device__ __forceinline__ uint32_t row_rol1(uint32_t v) {  // lane t <- lane (t + 1) % 16
  return static_cast<uint32_t>(
      __builtin_amdgcn_mov_dpp(static_cast<int>(v), 0x12F, 0xF, 0xF, false));
}
// xor over the 16 lanes of each row, in every lane of the row
__device__ __forceinline__ uint32_t row_xor16(uint32_t v) {
  v ^= dpp32<0xB1>(v);   // quad_perm [1,0,3,2]
  v ^= dpp32<0x4E>(v);   // quad_perm [2,3,0,1]
  v ^= dpp32<0x141>(v);  // row_half_mirror
  v ^= dpp32<0x140>(v);  // row_mirror
  return v;
}

// row_newbcast:c for a chain index the unrolled loops make constant
__device__ __forceinline__ uint32_t row_bcast_c(uint32_t v, int c) {
  switch (c) {
    case 0: return row_bcast<0>(v);
    case 1: return row_bcast<1>(v);
    case 2: return row_bcast<2>(v);
    default: return row_bcast<3>(v);
  }
}

// Stage 1 of a record's descriptor (desc lanes): what the batch's arrays
// hold. Stage 2: the header (log modes) or stored trailer (SST verify) bytes,
// three dwords from the aligned dword holding the first byte.
struct GrpRaw {
  uint32_t off_lo, off_hi, len, init;
};
struct GrpHdr {
  uint32_t d0, d1, d2;
};

__device__ __forceinline__ bool grp_log(uint32_t mode) {
  return mode == kModeLogVerify || mode == kModeLogFill;
}
__device__ __forceinline__ bool grp_sst(uint32_t mode) {
  return mode == kModeSstVerify || mode == kModeSstFill;
}

__device__ __forceinline__ GrpRaw grp_stage1(const KernelArgs& a, uint32_t b, bool live) {
  // desc lanes of live records only (the others load nothing: a shared
  // dummy address would put every wave of the launch on one L2 line)
  GrpRaw r;
  r.off_lo = r.off_hi = r.len = 0;
  r.init = a.init;
  if (a.offsets == nullptr) {
    const uint64_t off = static_cast<uint64_t>(b) * a.stride;
    r.off_lo = static_cast<uint32_t>(off);
    r.off_hi = static_cast<uint32_t>(off >> 32);
    r.len = live ? a.length : 0u;
  } else if (live) {
    const uint64_t off = a.offsets[b];
    r.off_lo = static_cast<uint32_t>(off);
    r.off_hi = static_cast<uint32_t>(off >> 32);
    if (!grp_log(a.mode)) r.len = a.lengths[b];
  }
  if (a.inits != nullptr && live) r.init = a.inits[b];
  return r;
}

__device__ __forceinline__ GrpHdr grp_stage2(const KernelArgs& a, const GrpRaw& r, bool live) {
  GrpHdr h;
  h.d0 = h.d1 = h.d2 = 0;
  const bool log = grp_log(a.mode), trl = a.mode == kModeSstVerify;
  if ((log || trl) && live) {
    const uint64_t at = reinterpret_cast<uint64_t>(a.base) +
                        ((static_cast<uint64_t>(r.off_hi) << 32) | r.off_lo);
    // the 7-byte log header at the offset; the 4-byte stored trailer after
    // an SST block's n + 1 bytes (table/format.cc:92-94): the dwords holding
    // them, no byte after them
    const uint64_t p = log ? at : at + r.len + 1u;
    const uint32_t nbytes = log ? 7u : 4u;
    const uint64_t a4 = p & ~uint64_t{3};
    const uint32_t span = static_cast<uint32_t>(p & 3u) + nbytes;
    h.d0 = gload32(a4);
    h.d1 = gload32(span > 4u ? a4 + 4u : a4);
    h.d2 = gload32(span > 8u ? a4 + 8u : a4);
  }
  return h;
}

// A record as its desc lane holds it.
struct GrpRec {
  uint32_t ptr_lo, ptr_hi, len, s0, expected, idx, kind;
  __device__ __forceinline__ uint64_t ptr() const {
    return (static_cast<uint64_t>(ptr_hi) << 32) | ptr_lo;
  }
};

__device__ __forceinline__ uint32_t grp_le32(const GrpHdr& h, uint32_t sh, int word) {
  const uint64_t v = word == 0 ? ((static_cast<uint64_t>(h.d1) << 32) | h.d0)
                               : ((static_cast<uint64_t>(h.d2) << 32) | h.d1);
  return static_cast<uint32_t>(v >> sh);
}

__device__ __forceinline__ GrpRec grp_record(const KernelArgs& a, const GrpRaw& r, const GrpHdr& h,
                                             bool live, uint32_t idx) {
  GrpRec g;
  uint64_t ptr = reinterpret_cast<uint64_t>(a.base) +
                 ((static_cast<uint64_t>(r.off_hi) << 32) | r.off_lo);
  uint32_t len = r.len, init = r.init, expected = 0;
  if (grp_log(a.mode)) {
    // [masked crc u32][len u16][type u8]; the CRC covers type + payload
    // (db/log_reader.cc:217-221, 243-247)
    const uint32_t sh = static_cast<uint32_t>(ptr & 3u) * 8u;
    expected = crc_unmask(grp_le32(h, sh, 0));
    len = 1u + (grp_le32(h, sh, 1) & 0xffffu);
    ptr += 6u;
    init = 0;
  } else if (grp_sst(a.mode)) {
    len += 1u;  // contents + type byte (table/format.cc:92-94)
    init = 0;
    if (a.mode == kModeSstVerify)
      expected = crc_unmask(grp_le32(h, static_cast<uint32_t>((ptr + len) & 3u) * 8u, 0));
  }
  g.ptr_lo = static_cast<uint32_t>(ptr);
  g.ptr_hi = static_cast<uint32_t>(ptr >> 32);
  g.len = len;
  g.s0 = init ^ 0xffffffffu;
  g.expected = expected;
  g.idx = idx;
  g.kind = !live ? kGrpNone : len < 4u ? kGrpTiny : kGrpRows;
  return g;
}

// The result of a record, stored by its desc lane in the batch's mode (the
// vector form of rag_store's compute / verify / fill branches).
__device__ __forceinline__ void grp_store(const KernelArgs& a, const GrpRec& g, uint32_t crc) {
  const uint32_t b = g.idx;
  if (a.mode == kModeCompute) {
    a.out_crc[b] = a.mask ? crc_mask(crc) : crc;
  } else if (a.mode == kModeSstFill || a.mode == kModeLogFill) {
    uint8_t* dst = reinterpret_cast<uint8_t*>(a.mode == kModeSstFill ? g.ptr() + g.len : g.ptr() - 6u);
    const uint32_t m = crc_mask(crc);
#pragma unroll
    for (int k = 0; k < 4; ++k) dst[k] = static_cast<uint8_t>(m >> (8 * k));
    if (a.out_crc != nullptr) a.out_crc[b] = crc;
  } else {
    a.out_crc[b] = crc;
    if (a.out_status != nullptr) a.out_status[b] = crc != g.expected ? 1 : 0;
  }
}

// The wave-round's records sorted by covered length before they are dealt
// to the chains: chain c takes ranks 4c .. 4c + 3, so the four records of a
// chain are of similar length and the walk to the chain's longest wastes
// little (random 0-2000 B records: E[max of 4] is 1.6x the mean unsorted).
// Ranks from the 4 NCH desc lanes' keys (readlane, compares); each record's
// fields move to its new desc lane by ds_permute (a push: the other lanes
// send to themselves).
template <int NCH>
__device__ __forceinline__ GrpRec grp_sort(const GrpRec& rec, uint32_t lane, bool desc_lane) {
  const uint32_t key = rec.kind == kGrpRows ? rec.len : 0u;
  const uint32_t me = 4u * (lane & 15u) + (lane >> 4);  // this desc lane's slot
  uint32_t rank = 0;
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const uint32_t other = lane_u32(key, 16u * g + c);
      const uint32_t slot = 4u * c + g;
      rank += (other < key || (other == key && slot < me)) ? 1u : 0u;
    }
  // rank rho goes to desc lane 16 (rho % 4) + rho / 4
  const uint32_t dst = desc_lane ? 16u * (rank & 3u) + (rank >> 2) : lane;
  const int addr = static_cast<int>(4u * dst);
  GrpRec r;
  r.ptr_lo = static_cast<uint32_t>(__builtin_amdgcn_ds_permute(addr, static_cast<int>(rec.ptr_lo)));
  r.ptr_hi = static_cast<uint32_t>(__builtin_amdgcn_ds_permute(addr, static_cast<int>(rec.ptr_hi)));
  r.len = static_cast<uint32_t>(__builtin_amdgcn_ds_permute(addr, static_cast<int>(rec.len)));
  r.s0 = static_cast<uint32_t>(__builtin_amdgcn_ds_permute(addr, static_cast<int>(rec.s0)));
  r.expected = static_cast<uint32_t>(__builtin_amdgcn_ds_permute(addr, static_cast<int>(rec.expected)));
  r.idx = static_cast<uint32_t>(__builtin_amdgcn_ds_permute(addr, static_cast<int>(rec.idx)));
  r.kind = static_cast<uint32_t>(__builtin_amdgcn_ds_permute(addr, static_cast<int>(rec.kind)));
  return r;
}

// One chain of one wave-round as its lanes see it: their group's record.
struct GrpChain {
  uint32_t rows;   // the group's rows (0: not walked in this pass)
  uint32_t fix;    // s0l | delta << 8 | e << 12 (front padding words and
                   // bytes, end misalignment)
  uint32_t s0;     // init ^ ~0
  uint32_t gb;     // low half of row 0, lane 0's dword address
  uint32_t voff0;  // chunk 0, row 0's offset from the window base (kGrpBad: zeros)
  // wave-uniform: rows over the chain's walked groups, the records' window,
  // the lowest row-0 address
  uint32_t rmax, rmin;
  uint64_t wlo, whi, gbmin, gbmax;
  bool aligned;
  __device__ __forceinline__ uint32_t s0l() const { return fix & 15u; }
  __device__ __forceinline__ uint32_t delta() const { return (fix >> 8) & 3u; }
  __device__ __forceinline__ uint32_t e() const { return fix >> 12; }
};

template <int NCH, int R>
struct GrpRound {
  GrpChain ch[NCH];
  uint32_t w[NCH][R + 1];

  // Chain c from the desc lanes (row_newbcast:c), the groups in `mask`
  // only. `rec` is this lane's own record (desc lanes).
  __device__ __forceinline__ void adopt(int c, const GrpRec& rec, uint32_t t, uint32_t lane,
                                        uint32_t mask) {
    GrpChain& x = ch[c];
    const bool in = rec.kind == kGrpRows && ((mask >> (lane >> 4)) & 1u);
    const uint32_t q = (rec.len + 3u) >> 2;
    const uint32_t rows = in ? (q + 15u) >> 4 : 0u;
    const uint64_t end = rec.ptr() + rec.len;
    const uint64_t gb = (end & ~uint64_t{3}) - 64ull * rows;  // row 0, lane 0's dword
    const uint32_t fix = ((16u * rows - q) & 15u) | (((4u * q - rec.len) & 3u) << 8) |
                         (static_cast<uint32_t>(end & 3u) << 12);
    const uint64_t lo = in ? (rec.ptr() & ~uint64_t{3}) : ~uint64_t{0};
    const uint64_t hi = in ? ((end + 3u) & ~uint64_t{3}) : 0u;
    const uint64_t gl = in ? gb : ~uint64_t{0};
    const uint64_t gh = in ? gb : 0u;
    uint32_t rmax = 0, rmin = 0xffffffffu, emask = 0;
    uint64_t wlo = ~uint64_t{0}, whi = 0, gbmin = ~uint64_t{0}, gbmax = 0;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const uint32_t src = 16u * g + c;
      const uint32_t r = lane_u32(rows, src);
      rmax = max(rmax, r);
      rmin = min(rmin, r);
      emask |= r != 0 ? lane_u32(fix, src) >> 12 : 0u;
      wlo = min(wlo, lane_u64(lo, src));
      whi = max(whi, lane_u64(hi, src));
      gbmin = min(gbmin, lane_u64(gl, src));
      gbmax = max(gbmax, lane_u64(gh, src));
    }
    x.rmax = rmax;
    x.rmin = rmin;
    x.aligned = emask == 0;
    x.wlo = wlo;
    x.whi = whi;
    x.gbmin = gbmin;
    x.gbmax = gbmax;
    x.rows = row_bcast_c(rows, c);
    x.fix = row_bcast_c(fix, c);
    x.s0 = row_bcast_c(rec.s0, c);
    x.gb = row_bcast_c(static_cast<uint32_t>(gb), c);
    // chunk 0, row 0: lane t's dword holds record bytes from the record's
    // first aligned dword on, lane s0l + (e + delta >= 4); the lanes before
    // it are front padding (zeros, no access)
    const uint32_t t0 = x.s0l() + ((x.e() + x.delta()) >= 4u ? 1u : 0u);
    x.voff0 = (x.rows != 0 && t >= t0) ? x.gb + 4u * t - static_cast<uint32_t>(wlo) : kGrpBad;
  }

  // The R + 1 row loads of chunk k of every chain (row R: the next row's
  // dwords, for the realignment) through a window of the chunk's own rows
  // ([wlo, whi) of the records, cut to the rows of this chunk, so a window
  // is never wider than the records' spread plus a chunk): unconditional; a
  // kGrpBad offset or a row past the window reads zeros without an access.
  __device__ __forceinline__ void issue(uint32_t k, uint32_t t) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const GrpChain& x = ch[c];
      const uint64_t kr = 64ull * R * k;
      const uint64_t b = k == 0 ? x.wlo : x.gbmin + kr;
      const uint64_t e = min(x.whi, x.gbmax + kr + 64ull * (R + 1));
      const bool any = x.rmax != 0 && e > b;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          reinterpret_cast<void*>(any ? b : 0u), 0, static_cast<int>(any ? e - b : 0u),
          kBufferDword3);
      const uint32_t lane_off = x.rows != 0 ? x.gb + static_cast<uint32_t>(kr) + 4u * t -
                                                  static_cast<uint32_t>(b)
                                            : kGrpBad;
      int32_t v0 = static_cast<int32_t>(k == 0 ? x.voff0 : lane_off);
      int32_t v1 = static_cast<int32_t>(lane_off + (x.rows != 0 ? 64u : 0u));
      asm volatile("" : "+v"(v0));
      asm volatile("" : "+v"(v1));
      w[c][0] = __builtin_amdgcn_raw_buffer_load_b32(rs, v0, 0, kRagCachePolicy);
#pragma unroll
      for (int j = 1; j <= R; ++j)
        w[c][j] = __builtin_amdgcn_raw_buffer_load_b32(
            rs, v1 + static_cast<int32_t>(kGrpRowBytes) * (j - 1), 0, kRagCachePolicy);
    }
  }

  // Grid words from the aligned dwords, rows [0, nrow): lane t's word is
  // alignbyte(lane t + 1's dword, its own, e); lane 15 takes lane 0 of the
  // next row.
  __device__ __forceinline__ void realign(int c, uint32_t t, uint32_t nrow) {
    const uint32_t e = ch[c].e();
    uint32_t r0 = row_rol1(w[c][0]);
#pragma unroll
    for (int j = 0; j < R; ++j) {
      if (static_cast<uint32_t>(j) < nrow) {
        const uint32_t r1 = row_rol1(w[c][j + 1]);
        const uint32_t hi = t == 15u ? r1 : r0;
        w[c][j] = __builtin_amdgcn_alignbyte(hi, w[c][j], e);
        r0 = r1;
      }
    }
  }

  // Row 0 of a record: the front padding zeroed, the initial state injected
  // into the first 4 data bytes and its spill into the next word (lane
  // s0l + 1, or lane 0 of row 1 when s0l = 15).
  __device__ __forceinline__ uint32_t first_row(int c, uint32_t t) {
    const GrpChain& x = ch[c];
    const uint32_t s0l = x.s0l(), sh = 8u * x.delta();
    const uint32_t spill = sh ? (x.s0 >> (32u - sh)) : 0u;
    uint32_t v = w[c][0];
    v = t < s0l ? 0u : v;
    v = t == s0l ? ((v & (0xffffffffu << sh)) ^ (x.s0 << sh)) : v;
    v = t == s0l + 1u ? v ^ spill : v;
    w[c][1] = (s0l == 15u && t == 0) ? w[c][1] ^ spill : w[c][1];
    return x.rows != 0 ? v : 0u;
  }
};

// CRC32C of a record of fewer than 4 bytes from `init ^ ~0` = s0, bit by bit
// (desc lanes).
__device__ __forceinline__ uint32_t grp_tiny(const GrpRec& g) {
  uint32_t reg = g.s0;
  if (g.len != 0) {
    const uint64_t a4 = g.ptr() & ~uint64_t{3};
    const uint32_t sh = static_cast<uint32_t>(g.ptr() & 3u) * 8u;
    const uint32_t d0 = gload32(a4);
    const uint32_t d1 = (g.ptr() & 3u) + g.len > 4u ? gload32(a4 + 4u) : 0u;
    const uint32_t bytes = static_cast<uint32_t>(((static_cast<uint64_t>(d1) << 32) | d0) >> sh);
    for (uint32_t i = 0; i < g.len; ++i) {
      reg ^= (bytes >> (8u * i)) & 0xffu;
#pragma unroll
      for (int k = 0; k < 8; ++k) reg = (reg >> 1) ^ (kCastagnoliReflected & (0u - (reg & 1u)));
    }
  }
  return reg ^ 0xffffffffu;
}

// Workgroup `grp` of G walks its run of [0, total) in groups of four records
// a chain. lds: the compact image (kCompactLdsBytes). Every thread calls it.
template <int W, int NCH, int R>
__device__ __forceinline__ void group_run(const KernelArgs& a, const uint32_t* zpow,
                                          const uint32_t* grp_cols, uint32_t* lds, uint32_t grp,
                                          uint32_t G, uint32_t total) {
  static_assert(NCH >= 1 && NCH <= 4 && R >= 2 && (R + 1) * kGrpRowBytes < 4096, "shape");
  constexpr uint32_t kPerWave = 4u * NCH;  // records per wave-round
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = lane_id();
  const uint32_t t = lane & 15u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t per = total / G, extra = total % G;
  const uint32_t n = per + (grp < extra ? 1u : 0u);
  const uint32_t start = grp * per + min(grp, extra);
  if (n == 0) return;  // the whole workgroup
  const bool desc_lane = t < static_cast<uint32_t>(NCH);
  // desc lane 16 g + c holds record 4c + g of the wave's round
  const uint32_t my = 4u * t + (lane >> 4);
  build_group_image<W>(lds, zpow, grp_cols, tid, wave, lane);  // (ends with a barrier)
  const LaneKeys keys = lane_keys(lane);
  const uint32_t lane_base = compact_lane_base(lane);

  // wave w takes rounds w, w + W, ... of kPerWave records
  const uint32_t nrounds = (n + kPerWave - 1) / kPerWave;
  uint32_t r = wave;
  auto live_of = [&](uint32_t rr) { return desc_lane && rr < nrounds && rr * kPerWave + my < n; };
  // the descriptor pipeline: stage 2 of this round, stage 1 of the next
  bool live0 = live_of(r);
  GrpRaw raw0 = grp_stage1(a, start + r * kPerWave + my, live0);
  GrpHdr hdr0 = grp_stage2(a, raw0, live0);
  bool live1 = live_of(r + W);
  GrpRaw raw1 = grp_stage1(a, start + (r + W) * kPerWave + my, live1);
  for (; r < nrounds; r += W) {
    GrpRec rec = grp_record(a, raw0, hdr0, live0, start + r * kPerWave + my);
    // the next round's stage 2, the one after's stage 1 (in flight during
    // this round's rows)
    const GrpHdr hdr1 = grp_stage2(a, raw1, live1);
    const bool live2 = live_of(r + 2 * W);
    const GrpRaw raw2 = grp_stage1(a, start + (r + 2 * W) * kPerWave + my, live2);
    rec = grp_sort<NCH>(rec, lane, desc_lane);

    // chains whose records lie more than a buffer window apart walk one
    // group per pass (four passes; scattered batches only)
    uint32_t far = 0;
    {
      const bool rk = rec.kind == kGrpRows;
      const uint64_t lo = rk ? (rec.ptr() & ~uint64_t{3}) : ~uint64_t{0};
      const uint64_t hi = rk ? ((rec.ptr() + rec.len + 3u) & ~uint64_t{3}) : 0u;
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        uint64_t wlo = ~uint64_t{0}, whi = 0, wmax = 0;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const uint64_t l = lane_u64(lo, 16u * g + c);
          wlo = min(wlo, l);
          wmax = l != ~uint64_t{0} ? max(wmax, l) : wmax;
          whi = max(whi, lane_u64(hi, 16u * g + c));
        }
        // the starts' spread (the chunk windows span it)
        if (whi > wlo && wmax - wlo > kGrpSpanMax) far |= 1u << c;
      }
    }
    const uint32_t npass = far != 0 ? 4u : 1u;
    for (uint32_t p = 0; p < npass; ++p) {
      GrpRound<NCH, R> rd;
      uint32_t nchunks = 0;
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const uint32_t m = ((far >> c) & 1u) ? (1u << p) : (p == 0 ? 15u : 0u);
        rd.adopt(c, rec, t, lane, m);
        nchunks = max(nchunks, (rd.ch[c].rmax + R - 1) / R);
      }
      uint32_t st[NCH];
      uint32_t crc[NCH];
#pragma unroll
      for (int c = 0; c < NCH; ++c) crc[c] = 0;
      if (nchunks != 0) rd.issue(0, t);
      for (uint32_t k = 0; k < nchunks; ++k) {
        // rows j0 .. R - 1 (row kR + j of the records): first every chain up
        // to its shortest group, interleaved, without the freeze; then each
        // chain's rows up to its longest, a group's state kept once its own
        // rows are done
        uint32_t nab = R, nmax[NCH], nmin[NCH];
        int32_t rem[NCH];
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
          const uint32_t kr = k * R;
          nmax[c] = rd.ch[c].rmax > kr ? min(static_cast<uint32_t>(R), rd.ch[c].rmax - kr) : 0u;
          nmin[c] = rd.ch[c].rmin > kr ? min(static_cast<uint32_t>(R), rd.ch[c].rmin - kr) : 0u;
          nab = min(nab, nmin[c]);
          rem[c] = static_cast<int32_t>(rd.ch[c].rows) - static_cast<int32_t>(kr);
        }
#pragma unroll
        for (int c = 0; c < NCH; ++c)
          if (!rd.ch[c].aligned) rd.realign(c, t, nmax[c]);
        const uint32_t j0 = k == 0 ? 1u : 0u;
        if (k == 0) {
#pragma unroll
          for (int c = 0; c < NCH; ++c) st[c] = rd.first_row(c, t);
        }
#pragma unroll
        for (int j = 0; j < R; ++j) {
          const uint32_t u = static_cast<uint32_t>(j);
          if (u >= j0 && u < nab) {
#pragma unroll
            for (int c = 0; c < NCH; ++c) st[c] = row_step_c(lds, st[c], rd.w[c][j], keys);
          }
        }
        const uint32_t jb = max(j0, nab);
#pragma unroll
        for (int j = 0; j < R; ++j) {
          const uint32_t u = static_cast<uint32_t>(j);
          if (u >= jb) {
#pragma unroll
            for (int c = 0; c < NCH; ++c) {
              if (u < nmin[c]) {
                st[c] = row_step_c(lds, st[c], rd.w[c][j], keys);
              } else if (u < nmax[c]) {
                const uint32_t nx = row_step_c(lds, st[c], rd.w[c][j], keys);
                st[c] = rem[c] > j ? nx : st[c];
              }
            }
          }
        }
        // chains whose last chunk this was: end shift, the group's xor
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
          if (rd.ch[c].rmax != 0 && rd.ch[c].rmax <= (k + 1) * R)
            crc[c] = row_xor16(lane_end_shift_c(lds, st[c], lane_base)) ^ 0xffffffffu;
        }
        if (k + 1 < nchunks) rd.issue(k + 1, t);
      }
      // desc lane 16 g + c stores its record (chain c's group g) in the pass
      // that walked it
      if (rec.kind == kGrpRows) {
        uint32_t mine = 0;
        bool walked = false;
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
          if (t == static_cast<uint32_t>(c)) {
            mine = crc[c];
            walked = ((far >> c) & 1u) ? (lane >> 4) == p : p == 0;
          }
        }
        if (walked) grp_store(a, rec, mine);
      }
    }
    // records of fewer than 4 bytes: bit by bit in their desc lanes
    if (__builtin_amdgcn_ballot_w64(rec.kind == kGrpTiny) != 0) {
      if (rec.kind == kGrpTiny) grp_store(a, rec, grp_tiny(rec));
    }
    raw0 = raw1;
    hdr0 = hdr1;
    live0 = live1;
    raw1 = raw2;
    live1 = live2;
  }
}

}  // namespace
}  // namespace lvkv

#endif  // LVKV_CRC32C_GROUP_BODY_H_
