// WAL / MANIFEST verify on the device: every physical
// record of a log image, with log::Reader::ReadPhysicalRecord's reporting
// (db/log_reader.cc:189-271, checksum = true, initial_offset = 0).
//
// Headers never straddle a 32 KiB block (the writer pads the tail of a block
// with zeros, db/log_writer.cc:44-55) and the reader drops the REST OF THE
// BLOCK on every error, so each block's verdict depends on that block only.
// One launch, one read of the image:
//
//   log_verify_kernel  persistent, one 512-thread workgroup per CU, blocks
//                      b = blockIdx.x + k * gridDim.x. Each block is read
//                      from HBM once (the next one's 16-byte loads in flight
//                      in registers while the current one is worked on) into
//                      one of two LDS buffers. Wave 0 walks the headers of
//                      the NEXT block from LDS (one lane; a few cycles per
//                      record) and finds the current block's first record
//                      slot by a decoupled look-back over the per-block
//                      record counts (published as soon as a block is
//                      walked, so no workgroup waits on another's CRCs);
//                      waves 1-7 checksum the current block's records from
//                      LDS (the end-aligned word grid of the other kernels,
//                      unaligned words rebuilt with v_alignbyte, rows folded
//                      with Z_256 on the compact image); records over 4 KiB
//                      are walked by the whole workgroup. Then the block's
//                      merge: the first mismatch drops the rest of the block,
//                      block status and reported drop bytes. The last
//                      workgroup to finish sums the per-block results into
//                      the report.
//
// Scratch (per-block record counts and good-record counts, one completion
// counter) is the caller's per-stream buffer (lvkv_capi.cpp): the count words
// are tagged with the call's generation, and the counter is left at 0 by the
// last workgroup of every call, so nothing is cleared per call.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <atomic>

#include "crc32c_compact_common.h"
#include "crc32c_device_common.h"
#include "lvkv_crc32c.h"
#include "lvkv_kernel_args.h"
#include "lvkv_log_events.h"

namespace lvkv {
namespace {

constexpr uint64_t kLogBlock = 32768;  // db/log_format.h kBlockSize
constexpr uint32_t kLogHeader = 7;     // db/log_format.h kHeaderSize

struct BlockSpan {
  uint64_t start, end;
  bool eof;  // a short read: the reader's eof_ (log_reader.cc:202-204)
};

__device__ __forceinline__ BlockSpan block_span(uint64_t b, uint64_t size) {
  BlockSpan s;
  s.start = b * kLogBlock;
  s.end = min(size, s.start + kLogBlock);
  s.eof = s.end - s.start < kLogBlock;
  return s;
}

// Walks one block's headers in LDS, blk[0, n), to the first stop (bad
// length, zero record, end) like ReadPhysicalRecord, with the stop position:
// one LDS round trip per header; returns the verdict, *stop = the block
// offset after the last record. Called by a whole wave with uniform
// arguments: every lane reads the same dwords (a broadcast) and the header
// arithmetic runs on the scalar unit (readfirstlane), so a step is the LDS
// latency plus a few SALU cycles; lane 0 writes the positions.
__device__ __forceinline__ uint8_t walk_positions(const uint8_t* blk, uint32_t n, bool eof,
                                                  uint16_t* pos, uint32_t* count, uint32_t* stop) {
  uint32_t p = 0, k = 0, length = 0, w = 0;
  // positions collect in a register, record k in lane k % 64 (a select),
  // written to pos[] 64 at a time: no per-step masked LDS store
  uint32_t held = 0;
  const uint32_t lane = threadIdx.x & 63u;
  // Every lane carries the same p in a VGPR, so the chain from one header to
  // the next is VALU + one LDS round trip (no readfirstlane, no scalar
  // funnel shift): the dwords holding bytes p + 4 .. p + 6 are (p & ~3) + 4
  // and + 8, the bytes shifted out by v_alignbyte(p & 3). The next header's
  // read is issued before this header's stop test (speculatively, clamped
  // into the buffer), so the test's compare and branch overlap the LDS trip.
  // The reads are inline asm so the compiler neither sinks the speculative
  // one below the branch nor turns the chain scalar; their registers are
  // tied to explicit lgkmcnt waits (an asm load's destination is written
  // late, so it must stay live until a wait has seen it land).
  if (n >= kLogHeader) {
    const uint32_t base = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(blk));
    uint64_t cur, nxt;
    // bp = base + p (the buffer is 16-byte aligned, so bp & 3 == p & 3): the
    // next read's address is two VALU ops from the length. A read past the
    // block (a bad length, about to stop the walk) lands elsewhere in LDS or
    // past the allocation (zeros): harmless, its bytes are never used.
    uint32_t bp = base;
    asm volatile("ds_read2_b32 %0, %1 offset0:1 offset1:2" : "=v"(cur) : "v"(base));
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(cur));
    for (;;) {
      w = __builtin_amdgcn_alignbyte(static_cast<uint32_t>(cur >> 32), static_cast<uint32_t>(cur),
                                     bp & 3u);
      length = w & 0xffffu;
      const uint32_t nbp = bp + kLogHeader + length;
      asm volatile("ds_read2_b32 %0, %1 offset0:1 offset1:2" : "=v"(nxt) : "v"(nbp & ~3u));
      const uint32_t np = p + kLogHeader + length;
      __builtin_amdgcn_sched_barrier(0);  // the read issues before the tests below
      // a bad length (:221-232) or a zero record (:234-240) ends the walk
      // (bit 0); bit 1: the record ends within 7 bytes of the block end
      const bool bad = np > n || (w & 0xffffffu) == 0;
      const uint32_t f =
          __builtin_amdgcn_readfirstlane((bad ? 1u : 0u) | (n - np < kLogHeader ? 2u : 0u));
      if (f & 1u) break;
      held = lane == (k & 63u) ? p : held;
      ++k;
      if (__builtin_expect((k & 63u) == 0, 0)) pos[k - 64u + lane] = static_cast<uint16_t>(held);
      p = np;
      bp = nbp;
      if (f & 2u) break;
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(nxt));
      cur = nxt;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(nxt));
  }
  p = __builtin_amdgcn_readfirstlane(p);
  length = __builtin_amdgcn_readfirstlane(length);
  if (lane < (k & 63u)) pos[(k & ~63u) + lane] = static_cast<uint16_t>(held);
  uint8_t v;
  if (n - p < kLogHeader)
    v = (eof && p < n) ? LVKV_LOGBLK_EOF : LVKV_LOGBLK_OK;  // :206-213
  else if (kLogHeader + length > n - p)
    v = eof ? LVKV_LOGBLK_EOF : LVKV_LOGBLK_BAD_LENGTH;
  else
    v = LVKV_LOGBLK_ZERO;
  *count = k;
  *stop = p;
  return v;
}

constexpr int kVW = 16;  // waves per workgroup
constexpr uint32_t kVThreads = 64 * kVW;
constexpr uint32_t kMaxRecs = (static_cast<uint32_t>(kLogBlock) + kLogHeader - 1) / kLogHeader;
constexpr uint32_t kLongRec = 16 * 256;  // CRC bytes walked by one wave, at most
constexpr uint32_t kMaxLong = static_cast<uint32_t>(kLogBlock) / kLongRec + 1;
constexpr uint32_t kBufBytes = static_cast<uint32_t>(kLogBlock) + 16;
constexpr uint32_t kPerThread = static_cast<uint32_t>(kLogBlock) / (kVThreads * 16u);  // uint4s

// look-back words: generation (26 bits) | flag (2) | value (36)
constexpr uint64_t kFlagAgg = 1, kFlagInc = 2;
__device__ __forceinline__ uint64_t link_word(uint32_t gen, uint64_t flag, uint64_t v) {
  return (static_cast<uint64_t>(gen & 0x3ffffffu) << 38) | (flag << 36) | v;
}
__device__ __forceinline__ bool link_is(uint64_t x, uint32_t gen) {
  return static_cast<uint32_t>(x >> 38) == (gen & 0x3ffffffu) && ((x >> 36) & 3u) != 0;
}

struct LogArgs {
  const uint8_t* file;
  uint64_t size;
  uint32_t nblocks, capacity, gen, pad_;
  uint64_t* hdr_off;
  uint32_t* actual;
  uint8_t* rec_status;
  uint8_t* block_status;
  uint32_t* block_drop;
  lvkv_log_report* r;
  uint64_t* agg;   // nblocks: the block's record count (published when walked)
  uint64_t* inc;   // nblocks: records in blocks 0..b (published when placed)
  uint32_t* good;  // nblocks records the reader returns
  uint64_t* done;  // finished workgroups (zeroed before the launch)
  const uint32_t* zpow;
  const uint32_t* lane_cols;
  uint32_t* events;  // nullable: the ReadRecord event stream (lvkv_log_events.h)
  uint64_t* stamps;  // probe build only: 8 u64 per (workgroup, iteration)
  uint32_t knobs;    // probe build only: 1 no record CRCs, 2 no walk wait, 4 no placement
};

__device__ __forceinline__ void log_stamp(const LogArgs& a, uint32_t k, int slot) {
#ifdef LVKV_PROBE_BUILD
  if (a.stamps != nullptr && lane_id() == 0)
    a.stamps[(static_cast<uint64_t>(blockIdx.x) * 16u + min(k, 15u)) * 8u + slot] =
        __builtin_amdgcn_s_memrealtime();
#endif
}

__device__ __forceinline__ uint32_t lds_word(const uint8_t* buf, uint32_t x) {
  const uint32_t* d = reinterpret_cast<const uint32_t*>(buf + (x & ~3u));
  const uint32_t lo = d[0];
  const uint32_t hi = d[1];
  return (x & 3u) ? __builtin_amdgcn_alignbyte(hi, lo, x & 3u) : lo;
}

// CRC32C of buf[a, a + n) (LDS, n >= 4) by one wave: the end-aligned word
// grid (grid word j = the 4 bytes ending 4 * (q - 1 - j) before the end,
// lane s of row r holds word 64 r + s), Horner over rows with Z_256, lane end
// shift, xor-reduce; init 0 (~0 xored into the first word, spill into the
// next), as fix_first_chunk / segment_register do. Two records at once (NR =
// 2; the second may be empty, n = 0) so their dependent LDS chains overlap.
struct LdsRec {
  uint32_t first, s0l, sh, spill;
};

// Geometry of a record of n >= 4 bytes at a on a grid of `rows` rows (at
// least its own; extra rows in front are all-zero words, which leave the
// register at 0, so two records can share one row count).
__device__ __forceinline__ LdsRec lds_rec(uint32_t a, uint32_t n, uint32_t rows) {
  LdsRec r;
  const uint32_t q = (n + 3u) >> 2;
  const uint32_t delta = 4u * q - n;
  r.s0l = 64u * rows - q;
  r.sh = 8u * delta;
  r.spill = delta ? (0xffffffffu >> (32u - r.sh)) : 0u;
  r.first = a - delta;  // byte address of grid word s0l
  return r;
}

// Byte address of grid word 64 r + lane (0 for a word before the record).
__device__ __forceinline__ uint32_t grid_addr(const LdsRec& g, uint32_t r, uint32_t lane) {
  const uint32_t j = 64u * r + lane;
  return j >= g.s0l ? g.first + 4u * (j - g.s0l) : 0u;
}

// The grid word from its two aligned dwords (masks and row-0 fix-ups).
__device__ __forceinline__ uint32_t grid_fix(const LdsRec& g, uint32_t r, uint32_t lane,
                                             uint32_t x, uint32_t lo, uint32_t hi) {
  const uint32_t j = 64u * r + lane;
  uint32_t w = __builtin_amdgcn_alignbyte(hi, lo, x & 3u);
  w = j >= g.s0l ? w : 0u;
  w = j == g.s0l ? ((w & (0xffffffffu << g.sh)) ^ (0xffffffffu << g.sh)) : w;
  return j == g.s0l + 1u ? (w ^ g.spill) : w;
}

// NR records at once. Each row issues every LDS read of every record (the
// two data dwords and the four Z_256 lookups of the running state) before
// any is consumed, so a row costs one LDS round trip for all of them; the
// scheduling barriers keep the compiler from pairing each read with its use.
template <int NR>
__device__ __forceinline__ void lds_record_crcs(const uint8_t* buf, const uint32_t (&at)[NR],
                                                const uint32_t (&n)[NR], const uint32_t* img,
                                                const LaneKeys& keys, uint32_t lane,
                                                uint32_t lane_base, uint32_t (&crc)[NR]) {
  uint32_t q = 0;
#pragma unroll
  for (int t = 0; t < NR; ++t) q = max(q, (n[t] + 3u) >> 2);
  const uint32_t rows = (q + 63u) >> 6;
  LdsRec g[NR];
  uint32_t st[NR];
  {
    uint32_t x[NR], lo[NR], hi[NR];
#pragma unroll
    for (int t = 0; t < NR; ++t) {
      g[t] = lds_rec(at[t], n[t], rows);
      x[t] = grid_addr(g[t], 0, lane);
      const uint32_t* d = reinterpret_cast<const uint32_t*>(buf + (x[t] & ~3u));
      lo[t] = d[0];
      hi[t] = d[1];
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t = 0; t < NR; ++t) st[t] = grid_fix(g[t], 0, lane, x[t], lo[t], hi[t]);
  }
  for (uint32_t r = 1; r < rows; ++r) {
    uint32_t x[NR], lo[NR], hi[NR], v[NR][4];
#pragma unroll
    for (int t = 0; t < NR; ++t) {
      x[t] = grid_addr(g[t], r, lane);
      const uint32_t* d = reinterpret_cast<const uint32_t*>(buf + (x[t] & ~3u));
      lo[t] = d[0];
      hi[t] = d[1];
#pragma unroll
      for (int p = 0; p < 4; ++p)
        v[t][p] = lds_ld(img, __builtin_amdgcn_perm(st[t], keys.kpack, keys.sel[p]));
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t = 0; t < NR; ++t) {
      const uint32_t w = grid_fix(g[t], r, lane, x[t], lo[t], hi[t]);
      st[t] = xor3(xor3(v[t][0], v[t][1], w), v[t][2], v[t][3]);
    }
  }
  // lane end shift (eight lane-private nibble lookups per record), all
  // issued before the xors
  uint32_t e[NR][8];
#pragma unroll
  for (int t = 0; t < NR; ++t)
#pragma unroll
    for (int k = 0; k < 8; ++k)
      e[t][k] = lds_ld(img, (lane_base | (((st[t] >> (4 * k)) & 15u) << 9)) + 8192u * k);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int t = 0; t < NR; ++t) {
    const uint32_t r = xor3(xor3(e[t][0], e[t][1], e[t][2]), xor3(e[t][3], e[t][4], e[t][5]),
                            e[t][6] ^ e[t][7]);
    crc[t] = wave_xor_dpp(r) ^ 0xffffffffu;
  }
}

// Bitwise CRC32C of fewer than 4 bytes (lane-uniform).
__device__ __forceinline__ uint32_t tiny_crc(const uint8_t* p, uint32_t n) {
  uint32_t reg = 0xffffffffu;
  for (uint32_t i = 0; i < n; ++i) {
    reg ^= p[i];
#pragma unroll
    for (int k = 0; k < 8; ++k) reg = (reg >> 1) ^ (kCastagnoliReflected & (0u - (reg & 1u)));
  }
  return reg ^ 0xffffffffu;
}

__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(static_cast<unsigned long long>(v), d, 64);
  return v;
}

// Wave 0: the first record slot of block b = w + k G (workgroup w, iteration
// k): this workgroup's own previous block b - G ends at prev_inc (its
// inclusive count, known locally), and the G - 1 blocks between are all
// walked an iteration ahead, so their counts are published: one memory round
// trip, no wait on another workgroup's placement (which would chain every
// workgroup's iterations together).
__device__ uint64_t log_base(const LogArgs& a, uint32_t b, uint32_t G, uint64_t prev_inc,
                             uint32_t lane) {
  const uint32_t lo = b >= G ? b - G + 1 : 0;
  uint64_t sum = 0;
  for (uint32_t j = lo + lane; j < b; j += 64) {
    uint64_t x;
    do {
      x = __hip_atomic_load(&a.agg[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } while (!link_is(x, a.gen));
    sum += x & ((uint64_t{1} << 36) - 1);
  }
  return (b >= G ? prev_inc : 0) + wave_sum64(sum);
}

// Block b's bytes into registers: 16 per lane-load, kPerThread loads, bounded
// by the image (a partial last block reads zeros past its end).
__device__ __forceinline__ void load_block(const LogArgs& a, uint32_t b, uint32_t tid,
                                           uint4 (&v)[kPerThread]) {
  const BlockSpan s = block_span(b, a.size);
  const uint32_t n = static_cast<uint32_t>(s.end - s.start);
  const uint8_t* src = a.file + s.start;
  // (a partial last block byte by byte: a buffer load that crosses the
  // bound returns zeros for the whole load, and the image may end anywhere)
  if ((reinterpret_cast<uintptr_t>(src) & 3u) == 0 && n == kLogBlock) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t*>(src), 0, static_cast<int>(n), kBufferDword3);
#pragma unroll
    for (uint32_t k = 0; k < kPerThread; ++k) {
      const auto x = __builtin_amdgcn_raw_buffer_load_b128(
          r, static_cast<int>(16u * (tid + kVThreads * k)), 0, 0);
      v[k] = make_uint4(x[0], x[1], x[2], x[3]);
    }
  } else {  // a partial block, or an image not on a 4-byte boundary
#pragma unroll
    for (uint32_t k = 0; k < kPerThread; ++k) {
      uint32_t w[4];
      for (uint32_t d = 0; d < 4; ++d) {
        uint32_t x = 0;
        for (uint32_t i = 0; i < 4; ++i) {
          const uint32_t o = 16u * (tid + kVThreads * k) + 4u * d + i;
          if (o < n) x |= static_cast<uint32_t>(src[o]) << (8 * i);
        }
        w[d] = x;
      }
      v[k] = make_uint4(w[0], w[1], w[2], w[3]);
    }
  }
}

__global__ void __launch_bounds__(kVThreads, 1) log_verify_kernel(LogArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t img[kCompactLdsBytes / 4 + kVW];
  __shared__ __attribute__((aligned(16))) uint8_t buf[2][kBufBytes];
  __shared__ uint16_t pos[2][kMaxRecs];
  __shared__ uint32_t cnt[2], stop[2];
  __shared__ uint8_t walked[2];
  __shared__ uint64_t base_s;
  __shared__ uint32_t ready, first_bad, nlong, bad_s, next_rec;
  __shared__ uint16_t longs[kMaxLong];
  __shared__ unsigned long long red_good, red_drop;
  __shared__ uint32_t red_corrupt, red_first, last_s;

  const uint32_t tid = threadIdx.x;
  const uint32_t lane = lane_id();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t G = gridDim.x;
  uint4 pre[kPerThread];
  uint64_t prev_inc = 0;  // wave 0: records in blocks 0 .. (this workgroup's last block)

  const uint32_t b0 = blockIdx.x;
  if (b0 < a.nblocks) load_block(a, b0, tid, pre);
  build_compact_image<kVW>(img, a.zpow, a.lane_cols, tid, wave, lane);  // ends with a barrier
  const LaneKeys keys = lane_keys(lane);
  const uint32_t lane_base = compact_lane_base(lane);
  if (b0 < a.nblocks) {
#pragma unroll
    for (uint32_t k = 0; k < kPerThread; ++k)
      reinterpret_cast<uint4*>(buf[0])[tid + kVThreads * k] = pre[k];
  }
  __syncthreads();
  if (b0 < a.nblocks) {
    if (wave == 0) {
      const BlockSpan s = block_span(b0, a.size);
      uint32_t c, st;
      const uint8_t v = walk_positions(buf[0], static_cast<uint32_t>(s.end - s.start), s.eof,
                                       pos[0], &c, &st);
      if (lane == 0) {
        walked[0] = v;
        cnt[0] = c;
        stop[0] = st;
        __hip_atomic_store(&a.agg[b0], link_word(a.gen, kFlagAgg, c), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    if (b0 + G < a.nblocks) load_block(a, b0 + G, tid, pre);
  }

  for (uint32_t k = 0;; ++k) {
    const uint32_t b = b0 + k * G;
    if (b >= a.nblocks) break;
    const uint32_t cur = k & 1u;
    const uint32_t nb = b + G;
    const BlockSpan s = block_span(b, a.size);
    if (nb < a.nblocks) {
#pragma unroll
      for (uint32_t i = 0; i < kPerThread; ++i)
        reinterpret_cast<uint4*>(buf[cur ^ 1u])[tid + kVThreads * i] = pre[i];
    }
    if (tid == 0) {
      ready = 0;
      first_bad = 0xffffffffu;
      nlong = 0;
      next_rec = 0;
    }
    __syncthreads();  // buf[cur ^ 1] written, pos[cur] / cnt[cur] visible
    if (tid == 0) log_stamp(a, k, 0);
    // the block after next into registers; wave 0 issues its share after its
    // placement loads (a wait on those would otherwise wait for these too)
    if (wave != 0 && nb + G < a.nblocks) load_block(a, nb + G, tid, pre);
    const uint32_t c = cnt[cur];
    const uint8_t* blk = buf[cur];

    // wave 0 places the block, wave 1 walks the next one; then both join the
    // other waves on this block's records (taken one at a time from an LDS
    // counter, so the late waves take fewer)
    if (wave == 0) {
#ifdef LVKV_PROBE_BUILD
      const uint64_t base = (a.knobs & 4u) ? uint64_t{b} * 30u : log_base(a, b, G, prev_inc, lane);
#else
      const uint64_t base = log_base(a, b, G, prev_inc, lane);
#endif
      prev_inc = base + c;
      if (lane == 0) {
        __hip_atomic_store(&a.inc[b], link_word(a.gen, kFlagInc, base + c), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        base_s = base;
        __atomic_store_n(&ready, 1u, __ATOMIC_RELEASE);
        log_stamp(a, k, 1);
      }
      if (nb + G < a.nblocks) load_block(a, nb + G, tid, pre);
    } else if (wave == 1 && nb < a.nblocks) {
      // the walk is the iteration's longest chain: this wave issues first
      __builtin_amdgcn_s_setprio(3);
      const BlockSpan ns = block_span(nb, a.size);
      uint32_t nc, nst;
      const uint8_t v = walk_positions(buf[cur ^ 1u], static_cast<uint32_t>(ns.end - ns.start),
                                       ns.eof, pos[cur ^ 1u], &nc, &nst);
      __builtin_amdgcn_s_setprio(0);
      if (lane == 0) {
        walked[cur ^ 1u] = v;
        cnt[cur ^ 1u] = nc;
        stop[cur ^ 1u] = nst;
        __hip_atomic_store(&a.agg[nb], link_word(a.gen, kFlagAgg, nc), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        log_stamp(a, k, 2);
      }
    }
    {
      bool have_base = false;
      uint64_t base = 0;
      for (;;) {
        // kGrab records per grab, walked together (their dependent LDS chains
        // overlap); long (> kLongRec) ones are queued for the workgroup, tiny
        // (< 4 bytes) ones done bitwise
        constexpr int kGrab = 2;
        uint32_t j0 = 0;
        if (lane == 0) j0 = atomicAdd(&next_rec, static_cast<uint32_t>(kGrab));
        j0 = __builtin_amdgcn_readfirstlane(j0);
        if (j0 >= c) break;
        uint32_t pp[kGrab], nn[kGrab], at[kGrab], len[kGrab], crc[kGrab];
        bool valid[kGrab], rows_ok[kGrab];
        int lead = -1;
#pragma unroll
        for (int t = 0; t < kGrab; ++t) {
          const uint32_t j = j0 + t;
          pp[t] = 0;
          nn[t] = 0;
          valid[t] = false;
          if (j < c) {
            pp[t] = pos[cur][j];
            nn[t] = 1u + (static_cast<uint32_t>(blk[pp[t] + 4]) |
                          (static_cast<uint32_t>(blk[pp[t] + 5]) << 8));
            if (nn[t] > kLongRec) {
              if (lane == 0) longs[atomicAdd(&nlong, 1u)] = static_cast<uint16_t>(j);
            } else {
              valid[t] = true;
            }
          }
          rows_ok[t] = valid[t] && nn[t] >= 4u;
          if (rows_ok[t] && lead < 0) lead = t;
        }
#ifdef LVKV_PROBE_BUILD
        if (a.knobs & 1u) {  // no CRC (timing only)
#pragma unroll
          for (int t = 0; t < kGrab; ++t) valid[t] = rows_ok[t] = false;
          lead = -1;
        }
#endif
        if (lead >= 0) {
          // a record that is absent or tiny is replaced by the first real one
#pragma unroll
          for (int t = 0; t < kGrab; ++t) {
            at[t] = rows_ok[t] ? pp[t] + 6 : pp[lead] + 6;
            len[t] = rows_ok[t] ? nn[t] : nn[lead];
          }
          lds_record_crcs<kGrab>(blk, at, len, img, keys, lane, lane_base, crc);
        }
        if (wave == 2 && !have_base) log_stamp(a, k, 7);
#pragma unroll
        for (int t = 0; t < kGrab; ++t)
          if (valid[t] && !rows_ok[t]) crc[t] = tiny_crc(blk + pp[t] + 6, nn[t]);
        if (!have_base) {
          while (__atomic_load_n(&ready, __ATOMIC_ACQUIRE) == 0) __builtin_amdgcn_s_sleep(1);
          base = base_s;
          have_base = true;
        }
        if (lane == 0) {
#pragma unroll
          for (int t = 0; t < kGrab; ++t) {
            if (!valid[t]) continue;
            const uint32_t j = j0 + t;
            const bool ok = crc[t] == crc_unmask(lds_word(blk, pp[t]));
            if (!ok) atomicMin(&first_bad, j);
            const uint64_t gi = base + j;
            if (gi < a.capacity) {
              a.hdr_off[gi] = s.start + pp[t];
              a.actual[gi] = crc[t];
              a.rec_status[gi] = ok ? LVKV_REC_OK : LVKV_REC_CHECKSUM;
              if (a.events != nullptr)
                a.events[gi + b] = ok ? log_event(kEvRec, blk[pp[t] + 6], nn[t] - 1u)
                                      : log_event(kEvSkip, 0, 0);
            }
          }
        }
      }
    }
    if (wave == 2) log_stamp(a, k, 3);
    __syncthreads();
    if (tid == 0) log_stamp(a, k, 4);
    // records over kLongRec: the whole workgroup, from the image (L2-warm)
    const uint32_t nl = nlong;
    for (uint32_t i = 0; i < nl; ++i) {
      const uint32_t j = longs[i];
      const uint32_t p = pos[cur][j];
      const uint32_t n = 1u + (static_cast<uint32_t>(blk[p + 4]) |
                               (static_cast<uint32_t>(blk[p + 5]) << 8));
      const uint64_t at = reinterpret_cast<uint64_t>(a.file) + s.start + p + 6;
      const uint32_t crc = workgroup_crc<kVW, 4096>(img, img + kCompactLdsBytes / 4, at, at + n,
                                                    0u, keys, tid, wave, lane, lane_base, a.zpow);
      if (tid == 0) {
        const bool ok = crc == crc_unmask(lds_word(blk, p));
        if (!ok) first_bad = min(first_bad, j);
        const uint64_t gi = base_s + j;
        if (gi < a.capacity) {
          a.hdr_off[gi] = s.start + p;
          a.actual[gi] = crc;
          a.rec_status[gi] = ok ? LVKV_REC_OK : LVKV_REC_CHECKSUM;
          if (a.events != nullptr)
            a.events[gi + b] = ok ? log_event(kEvRec, blk[p + 6], n - 1u) : log_event(kEvSkip, 0, 0);
        }
      }
    }
    // the block's merge (db/log_reader.cc:221-255)
    if (tid == 0) {
      log_stamp(a, k, 5);
      const uint32_t bad = first_bad;
      uint8_t status = walked[cur];
      uint64_t drop = 0;
      if (bad != 0xffffffffu) {
        status = LVKV_LOGBLK_CHECKSUM;
        drop = s.end - (s.start + pos[cur][bad]);  // ReportCorruption(buffer_.size(), ...)
      } else if (status == LVKV_LOGBLK_BAD_LENGTH) {
        drop = (s.end - s.start) - stop[cur];  // ReportCorruption(drop_size, "bad record length")
      }
      a.block_status[b] = status;
      a.block_drop[b] = static_cast<uint32_t>(drop);
      // the block's event follows its c records: item base + c + b
      if (a.events != nullptr && base_s + c <= a.capacity)
        a.events[base_s + c + b] = log_block_event(status, static_cast<uint32_t>(drop));
      a.good[b] = bad != 0xffffffffu ? bad : c;
      bad_s = bad;
    }
    __syncthreads();
    // records after the first mismatch: the reader cleared the buffer (:248-255)
    const uint32_t bad = bad_s;
    if (bad != 0xffffffffu)
      for (uint32_t j = bad + 1 + tid; j < c; j += kVThreads)
        if (base_s + j < a.capacity) {
          a.rec_status[base_s + j] = LVKV_REC_DROPPED;
          if (a.events != nullptr) a.events[base_s + j + b] = log_event(kEvSkip, 0, 0);
        }
    __syncthreads();  // pos[cur], ready, first_bad are reused
    if (tid == 0) log_stamp(a, k, 6);
  }

  // The last workgroup to finish writes the report (one fetch-add each on a
  // counter zeroed on the stream before the launch: a compare-and-swap loop
  // over 256 contending workgroups serialises hundreds of memory round trips).
  if (tid == 0) {
    __threadfence();
    const uint64_t old = __hip_atomic_fetch_add(a.done, uint64_t{1}, __ATOMIC_ACQ_REL,
                                                __HIP_MEMORY_SCOPE_AGENT);
    last_s = old + 1 == G ? 1u : 0u;
    red_good = 0;
    red_drop = 0;
    red_corrupt = 0;
    red_first = 0xffffffffu;
  }
  __syncthreads();
  if (!last_s) return;
  __threadfence();
  // the next call on this stream reuses the scratch: leave the counter at 0
  if (tid == 0) __hip_atomic_store(a.done, uint64_t{0}, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  unsigned long long g = 0, d = 0;
  uint32_t nc = 0, fb = 0xffffffffu;
  for (uint32_t b = tid; b < a.nblocks; b += kVThreads) {
    const uint8_t st = __hip_atomic_load(&a.block_status[b], __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    g += __hip_atomic_load(&a.good[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (st == LVKV_LOGBLK_CHECKSUM || st == LVKV_LOGBLK_BAD_LENGTH) {
      ++nc;
      d += __hip_atomic_load(&a.block_drop[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      fb = min(fb, b);
    }
  }
  atomicAdd(&red_good, g);
  atomicAdd(&red_drop, d);
  atomicAdd(&red_corrupt, nc);
  atomicMin(&red_first, fb);
  __syncthreads();
  if (tid == 0) {
    const uint64_t total =
        a.nblocks ? (__hip_atomic_load(&a.inc[a.nblocks - 1], __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT) &
                     ((uint64_t{1} << 36) - 1))
                  : 0;
    lvkv_log_report* r = a.r;
    r->status = total > a.capacity ? LVKV_LOG_CAPACITY : LVKV_OK;
    r->nblocks = a.nblocks;
    r->nrecords = static_cast<uint32_t>(total);
    r->ngood = static_cast<uint32_t>(red_good);
    r->ncorrupt = red_corrupt;
    r->first_bad_block = red_first;
    r->dropped_bytes = red_drop;
    r->count_ = total > a.capacity ? 0u : static_cast<uint32_t>(total);
    r->reserved_ = 0;
  }
}

}  // namespace

uint32_t next_log_generation() {
  static std::atomic<uint32_t> g{0};
  uint32_t v;
  do {
    v = (g.fetch_add(1, std::memory_order_relaxed) + 1) & 0x3ffffffu;
  } while (v == 0);
  return v;
}

#ifdef LVKV_PROBE_BUILD
uint64_t* g_log_stamps = nullptr;  // lvkv_debug_log_stamps
uint32_t g_log_knobs = 0;          // lvkv_debug_log_knobs
#endif

size_t log_scratch_bytes(uint64_t size) {
  const uint64_t nblocks = (size + kLogBlock - 1) / kLogBlock;
  return 16 + static_cast<size_t>(nblocks) * 20 + 8;
}

// `scratch`: log_scratch_bytes(size) bytes, 8-byte aligned, its first word 0
// (zeroed when allocated; every call leaves it at 0), used by one stream.
hipError_t launch_log_blocks(const uint8_t* file, uint64_t size, uint64_t* hdr_off,
                             uint32_t* actual, uint8_t* rec_status, uint32_t capacity,
                             uint8_t* block_status, uint32_t* block_drop, lvkv_log_report* r,
                             const uint32_t* zpow, const uint32_t* lane_cols, int cus,
                             void* scratch, uint32_t* events, hipStream_t stream) {
  const uint32_t nblocks = static_cast<uint32_t>((size + kLogBlock - 1) / kLogBlock);
  LogArgs a;
  memset(&a, 0, sizeof(a));
  a.file = file;
  a.size = size;
  a.nblocks = nblocks;
  a.capacity = capacity;
  a.gen = next_log_generation();
  a.hdr_off = hdr_off;
  a.actual = actual;
  a.rec_status = rec_status;
  a.block_status = block_status;
  a.block_drop = block_drop;
  a.r = r;
  a.done = static_cast<uint64_t*>(scratch);
  a.agg = a.done + 2;
  a.inc = a.agg + nblocks;
  a.good = reinterpret_cast<uint32_t*>(a.inc + nblocks);
  a.zpow = zpow;
  a.lane_cols = lane_cols;
  a.events = events;
#ifdef LVKV_PROBE_BUILD
  a.stamps = g_log_stamps;
  a.knobs = g_log_knobs;
#endif
  // every workgroup resident at once (one per CU): a placement only waits on
  // block counts, and every block is walked an iteration before it is placed
  const uint32_t groups = max(1u, min(nblocks, static_cast<uint32_t>(cus)));
  hipLaunchKernelGGL(log_verify_kernel, dim3(groups), dim3(kVThreads), 0, stream, a);
  return hipGetLastError();
}

}  // namespace lvkv
