// Zstd block compressor on the device (the write side
// of kZstdCompression): port::Zstd_Compress (port/port_stdcxx.h:133-161) as
// TableBuilder::WriteBlock calls it (table/table_builder.cc:172-185) --
// ZSTD_getCParams(level, max(n, 1), 0), ZSTD_CCtx_setCParams, ZSTD_compress2.
// The frames are byte-identical to libzstd 1.4.9's (the library the image
// carries); oracle/zstd_encoder.py restates that library's code for the
// parameters this call sequence produces under ZSTD_fast (levels <= 1 at any
// size, level 2 outside 128-256 KiB; LevelDB's default level is 1) and is
// pinned to it byte for byte (tests/test_zstd_write.py).
//
// One wave per block (64-thread workgroups); the block, its hash table, its
// literals and its sequences in LDS. The match finder
// (ZSTD_compressBlock_fast_generic) is a chain -- each step's table reads
// see every earlier step's writes, and a match moves the next step -- so it
// runs 64 steps a window, one a lane:
//   - step j's positions (ip0, ip0 + 1) do not depend on the data: step =
//     (ip0 - anchor) >> 7 + stepSize, a closed form per lane;
//   - its repcode test at ip0 + 2 reads only the input;
//   - its two table reads see the table before the window, or the latest
//     earlier step of the window with the same hash. A 1024-slot LDS scratch
//     keeps the first writer per (hash & 1023) by an atomic min: a read with
//     no earlier writer in its slot is exact; the few others are resolved
//     one by one with ballots on the full hash;
//   - the window's table writes (each hash's last writer up to the hit, by an
//     atomic max over the same slots) go in once.
// The entropy stage (ZSTD_entropyCompressSequences) is a chain of small
// serial decisions around parallel parts: the lanes count, sort and pack
// (Huffman codes 16 lanes a stream with atomic ORs into LDS words, FSE table
// spreads by ballot ranks); the wave runs the tree build, the normalisation
// and the three interleaved FSE state chains.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lvkv_zstd.h"

namespace lvkv {
namespace {

constexpr uint32_t kTags = 1024;  // window-scratch slots (u32)
constexpr uint32_t kLitStage = 32;  // the literals' offset in the frame slot (past the header)

__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
// Every lane's LDS operations so far are ordered before what follows. The
// workgroup is one wave, and one wave's LDS instructions execute in issue
// order (the counted lgkmcnt waits rest on it), so a later LDS access of any
// lane sees every earlier one: only the compiler must not move LDS accesses
// across this point -- no lgkmcnt(0) wait, which __syncthreads() would add
// (the loaded values' own waits stay). The CPU SIMT emulator (threads, not
// one instruction stream) keeps the barrier.
__device__ __forceinline__ void lds_sync() {
#ifdef LVKV_SIMT_EMU
  __syncthreads();
#else
  asm volatile("" ::: "memory");
#endif
}

__host__ __device__ __forceinline__ uint32_t hibit(uint32_t v) { return 31u - __builtin_clz(v); }

__device__ __forceinline__ uint32_t ld32(const uint8_t* b, uint32_t p) {
  const uint32_t* d = reinterpret_cast<const uint32_t*>(b + (p & ~3u));
  return __builtin_amdgcn_alignbyte(d[1], d[0], p & 3u);
}
__device__ __forceinline__ uint64_t ld64(const uint8_t* b, uint32_t p) {
  const uint32_t* d = reinterpret_cast<const uint32_t*>(b + (p & ~3u));
  const uint32_t s = p & 3u;
  const uint32_t lo = __builtin_amdgcn_alignbyte(d[1], d[0], s);
  const uint32_t hi = __builtin_amdgcn_alignbyte(d[2], d[1], s);
  return (static_cast<uint64_t>(hi) << 32) | lo;
}

__device__ __forceinline__ void stage(uint8_t* dst, const uint8_t* src, uint32_t n, uint32_t pad,
                                      uint32_t lane) {
  const uint32_t mis = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(src)) & 3u;
  const uint32_t* s = reinterpret_cast<const uint32_t*>(src - mis);
  const uint32_t nd = (n + 3u) >> 2;
  for (uint32_t i = lane; i < nd; i += 64) {
    const uint32_t lo = s[i];
    const uint32_t hi = (mis != 0 && 4u * (i + 1u) < mis + n) ? s[i + 1] : 0u;
    reinterpret_cast<uint32_t*>(dst)[i] = __builtin_amdgcn_alignbyte(hi, lo, mis);
  }
  for (uint32_t i = n + lane; i < n + pad; i += 64) dst[i] = 0;
}

// ---- parameters (ZSTD_getCParams + ZSTD_adjustCParams, 1.4.9) -------------

}  // namespace

// W | H << 8 | minMatch << 16 of ZSTD_defaultCParameters' fast rows; 0 where
// the strategy is not ZSTD_fast. Table 0: > 256 KiB, 1: <= 256 KiB, 2: <=
// 128 KiB, 3: <= 16 KiB; row 0 is the base row of the negative levels.
__host__ __device__ __forceinline__ uint32_t zstd_fast_row(uint32_t tid, uint32_t row) {
  constexpr uint32_t r00 = 19 | 13 << 8 | 6 << 16, r01 = 19 | 14 << 8 | 7 << 16,
                     r02 = 20 | 16 << 8 | 6 << 16;
  constexpr uint32_t r10 = 18 | 13 << 8 | 5 << 16, r11 = 18 | 14 << 8 | 6 << 16;
  constexpr uint32_t r20 = 17 | 12 << 8 | 5 << 16, r21 = 17 | 13 << 8 | 6 << 16,
                     r22 = 17 | 15 << 8 | 5 << 16;
  constexpr uint32_t r30 = 14 | 13 << 8 | 5 << 16, r31 = 14 | 15 << 8 | 5 << 16,
                     r32 = 14 | 15 << 8 | 4 << 16;
  switch (tid * 3 + row) {
    case 0: return r00;
    case 1: return r01;
    case 2: return r02;
    case 3: return r10;
    case 4: return r11;
    case 6: return r20;
    case 7: return r21;
    case 8: return r22;
    case 9: return r30;
    case 10: return r31;
    case 11: return r32;
    default: return 0;
  }
}

struct ZParams {
  uint32_t wlog, hlog, mls, tl, ok;
};

// The parameters ZSTD_compress2 runs with for port::Zstd_Compress(level, n
// bytes): getCParams(level, max(n, 1)) set field by field over the context's
// level-3 row, adjusted to the pledged size (the same fit again).
__host__ __device__ __forceinline__ ZParams zstd_port_params(int level, uint32_t n) {
  ZParams p{0, 0, 0, 0, 0};
  if (level == 0 || level > 2) return p;
  const uint32_t s = n ? n : 1u;
  const uint32_t tid = (s <= 262144u) + (s <= 131072u) + (s <= 16384u);
  const uint32_t row = zstd_fast_row(tid, level < 0 ? 0u : static_cast<uint32_t>(level));
  if (row == 0) return p;
  uint32_t w = row & 255u, h = (row >> 8) & 255u;
  const uint32_t mm = row >> 16;
  const uint32_t srclog = s < 64 ? 6u : hibit(s - 1) + 1u;
  if (w > srclog) w = srclog;
  if (h > w + 1) h = w + 1;
  if (w < 10) w = 10;
  p.wlog = w;
  p.hlog = h;
  p.mls = mm < 4 ? 4u : (mm > 7 ? 7u : mm);  // ZSTD_compressBlock_fast: 3 -> 4
  p.tl = level < 0 ? (level < -131072 ? 131072u : static_cast<uint32_t>(-level)) : 0u;
  p.ok = 1;
  return p;
}

namespace {

// ---- LDS layout -------------------------------------------------------------

// entropy scratch (over the hash table's region once the matcher is done)
constexpr uint32_t kECnt = 0;        // u32[256] counts
constexpr uint32_t kEHuf = 1024;     // u32[256] code | nbBits << 16
constexpr uint32_t kEStLL = 2048;    // u16[512] FSE next states
constexpr uint32_t kEStML = 3072;    // u16[512]
constexpr uint32_t kEStOF = 4096;    // u16[256]
constexpr uint32_t kEStW = 4608;     // u16[64]
constexpr uint32_t kENxt = 4864;     // u16[64] per-symbol next slot
constexpr uint32_t kESpread = 4992;  // u8[512] symbol of each spread rank
constexpr uint32_t kEPosSym = 5504;  // u8[512] symbol of each table position
constexpr uint32_t kEWts = 6016;     // u8[512] the Huffman weights' FSE form
constexpr uint32_t kECodes = 6528;   // u8[3][smax]: LL, OF, ML codes
constexpr uint32_t round16(uint32_t x) { return (x + 15u) & ~15u; }

struct ZcArgs {
  const uint8_t* src;
  const uint64_t* src_off;
  const uint32_t* src_len;
  uint8_t* dst;
  const uint64_t* dst_off;
  uint32_t* dst_len;
  uint8_t* status;
  uint32_t nblocks;
  int32_t level;
  uint32_t max_len;     // blocks longer are TOO_LARGE
  uint64_t dst_stride;  // dst_off == nullptr: block b's frame at b * dst_stride
  // LDS offsets
  uint32_t o_tbl, o_tag, o_lit, o_sll, o_sof, smax;
  uint64_t* stamps;  // probe build: 16 clock stamps a block (nullptr: none)
};

// s_memtime into stamp slot k of the block's LDS stamp area (probe build
// only; copied to a.stamps at the end, so that no global store or pointer
// test sits between the phases)
#ifndef ZC_STAMP_MASK
#define ZC_STAMP_MASK 0xFFFFu
#endif
__device__ __forceinline__ void zcstamp(uint64_t* slot, uint32_t k) {
#ifdef LVKV_PROBE_BUILD
  if (((ZC_STAMP_MASK >> k) & 1u) && threadIdx.x == 0) slot[k] = __builtin_amdgcn_s_memtime();
#else
  (void)slot;
  (void)k;
#endif
}

// ---- LL / ML codes (ZSTD_LLcode / ZSTD_MLcode) -----------------------------

__device__ __forceinline__ uint32_t ll_code(uint32_t ll) {
  if (ll > 63) return hibit(ll) + 19u;
  if (ll < 16) return ll;
  if (ll < 24) return 16u + ((ll - 16u) >> 1);
  if (ll < 32) return 20u + ((ll - 24u) >> 2);
  if (ll < 40) return 22u;
  return ll < 48 ? 23u : 24u;
  // (LL_Code: 16,16,17,17,18,18,19,19, 20 x4, 21 x4, 22 x8, 23 x8, 24 x16)
}
__device__ __forceinline__ uint32_t ml_code(uint32_t ml) {
  if (ml > 127) return hibit(ml) + 36u;
  if (ml < 32) return ml;
  if (ml < 40) return 32u + ((ml - 32u) >> 1);
  if (ml < 48) return 36u + ((ml - 40u) >> 2);
  if (ml < 64) return 38u + ((ml - 48u) >> 3);
  return ml < 80 ? 40u : (ml < 96 ? 41u : 42u);
}
__device__ __forceinline__ uint32_t ll_bits(uint32_t c) {
  return c < 16 ? 0u : (c < 20 ? 1u : (c < 22 ? 2u : (c < 24 ? 3u : (c == 24 ? 4u : c - 19u))));
}
__device__ __forceinline__ uint32_t ml_bits(uint32_t c) {
  return c < 32 ? 0u
                : (c < 36 ? 1u : (c < 38 ? 2u : (c < 40 ? 3u : (c < 42 ? 4u : (c == 42 ? 5u : c - 36u)))));
}

// ---- bit writer (BIT_CStream: LSB first) into an LDS byte buffer ----------
// Uniform: every lane holds the same state; lane 0 stores whole dwords.

struct BitW {
  uint8_t* out;  // dword-aligned base
  uint32_t d;    // dword index of the dword being filled
  uint64_t acc;  // pending bits, bit 0 = bit 32 d
  uint32_t n;    // pending bits count (< 32 between adds)
  uint32_t d0;   // the first dword, whose low `keep` bytes hold earlier data
  uint32_t keep;
};
__device__ __forceinline__ void bw_init(BitW& w, uint8_t* out, uint32_t byte_pos) {
  w.out = out;
  w.d = byte_pos >> 2;
  w.d0 = w.d;
  w.n = 8u * (byte_pos & 3u);
  w.keep = byte_pos & 3u;
  w.acc = 0;
}
__device__ __forceinline__ void bw_put(BitW& w, uint32_t lane, uint32_t v32) {
  uint32_t* o = reinterpret_cast<uint32_t*>(w.out) + w.d;
  if (w.keep && w.d == w.d0) {  // (every write of the first dword, flushes included)
    const uint32_t m = (1u << (8u * w.keep)) - 1u;
    v32 = (*o & m) | (v32 & ~m);
  }
  if (lane == 0) *o = v32;
}
__device__ __forceinline__ void bw_add(BitW& w, uint64_t v, uint32_t nb, uint32_t lane) {
  if (nb == 0) return;
  w.acc |= (v & ((uint64_t{1} << nb) - 1u)) << w.n;
  w.n += nb;
  while (w.n >= 32) {
    bw_put(w, lane, static_cast<uint32_t>(w.acc));
    ++w.d;
    w.acc >>= 32;
    w.n -= 32;
  }
}
// the bytes written up to now counted from byte_pos0 (pending bits rounded up)
__device__ __forceinline__ uint32_t bw_end(const BitW& w) { return 4u * w.d + ((w.n + 7u) >> 3); }
__device__ __forceinline__ void bw_flush(BitW& w, uint32_t lane) {
  if (w.n) bw_put(w, lane, static_cast<uint32_t>(w.acc));
}

// ---- FSE (fse_compress.c) ---------------------------------------------------

__constant__ uint32_t kRtb[8] = {0, 473195, 504333, 520860, 550000, 700000, 750000, 830000};

__device__ __forceinline__ uint32_t fse_min_log(uint32_t src, uint32_t max_sym) {
  const uint32_t a = hibit(src) + 1u, b = hibit(max_sym) + 2u;
  return a < b ? a : b;
}
__device__ __forceinline__ uint32_t fse_opt_log(uint32_t max_log, uint32_t src, uint32_t max_sym,
                                                uint32_t minus) {
  const uint32_t mbs = hibit(src - 1u) - minus;  // (src >= 2)
  uint32_t tl = max_log;
  if (mbs < tl) tl = mbs;
  const uint32_t mb = fse_min_log(src, max_sym);
  if (mb > tl) tl = mb;
  if (tl < 5) tl = 5;
  if (tl > 12) tl = 12;
  return tl;
}

// FSE_normalizeCount (+ FSE_normalizeM2) over counts held a symbol a lane
// (cnt, symbols < 64): returns this lane's normalized count (0 past
// max_sym). The wave works on the counts together; the serial parts are
// reductions and ballots.
__device__ __forceinline__ int32_t fse_normalize(uint32_t cnt, uint32_t tl, uint32_t total, uint32_t max_sym,
                                 bool low_prob, uint32_t lane) {
  const int32_t low = low_prob ? -1 : 1;
  const uint32_t scale = 62u - tl;
  const uint64_t step = (uint64_t{1} << 62) / total;
  const uint64_t vstep = uint64_t{1} << (scale - 20u);
  const uint32_t lowt = total >> tl;
  // every lane its own symbol's share (FSE_normalizeCount's loop body)
  int32_t p = 0, used = 0;
  bool big = false;
  if (lane <= max_sym && cnt != 0) {
    if (cnt <= lowt) {
      p = low;
      used = 1;
    } else {
      const uint64_t x = static_cast<uint64_t>(cnt) * step;
      uint32_t q = static_cast<uint32_t>(x >> scale);
      if (q < 8) {
        const uint64_t rest = vstep * kRtb[q];
        q += (x - (static_cast<uint64_t>(q) << scale)) > rest ? 1u : 0u;
      }
      p = static_cast<int32_t>(q);
      used = p;
      big = true;
    }
  }
  int32_t sum = used;
  for (uint32_t dd = 32; dd >= 1; dd >>= 1) sum += __shfl_xor(sum, dd);
  const int32_t still = (1 << tl) - static_cast<int32_t>(uni(static_cast<uint32_t>(sum)));
  // the first symbol of the largest share (strictly larger replaces)
  int32_t best = big ? p : 0;
  for (uint32_t dd = 32; dd >= 1; dd >>= 1) {
    const int32_t o = __shfl_xor(best, dd);
    best = o > best ? o : best;
  }
  const int32_t largest_p = static_cast<int32_t>(uni(static_cast<uint32_t>(best)));
  const uint64_t lm = __ballot(big && p == largest_p && largest_p > 0);
  const uint32_t largest = lm ? static_cast<uint32_t>(__builtin_ctzll(lm)) : 0u;
  const int32_t nl = static_cast<int32_t>(uni(__builtin_amdgcn_readlane(static_cast<uint32_t>(p), largest)));
  if (-still < (nl >> 1)) return lane == largest ? p + still : p;
  // FSE_normalizeM2
  const int16_t kNA = -2;
  uint32_t distributed = 0;
  uint32_t tot = total;
  uint32_t low_one = static_cast<uint32_t>((static_cast<uint64_t>(total) * 3u) >> (tl + 1u));
  int32_t q = 0;
  bool counted = false;
  if (lane <= max_sym) {
    if (cnt == 0) {
      q = 0;
    } else if (cnt <= lowt) {
      q = low;
      counted = true;
    } else if (cnt <= low_one) {
      q = 1;
      counted = true;
    } else {
      q = kNA;
    }
  }
  {
    const uint64_t m = __ballot(counted);
    distributed = __popcll(m);
    uint32_t sub = counted ? cnt : 0u;
    for (uint32_t dd = 32; dd >= 1; dd >>= 1) sub += __shfl_xor(sub, dd);
    tot -= uni(sub);
  }
  uint32_t to_dist = (1u << tl) - distributed;
  if (to_dist != 0) {
    if (tot / to_dist > low_one) {
      low_one = static_cast<uint32_t>((static_cast<uint64_t>(tot) * 3u) / (to_dist * 2u));
      const bool now = q == kNA && cnt <= low_one;
      if (now) q = 1;
      const uint64_t m = __ballot(now);
      distributed += __popcll(m);
      uint32_t sub = now ? cnt : 0u;
      for (uint32_t dd = 32; dd >= 1; dd >>= 1) sub += __shfl_xor(sub, dd);
      tot -= uni(sub);
      to_dist = (1u << tl) - distributed;
    }
    if (distributed == max_sym + 1u) {
      uint32_t mc = lane <= max_sym ? cnt : 0u;
      for (uint32_t dd = 32; dd >= 1; dd >>= 1) {
        const uint32_t o = __shfl_xor(mc, dd);
        mc = o > mc ? o : mc;
      }
      mc = uni(mc);
      const uint64_t m = __ballot(lane <= max_sym && cnt == mc && mc > 0);
      const uint32_t mv = m ? static_cast<uint32_t>(__builtin_ctzll(m)) : 0u;
      if (lane == mv) q += static_cast<int32_t>(to_dist);
    } else if (tot == 0) {
      // round robin over the positive ones
      const uint64_t pos = __ballot(lane <= max_sym && q > 0);
      const uint32_t np = __popcll(pos);
      if (np) {
        const uint32_t full = to_dist / np, rem = to_dist % np;
        const uint32_t rank = __popcll(pos & ((uint64_t{1} << lane) - 1u));
        if ((pos >> lane) & 1u) q += static_cast<int32_t>(full + (rank < rem ? 1u : 0u));
      }
    } else {
      const uint32_t vlog = 62u - tl;
      const uint64_t mid = (uint64_t{1} << (vlog - 1u)) - 1u;
      const uint64_t rstep = (((uint64_t{1} << vlog) * to_dist) + mid) / tot;
      // serial over the NOT_YET_ASSIGNED symbols (their running total)
      uint64_t tmp = mid;
      const uint64_t na = __ballot(q == kNA);
      uint64_t rest = na;
      while (rest) {
        const uint32_t s = static_cast<uint32_t>(__builtin_ctzll(rest));
        rest &= rest - 1u;
        const uint32_t cs = uni(__builtin_amdgcn_readlane(cnt, s));
        const uint64_t end = tmp + static_cast<uint64_t>(cs) * rstep;
        const uint32_t wgt = static_cast<uint32_t>(end >> vlog) - static_cast<uint32_t>(tmp >> vlog);
        if (lane == s) q = static_cast<int32_t>(wgt);
        tmp = end;
      }
    }
  }
  return lane <= max_sym ? q : 0;
}

// FSE_writeNCount of the normalized counts (a symbol a lane, symbols
// 0..max_sym) at accuracy tl through bw. Uniform serial code on readlanes.
__device__ __forceinline__ void fse_write_ncount(int32_t normv, uint32_t max_sym, uint32_t tl, BitW& bw,
                                 uint32_t lane) {
  bw_add(bw, tl - 5u, 4, lane);
  int32_t remaining = (1 << tl) + 1;
  int32_t threshold = 1 << tl;
  uint32_t nb = tl + 1u;
  uint32_t s = 0;
  const uint32_t alpha = max_sym + 1u;
  const uint64_t nzm = __ballot(normv != 0);
  bool prev0 = false;
  while (s < alpha && remaining > 1) {
    if (prev0) {
      uint32_t start = s;
      const uint64_t ahead = nzm >> s;  // the next non-zero symbol
      s = ahead ? s + static_cast<uint32_t>(__builtin_ctzll(ahead)) : alpha;
      if (s >= alpha) break;
      while (s >= start + 24u) {
        start += 24u;
        bw_add(bw, 0xFFFFu, 16, lane);
      }
      while (s >= start + 3u) {
        start += 3u;
        bw_add(bw, 3u, 2, lane);
      }
      bw_add(bw, s - start, 2, lane);
    }
    int32_t count = static_cast<int32_t>(__builtin_amdgcn_readlane(static_cast<uint32_t>(normv), s));
    ++s;
    const int32_t mx = (2 * threshold - 1) - remaining;
    remaining -= count < 0 ? -count : count;
    ++count;
    if (count >= threshold) count += mx;
    bw_add(bw, static_cast<uint32_t>(count), nb - (count < mx ? 1u : 0u), lane);
    prev0 = count == 1;
    if (remaining < 1) break;  // (a bad distribution: FSE_writeNCount's error)
    while (remaining < threshold) {
      --nb;
      threshold >>= 1;
    }
  }
}

// FSE_buildCTable_wksp for norm[0..max_sym] (max_sym < 64) at accuracy tl:
// next states into st[], and per symbol (lane s) the transform dnb / dfs.
__device__ __forceinline__ void fse_build_ctable(int32_t normv, uint32_t max_sym, uint32_t tl, uint16_t* st,
                                 uint8_t* ent, uint32_t lane, uint32_t* dnb_out, int32_t* dfs_out) {
  uint8_t* spread = ent + kESpread;
  uint8_t* psym = ent + kEPosSym;
  uint16_t* nxt = reinterpret_cast<uint16_t*>(ent + kENxt);
  const uint32_t size = 1u << tl;
  const uint64_t below = (uint64_t{1} << lane) - 1u;
  const int32_t c = lane <= max_sym ? normv : 0;
  const bool lowp = c == -1;
  const uint32_t take = lowp ? 1u : (c > 0 ? static_cast<uint32_t>(c) : 0u);
  uint32_t cum = take;
  for (uint32_t dd = 1; dd < 64; dd <<= 1) {
    const uint32_t v = __shfl_up(cum, dd);
    if (lane >= dd) cum += v;
  }
  const uint32_t cumul = cum - take;  // the symbol's first slot (cumul[s])
  const uint64_t lm = __ballot(lowp);
  const uint32_t kept = size - static_cast<uint32_t>(__popcll(lm));  // highThreshold + 1
  // symbol of every spread rank: the positive counts laid end to end
  const uint32_t pc = c > 0 ? static_cast<uint32_t>(c) : 0u;
  uint32_t pcum = pc;
  for (uint32_t dd = 1; dd < 64; dd <<= 1) {
    const uint32_t v = __shfl_up(pcum, dd);
    if (lane >= dd) pcum += v;
  }
  for (uint32_t r = lane; r < size; r += 64) spread[r] = 0;
  lds_sync();
  if (pc) spread[pcum - pc] = static_cast<uint8_t>(lane);
  lds_sync();
  uint32_t carry = 0;
  for (uint32_t r0 = 0; r0 < kept; r0 += 64) {
    const uint32_t r = r0 + lane;
    uint32_t v = r < kept ? spread[r] : 0u;
    v = v > carry ? v : carry;
    for (uint32_t dd = 1; dd < 64; dd <<= 1) {
      const uint32_t o = __shfl_up(v, dd);
      if (lane >= dd && o > v) v = o;
    }
    carry = uni(__shfl(v, 63));
    lds_sync();
    if (r < kept) spread[r] = static_cast<uint8_t>(v);
    lds_sync();
  }
  // rank k lands at the k-th j (j * step & mask) below kept; the
  // low-probability symbols fill the top in symbol order
  const uint32_t step = (size >> 1) + (size >> 3) + 3u;
  const uint32_t mask = size - 1u;
  uint32_t rank = 0;
  for (uint32_t j0 = 0; j0 < size; j0 += 64) {
    const uint32_t j = j0 + lane;
    const uint32_t t = (j * step) & mask;
    const bool keep = j < size && t < kept;
    const uint64_t m = __ballot(keep);
    if (keep) psym[t] = spread[rank + __popcll(m & below)];
    rank += __popcll(m);
  }
  if (lowp) psym[size - 1u - __popcll(lm & below)] = static_cast<uint8_t>(lane);
  if (lane <= max_sym) nxt[lane] = static_cast<uint16_t>(cumul);
  lds_sync();
  // tableU16[cumul[s]++] = size + u in position order: a position's slot is
  // cumul[s] plus its rank among the earlier positions of s
  for (uint32_t u0 = 0; u0 < size; u0 += 64) {
    const uint32_t u = u0 + lane;
    const bool in = u < size;
    const uint32_t s = in ? psym[u] : 0x1000u;
    uint64_t todo = __ballot(in), peers = 0;
    while (todo) {
      const uint32_t sl = uni(__builtin_amdgcn_readlane(s, static_cast<uint32_t>(__builtin_ctzll(todo))));
      const uint64_t m = __ballot(s == sl);
      if (s == sl) peers = m;
      todo &= ~m;
    }
    const uint32_t before = __popcll(peers & below);
    const bool last = in && (peers >> lane) == 1u;
    const uint32_t slot = (in ? nxt[s] : 0u) + before;
    lds_sync();
    if (last) nxt[s] = static_cast<uint16_t>(slot + 1u);
    if (in) st[slot] = static_cast<uint16_t>(size + u);
    lds_sync();
  }
  // symbol transforms
  uint32_t dnb = 0;
  int32_t dfs = 0;
  if (lane <= max_sym) {
    if (c == 0) {
      dnb = ((tl + 1u) << 16) - (1u << tl);
    } else if (c == -1 || c == 1) {
      dnb = (tl << 16) - (1u << tl);
      dfs = static_cast<int32_t>(cumul) - 1;
    } else {
      const uint32_t mbo = tl - hibit(static_cast<uint32_t>(c) - 1u);
      dnb = (mbo << 16) - (static_cast<uint32_t>(c) << mbo);
      dfs = static_cast<int32_t>(cumul) - c;
    }
  }
  *dnb_out = dnb;
  *dfs_out = dfs;
}

// FSE state coder over a table whose transforms sit a symbol a lane. A
// table of <= 64 states is also held a state a lane (stv), so that the
// serial coders read it with v_readlane instead of an LDS round trip.
struct FseC {
  const uint16_t* st;
  uint32_t stv;  // lane u: st[u] (reg tables)
  uint32_t dnb;  // lane s: symbol s's deltaNbBits
  int32_t dfs;   // lane s: deltaFindState
  uint32_t log;
  bool reg;
};
__device__ __forceinline__ void fse_regs(FseC& t, uint32_t lane) {
  t.reg = t.log <= 6;
  if (t.reg) t.stv = lane < (1u << t.log) ? t.st[lane] : 0u;
}
__device__ __forceinline__ uint32_t fse_state(const FseC& t, int32_t idx) {
  return t.reg ? __builtin_amdgcn_readlane(t.stv, static_cast<uint32_t>(idx)) : uni(t.st[idx]);
}
__device__ __forceinline__ uint32_t fse_init(const FseC& t, uint32_t sym) {
  const uint32_t dnb = __builtin_amdgcn_readlane(t.dnb, sym);
  const int32_t dfs = static_cast<int32_t>(__builtin_amdgcn_readlane(static_cast<uint32_t>(t.dfs), sym));
  const uint32_t nbo = (dnb + (1u << 15)) >> 16;
  const uint32_t v = (nbo << 16) - dnb;
  return fse_state(t, static_cast<int32_t>(v >> nbo) + dfs);
}
__device__ __forceinline__ uint32_t fse_enc(const FseC& t, uint32_t state, uint32_t sym, BitW& bw,
                                            uint32_t lane) {
  const uint32_t dnb = __builtin_amdgcn_readlane(t.dnb, sym);
  const int32_t dfs = static_cast<int32_t>(__builtin_amdgcn_readlane(static_cast<uint32_t>(t.dfs), sym));
  const uint32_t nbo = (state + dnb) >> 16;
  bw_add(bw, state, nbo, lane);
  return fse_state(t, static_cast<int32_t>(state >> nbo) + dfs);
}

// ---- Huffman (huf_compress.c) -----------------------------------------------

struct HNode {
  uint32_t count;
  uint16_t parent;
  uint8_t byte;
  uint8_t nb;
};

// HUF_setMaxHeight over node[0..last] (node = huffNode, node[-1] the barrier)
__device__ __forceinline__ uint32_t huf_set_max_height(HNode* node, int32_t last, uint32_t max_nb) {
  const uint32_t largest = uni(node[last].nb);
  if (largest <= max_nb) return largest;
  int32_t total = 0;
  const int32_t base_cost = 1 << (largest - max_nb);
  int32_t n = last;
  while (uni(node[n].nb) > max_nb) {
    total += base_cost - (1 << (largest - uni(node[n].nb)));
    node[n].nb = static_cast<uint8_t>(max_nb);
    lds_sync();
    --n;
  }
  while (n >= 0 && uni(node[n].nb) == max_nb) --n;
  total >>= (largest - max_nb);
  constexpr uint32_t kNo = 0xF0F0F0F0u;
  uint32_t rl[14];
#pragma unroll
  for (int i = 0; i < 14; ++i) rl[i] = kNo;
  {
    uint32_t cur = max_nb;
    for (int32_t pos = n; pos >= 0; --pos) {
      const uint32_t b = uni(node[pos].nb);
      if (b >= cur) continue;
      cur = b;
      rl[max_nb - cur] = static_cast<uint32_t>(pos);
    }
  }
  while (total > 0) {
    uint32_t nbd = hibit(static_cast<uint32_t>(total)) + 1u;
    for (; nbd > 1; --nbd) {
      const uint32_t hi = rl[nbd], lo = rl[nbd - 1];
      if (hi == kNo) continue;
      if (lo == kNo) break;
      if (uni(node[hi].count) <= 2u * uni(node[lo].count)) break;
    }
    while (nbd <= 12 && rl[nbd] == kNo) ++nbd;
    total -= 1 << (nbd - 1u);
    if (rl[nbd - 1] == kNo) rl[nbd - 1] = rl[nbd];
    node[rl[nbd]].nb = static_cast<uint8_t>(uni(node[rl[nbd]].nb) + 1u);
    lds_sync();
    if (rl[nbd] == 0) {
      rl[nbd] = kNo;
    } else {
      rl[nbd] -= 1u;
      if (uni(node[rl[nbd]].nb) != max_nb - nbd) rl[nbd] = kNo;
    }
  }
  while (total < 0) {
    if (rl[1] == kNo) {
      while (n >= 0 && uni(node[n].nb) == max_nb) --n;
      node[n + 1].nb = static_cast<uint8_t>(uni(node[n + 1].nb) - 1u);
      lds_sync();
      rl[1] = static_cast<uint32_t>(n + 1);
      ++total;
      continue;
    }
    node[rl[1] + 1].nb = static_cast<uint8_t>(uni(node[rl[1] + 1].nb) - 1u);
    lds_sync();
    rl[1] += 1u;
    ++total;
  }
  return max_nb;
}

// 256-entry arrays held a value a lane in 4 VGPRs: element i at lane i & 63
// of register i >> 6 (i uniform).
__device__ __forceinline__ uint32_t rd256(const uint32_t (&a)[4], uint32_t i) {
  const uint32_t g = i >> 6;
  const uint32_t v = g == 0 ? a[0] : (g == 1 ? a[1] : (g == 2 ? a[2] : a[3]));
  return __builtin_amdgcn_readlane(v, i & 63u);
}
__device__ __forceinline__ void wr256(uint32_t (&a)[4], uint32_t i, uint32_t v) {
  const uint32_t g = i >> 6, l = i & 63u;
  const bool me = threadIdx.x == l;  // (v_cmp + v_cndmask: a lane write)
  a[0] = (g == 0 && me) ? v : a[0];
  a[1] = (g == 1 && me) ? v : a[1];
  a[2] = (g == 2 && me) ? v : a[2];
  a[3] = (g == 3 && me) ? v : a[3];
}
// lane-varying gather from a 256-entry register array
__device__ __forceinline__ uint32_t gather256(const uint32_t (&a)[4], uint32_t i) {
  const int addr = static_cast<int>((i & 63u) << 2);
  const uint32_t v0 = __builtin_amdgcn_ds_bpermute(addr, static_cast<int>(a[0]));
  const uint32_t v1 = __builtin_amdgcn_ds_bpermute(addr, static_cast<int>(a[1]));
  const uint32_t v2 = __builtin_amdgcn_ds_bpermute(addr, static_cast<int>(a[2]));
  const uint32_t v3 = __builtin_amdgcn_ds_bpermute(addr, static_cast<int>(a[3]));
  const uint32_t g = i >> 6;
  return g == 0 ? v0 : (g == 1 ? v1 : (g == 2 ? v2 : v3));
}

// HUF_buildCTable_wksp: counts a symbol a lane x 4 (c[g] for g * 64 + lane),
// symbols 0..max_sym. Codes go to huf[s] = code | nbBits << 16. Returns the
// table's max bits. The sorted leaves and the created nodes' counts live in
// registers: the merge is a chain of v_readlane and lane writes (no LDS
// round trip), recording only where each pick came from; the parents are
// then placed all at once and the depths found by pointer jumping. node0
// (LDS) serves the rank scatter, the parents' scatter and the rare
// HUF_setMaxHeight.
__device__ __forceinline__ uint32_t huf_build(const uint32_t (&c)[4], uint32_t max_sym, uint32_t max_nb,
                              HNode* node0, uint32_t* huf, uint32_t lane) {
  HNode* node = node0 + 1;
  // HUF_sort: decreasing count, ties in symbol order -- each symbol's rank
  uint32_t rank[4] = {0, 0, 0, 0};
#pragma unroll
  for (uint32_t g2 = 0; g2 < 4; ++g2) {
    if (g2 * 64u > max_sym) break;
    const uint32_t top = max_sym - g2 * 64u < 63u ? max_sym - g2 * 64u : 63u;
    for (uint32_t l = 0; l <= top; ++l) {
      const uint32_t t = g2 * 64u + l;
      const uint32_t ct = __builtin_amdgcn_readlane(c[g2], l);
#pragma unroll
      for (uint32_t g = 0; g < 4; ++g) {
        const uint32_t s = g * 64u + lane;
        rank[g] += (ct > c[g] || (ct == c[g] && t < s)) ? 1u : 0u;
      }
    }
  }
  uint32_t nnz = 0;
#pragma unroll
  for (uint32_t g = 0; g < 4; ++g) {
    const uint32_t s = g * 64u + lane;
    if (s <= max_sym) {
      node[rank[g]].count = c[g];
      node[rank[g]].byte = static_cast<uint8_t>(s);
    }
    nnz += __popcll(__ballot(s <= max_sym && c[g] != 0));
  }
  lds_sync();
  // the sorted leaves, a rank a lane
  uint32_t L[4], S[4];
#pragma unroll
  for (uint32_t g = 0; g < 4; ++g) {
    const uint32_t r = g * 64u + lane;
    L[g] = r <= max_sym ? node[r].count : 0u;
    S[g] = r <= max_sym ? node[r].byte : 0u;
  }
  const uint32_t non_null = nnz - 1u;  // (nnz >= 2: one symbol is the RLE case)
  constexpr uint32_t kBarrier = 1u << 31, kUnmade = 1u << 30;
  // The two-queue merge (sorted leaves from the smallest, created nodes in
  // order): created node k's count in IC (lane k & 63 of IC[k >> 6]), and
  // per step only which queue each of its two picks came from (DEC: bit 0
  // the first pick was a leaf, bit 1 the second), both lane writes into a
  // register fixed per group of 64 steps. The parents follow from
  // the pick order afterwards, all at once.
  uint32_t IC[4] = {kUnmade, kUnmade, kUnmade, kUnmade}, DEC[4] = {0, 0, 0, 0};
  const uint32_t root = non_null - 1u;  // the last created node
  int32_t low_s = static_cast<int32_t>(non_null);
  {
    const uint32_t c1 = rd256(L, non_null), c0 = rd256(L, non_null - 1u);
    IC[0] = lane == 0 ? c1 + c0 : IC[0];
    DEC[0] = lane == 0 ? 3u : DEC[0];  // node 0: the two smallest leaves
  }
  low_s -= 2;
  uint32_t low_n = 0;
  uint32_t cs = low_s >= 0 ? rd256(L, static_cast<uint32_t>(low_s)) : kBarrier;
  uint32_t cn = rd256(IC, 0);
#pragma unroll
  for (uint32_t g = 0; g < 4; ++g) {
    if (64u * g > root) break;
    for (uint32_t l = g == 0 ? 1u : 0u; l < 64u; ++l) {
      const uint32_t made = 64u * g + l;
      if (made > root) break;
      uint32_t c1, c2, dec = 0;
      if (cs < cn) {
        c1 = cs;
        dec = 1;
        --low_s;
        cs = low_s >= 0 ? rd256(L, static_cast<uint32_t>(low_s)) : kBarrier;
      } else {
        c1 = cn;
        ++low_n;
        cn = low_n < made ? rd256(IC, low_n) : kUnmade;
      }
      if (cs < cn) {
        c2 = cs;
        dec |= 2;
        --low_s;
        cs = low_s >= 0 ? rd256(L, static_cast<uint32_t>(low_s)) : kBarrier;
      } else {
        c2 = cn;
        ++low_n;
        cn = low_n < made ? rd256(IC, low_n) : kUnmade;
      }
      IC[g] = lane == l ? c1 + c2 : IC[g];
      DEC[g] = lane == l ? dec : DEC[g];
      if (low_n == made) cn = c1 + c2;
    }
  }
  // Parents from the pick order: step m's picks are slots 2m and 2m + 1; the
  // r-th leaf pick takes leaf non_null - r, the q-th created-node pick node
  // q, and both get parent m. Scattered through LDS (u8: parents <= 254),
  // after the sort's nodes.
  uint8_t* par_l = reinterpret_cast<uint8_t*>(node0 + 257);
  uint8_t* par_i = par_l + 256;
  {
    const uint64_t below = (uint64_t{1} << lane) - 1u;
    uint32_t carry = 0;
#pragma unroll
    for (uint32_t g = 0; g < 4; ++g) {
      const uint32_t m = 64u * g + lane;
      const bool on = m <= root;
      const bool l0 = on && (DEC[g] & 1u), l1 = on && (DEC[g] & 2u);
      const uint64_t b0 = __ballot(l0), b1 = __ballot(l1);
      const uint32_t pre = carry + __popcll(b0 & below) + __popcll(b1 & below);
      if (on) {
        const uint32_t r1 = pre + (l0 ? 1u : 0u);
        if (l0) par_l[non_null - pre] = static_cast<uint8_t>(m);
        else par_i[2u * m - pre] = static_cast<uint8_t>(m);
        if (l1) par_l[non_null - r1] = static_cast<uint8_t>(m);
        else par_i[2u * m + 1u - r1] = static_cast<uint8_t>(m);
      }
      carry += __popcll(b0) + __popcll(b1);
    }
  }
  lds_sync();
  uint32_t PL[4], PI[4];
#pragma unroll
  for (uint32_t g = 0; g < 4; ++g) {
    const uint32_t k = 64u * g + lane;
    PL[g] = k <= non_null ? par_l[k] : 0u;
    PI[g] = k < root ? par_i[k] : k;  // (the root and past it: their own parent)
  }
  // depths of the created nodes: pointer jumping to the root (8 rounds:
  // depth <= 254)
  uint32_t DI[4], AN[4];
#pragma unroll
  for (uint32_t g = 0; g < 4; ++g) {
    const uint32_t k = 64u * g + lane;
    DI[g] = k < root ? 1u : 0u;
    AN[g] = PI[g];
  }
  for (int round = 0; round < 8; ++round) {
    uint32_t nd[4], na[4];
#pragma unroll
    for (uint32_t g = 0; g < 4; ++g) {
      nd[g] = DI[g] + gather256(DI, AN[g]);
      na[g] = gather256(AN, AN[g]);
    }
#pragma unroll
    for (uint32_t g = 0; g < 4; ++g) {
      DI[g] = nd[g];
      AN[g] = na[g];
    }
  }
  uint32_t NB[4];
  uint32_t deepest = 0;
#pragma unroll
  for (uint32_t g = 0; g < 4; ++g) {
    const uint32_t r = g * 64u + lane;
    const uint32_t d = gather256(DI, PL[g]) + 1u;
    NB[g] = r <= non_null ? d : 0u;
  }
  deepest = rd256(NB, non_null);
  if (deepest > max_nb) {  // HUF_setMaxHeight (on the LDS nodes)
#pragma unroll
    for (uint32_t g = 0; g < 4; ++g) {
      const uint32_t r = g * 64u + lane;
      if (r <= max_sym) node[r].nb = static_cast<uint8_t>(NB[g]);
    }
    if (lane == 0) node0[0].nb = 0;
    lds_sync();
    max_nb = huf_set_max_height(node, static_cast<int32_t>(non_null), max_nb);
    lds_sync();
#pragma unroll
    for (uint32_t g = 0; g < 4; ++g) {
      const uint32_t r = g * 64u + lane;
      NB[g] = r <= non_null ? node[r].nb : 0u;
    }
  } else {
    max_nb = deepest;
  }
  // codes: valPerRank from the counts per bit length, then each symbol's
  // rank among the symbols of its length in symbol order
#pragma unroll
  for (uint32_t g = 0; g < 4; ++g) {
    const uint32_t r = g * 64u + lane;
    if (r <= max_sym) huf[S[g]] = NB[g] << 16;
  }
  lds_sync();
  uint32_t nbs[4];
#pragma unroll
  for (uint32_t g = 0; g < 4; ++g) {
    const uint32_t s = g * 64u + lane;
    nbs[g] = s <= max_sym ? huf[s] >> 16 : 0u;
  }
  uint32_t per[13];
#pragma unroll
  for (uint32_t k = 0; k < 13; ++k) {
    uint32_t t = 0;
#pragma unroll
    for (uint32_t g = 0; g < 4; ++g) t += __popcll(__ballot(nbs[g] == k && k != 0));
    per[k] = t;
  }
  uint32_t start[13];
  {
    uint32_t mn = 0;
#pragma unroll
    for (int32_t k = 12; k > 0; --k) {
      start[k] = 0;
      if (static_cast<uint32_t>(k) <= max_nb) {
        start[k] = mn;
        mn = (mn + per[k]) >> 1;
      }
    }
    start[0] = 0;
  }
  const uint64_t below = (uint64_t{1} << lane) - 1u;
#pragma unroll
  for (uint32_t g = 0; g < 4; ++g) {
    uint32_t code = 0;
#pragma unroll
    for (uint32_t k = 1; k < 13; ++k) {
      const bool mine = nbs[g] == k;
      const uint64_t m = __ballot(mine);
      if (mine) code = start[k] + __popcll(m & below);
      start[k] += __popcll(m);
    }
    const uint32_t s = g * 64u + lane;
    if (s <= max_sym) huf[s] = (code & 0xFFFFu) | (nbs[g] << 16);
  }
  lds_sync();
  return max_nb;
}

// ---- the literals section (ZSTD_compressLiterals) ---------------------------

__device__ __forceinline__ uint32_t raw_literals(uint8_t* out, const uint8_t* lits, uint32_t n, uint32_t lane) {
  const uint32_t fl = 1u + (n > 31) + (n > 4095);
  if (lane == 0) {
    if (fl == 1) {
      out[0] = static_cast<uint8_t>(n << 3);
    } else if (fl == 2) {
      const uint32_t h = (1u << 2) + (n << 4);
      out[0] = static_cast<uint8_t>(h);
      out[1] = static_cast<uint8_t>(h >> 8);
    } else {
      const uint32_t h = (3u << 2) + (n << 4);
      out[0] = static_cast<uint8_t>(h);
      out[1] = static_cast<uint8_t>(h >> 8);
      out[2] = static_cast<uint8_t>(h >> 16);
    }
  }
  for (uint32_t k = lane; k < n; k += 64) out[fl + k] = lits[k];
  lds_sync();
  return fl + n;
}

__device__ __forceinline__ uint32_t rle_literals(uint8_t* out, const uint8_t* lits, uint32_t n, uint32_t lane) {
  const uint32_t fl = 1u + (n > 31) + (n > 4095);
  if (lane == 0) {
    if (fl == 1) {
      out[0] = static_cast<uint8_t>(1u + (n << 3));
    } else if (fl == 2) {
      const uint32_t h = 1u + (1u << 2) + (n << 4);
      out[0] = static_cast<uint8_t>(h);
      out[1] = static_cast<uint8_t>(h >> 8);
    } else {
      const uint32_t h = 1u + (3u << 2) + (n << 4);
      out[0] = static_cast<uint8_t>(h);
      out[1] = static_cast<uint8_t>(h >> 8);
      out[2] = static_cast<uint8_t>(h >> 16);
    }
    out[fl] = lits[0];
  }
  lds_sync();
  return fl + 1u;
}

// Packs `count` (<= 256) bit chunks, chunk e = the low nb[e >> 6] bits of
// val[e >> 6] at lane e & 63, one after another from bit `bit0` of words
// (LDS; the bits below bit0 are kept, the rest of the words the stream
// covers are zeroed first): an exclusive scan of the counts places every
// chunk, and each lane ORs its chunks into the one or two words they touch.
// Chunks of 0-32 bits. Returns the bit after the last chunk.
__device__ __forceinline__ uint32_t pack_bits(uint32_t* words, uint32_t bit0, const uint32_t (&val)[4],
                                              const uint32_t (&nb)[4], uint32_t count, uint32_t lane) {
  uint32_t off[4];
  uint32_t carry = bit0;
#pragma unroll
  for (uint32_t g = 0; g < 4; ++g) {
    const uint32_t n = 64u * g + lane < count ? nb[g] : 0u;
    uint32_t incl = n;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
      const uint32_t v = __shfl_up(incl, d);
      if (lane >= d) incl += v;
    }
    off[g] = carry + incl - n;
    carry += uni(__shfl(incl, 63));
  }
  const uint32_t w0 = bit0 >> 5, w1 = (carry + 31u) >> 5;
  for (uint32_t k = w0 + lane; k < w1; k += 64) {
    const uint32_t keep = k == w0 ? (bit0 & 31u) : 0u;
    words[k] = keep ? words[k] & ((1u << keep) - 1u) : 0u;
  }
  lds_sync();
#pragma unroll
  for (uint32_t g = 0; g < 4; ++g) {
    const uint32_t n = 64u * g + lane < count ? nb[g] : 0u;
    if (n != 0) {
      const uint64_t v = static_cast<uint64_t>(val[g] & (n == 32u ? 0xFFFFFFFFu : (1u << n) - 1u))
                         << (off[g] & 31u);
      atomicOr(&words[off[g] >> 5], static_cast<uint32_t>(v));
      if ((off[g] & 31u) + n > 32u) atomicOr(&words[(off[g] >> 5) + 1u], static_cast<uint32_t>(v >> 32));
    }
  }
  lds_sync();
  return carry;
}

// HUF_writeCTable's weights through FSE (HUF_compressWeights) into buf (LDS,
// dword-aligned): returns the bytes (0: no FSE form). w[g] = weight of
// symbol g * 64 + lane for symbols < nw.
__device__ __forceinline__ uint32_t huf_compress_weights(const uint32_t (&w)[4], uint32_t nw, uint8_t* ent,
                                         uint8_t* buf, uint32_t lane) {
  if (nw <= 1) return 0;
  // histogram of the weights (0..12): a value a lane
  uint32_t cnt = 0;
#pragma unroll
  for (uint32_t v = 0; v < 13; ++v) {
    uint32_t t = 0;
#pragma unroll
    for (uint32_t g = 0; g < 4; ++g) t += __popcll(__ballot(g * 64u + lane < nw && w[g] == v));
    if (lane == v) cnt = t;
  }
  const uint64_t nzm = __ballot(lane < 13 && cnt != 0);
  const uint32_t max_sym = 63u - __builtin_clzll(nzm);
  uint32_t mc = cnt;
  for (uint32_t dd = 32; dd >= 1; dd >>= 1) {
    const uint32_t o = __shfl_xor(mc, dd);
    mc = o > mc ? o : mc;
  }
  mc = uni(mc);
  if (mc == nw || mc == 1) return 0;
  const uint32_t tl = fse_opt_log(6, nw, max_sym, 2);
  const int32_t normv = fse_normalize(cnt, tl, nw, max_sym, false, lane);
  BitW bw;
  bw_init(bw, buf, 0);
  fse_write_ncount(normv, max_sym, tl, bw, lane);
  bw_flush(bw, lane);
  lds_sync();
  const uint32_t nc = bw_end(bw);
  if (nw <= 2) return 0;  // (FSE_compress_usingCTable: no stream)
  FseC t;
  t.st = reinterpret_cast<uint16_t*>(ent + kEStW);
  t.log = tl;
  fse_build_ctable(normv, max_sym, tl, reinterpret_cast<uint16_t*>(ent + kEStW), ent, lane, &t.dnb,
                   &t.dfs);
  lds_sync();
  fse_regs(t, lane);
  // The weights from the end, two interleaved states (FSE_compress_usingCTable):
  // the states are two independent chains, so they run first, each step's
  // (bits, count) recorded in emission order; the lanes then pack the stream
  // at once (pack_bits). Chain A takes the indices with i = nw - 1 (mod 2),
  // chain B the others, each from its highest index down; emission step e
  // (e = 0..nw-3) encodes index nw - 3 - e: chain A's on even e. A is s1
  // when nw is odd, s2 when it is even.
  auto wat = [&](uint32_t i) -> uint32_t {
    const uint32_t g = i >> 6, l = i & 63u;
    const uint32_t v = g == 0 ? w[0] : (g == 1 ? w[1] : (g == 2 ? w[2] : w[3]));
    return uni(__builtin_amdgcn_readlane(v, l));
  };
  uint32_t sa = fse_init(t, wat(nw - 1u)), sb = fse_init(t, wat(nw - 2u));
  const bool odd = (nw & 1u) != 0;
  const uint32_t E = nw - 2u;
  // per step, in parallel: its symbol's (deltaNbBits, deltaFindState)
  uint32_t DNB[4], DFS[4];
#pragma unroll
  for (uint32_t g = 0; g < 4; ++g) {
    const uint32_t e = 64u * g + lane;
    // (every lane joins the gather: a lane-permute reads inactive lanes as 0)
    const uint32_t gw = gather256(w, e < E ? nw - 3u - e : 0u);
    const uint32_t sym = e < E ? gw : 0u;
    DNB[g] = __shfl(t.dnb, static_cast<int>(sym));
    DFS[g] = __shfl(static_cast<uint32_t>(t.dfs), static_cast<int>(sym));
  }
  // the two chains a step each per turn (independent: they overlap); each
  // step's state before it recorded at its lane
  uint32_t VAL[4] = {0, 0, 0, 0}, NBT[4] = {0, 0, 0, 0};
  auto step = [&](uint32_t st, uint32_t dnb, uint32_t dfs) -> uint32_t {
    const uint32_t nbo = (st + dnb) >> 16;
    return fse_state(t, static_cast<int32_t>(st >> nbo) + static_cast<int32_t>(dfs));
  };
#pragma unroll
  for (uint32_t g = 0; g < 4; ++g) {
    if (64u * g >= E) break;
    for (uint32_t l = 0; l < 64u; l += 2u) {
      const uint32_t e = 64u * g + l;
      if (e >= E) break;
      const uint32_t da = __builtin_amdgcn_readlane(DNB[g], l), fa = __builtin_amdgcn_readlane(DFS[g], l);
      VAL[g] = lane == l ? sa : VAL[g];
      if (e + 1u < E) {
        const uint32_t db = __builtin_amdgcn_readlane(DNB[g], l + 1u),
                       fb = __builtin_amdgcn_readlane(DFS[g], l + 1u);
        VAL[g] = lane == l + 1u ? sb : VAL[g];
        sa = step(sa, da, fa);
        sb = step(sb, db, fb);
      } else {
        sa = step(sa, da, fa);
      }
    }
  }
#pragma unroll
  for (uint32_t g = 0; g < 4; ++g) NBT[g] = 64u * g + lane < E ? (VAL[g] + DNB[g]) >> 16 : 0u;
  // the flush: s2 then s1, the end mark
  const uint32_t s2 = odd ? sb : sa, s1 = odd ? sa : sb;
  const uint32_t tail_v[3] = {s2, s1, 1u}, tail_n[3] = {tl, tl, 1u};
#pragma unroll
  for (uint32_t k = 0; k < 3; ++k) {
    const uint32_t e = E + k, g = e >> 6, l = e & 63u;
#pragma unroll
    for (uint32_t gg = 0; gg < 4; ++gg) {
      VAL[gg] = (gg == g && lane == l) ? tail_v[k] : VAL[gg];
      NBT[gg] = (gg == g && lane == l) ? tail_n[k] : NBT[gg];
    }
  }
  const uint32_t bits = pack_bits(reinterpret_cast<uint32_t*>(buf), 8u * nc, VAL, NBT, E + 3u, lane);
  return (bits + 7u) >> 3;
}

// The literals section into out (LDS, dword-aligned): its size.
__device__ __forceinline__ uint32_t compress_literals(uint8_t* out, const uint8_t* lits, uint32_t n, bool disable,
                                      uint8_t* ent, HNode* nodes, uint32_t lane, uint64_t* stamp) {
  if (disable || n <= 63) return raw_literals(out, lits, n, lane);
  uint32_t* cnt = reinterpret_cast<uint32_t*>(ent + kECnt);
  for (uint32_t k = lane; k < 256; k += 64) cnt[k] = 0;
  lds_sync();
  for (uint32_t k = lane; k < n; k += 64) atomicAdd(&cnt[lits[k]], 1u);
  lds_sync();
  uint32_t c[4];
  uint32_t largest = 0;
  uint64_t nzm[4];
#pragma unroll
  for (uint32_t g = 0; g < 4; ++g) {
    c[g] = cnt[g * 64u + lane];
    largest = c[g] > largest ? c[g] : largest;
    nzm[g] = __ballot(c[g] != 0);
  }
  for (uint32_t dd = 32; dd >= 1; dd >>= 1) {
    const uint32_t o = __shfl_xor(largest, dd);
    largest = o > largest ? o : largest;
  }
  largest = uni(largest);
  uint32_t max_sym = 0;
#pragma unroll
  for (uint32_t g = 0; g < 4; ++g)
    if (nzm[g]) max_sym = g * 64u + 63u - __builtin_clzll(nzm[g]);
  if (largest == n) return rle_literals(out, lits, n, lane);
  if (largest <= (n >> 7) + 4u) return raw_literals(out, lits, n, lane);
  const uint32_t min_gain = (n >> 6) + 2u;
  const uint32_t lh = 3u + (n >= 1024) + (n >= 16384);
  const bool single = n < 256;
  // HUF_optimalTableLog, the tree, its description
  const uint32_t huf_log = fse_opt_log(11, n, max_sym, 1);
  uint32_t* huf = reinterpret_cast<uint32_t*>(ent + kEHuf);
  zcstamp(stamp, 8);
  const uint32_t mb = huf_build(c, max_sym, huf_log, nodes, huf, lane);
  zcstamp(stamp, 9);
  uint32_t w[4];
#pragma unroll
  for (uint32_t g = 0; g < 4; ++g) {
    const uint32_t s = g * 64u + lane;
    const uint32_t nb = s <= max_sym ? huf[s] >> 16 : 0u;
    w[g] = nb ? mb + 1u - nb : 0u;
  }
  uint8_t* wbuf = ent + kEWts;
  uint32_t hsize = huf_compress_weights(w, max_sym, ent, wbuf, lane);
  zcstamp(stamp, 10);
  bool fse_form = hsize > 1 && hsize < max_sym / 2u;
  if (!fse_form) {
    if (max_sym > 128) return raw_literals(out, lits, n, lane);  // (HUF_writeCTable error)
    hsize = (max_sym + 1u) / 2u;
  }
  hsize += 1u;
  if (hsize + 12u >= n) return raw_literals(out, lits, n, lane);
  // stream sizes: the code lengths summed per stream
  const uint32_t ns = single ? 1u : 4u;
  const uint32_t seg = single ? n : (n + 3u) / 4u;
  const uint32_t lps = 64u / ns;  // lanes a stream
  const uint32_t sid = lane / lps, r = lane % lps;
  const uint32_t a = sid * seg;
  const uint32_t b = sid == ns - 1u ? n : a + seg;
  const uint32_t len = b > a ? b - a : 0u;
  const uint32_t chunk = (len + lps - 1u) / lps;
  const uint32_t x = a + r * chunk < b ? a + r * chunk : b;
  const uint32_t y = x + chunk < b ? x + chunk : b;
  uint32_t bits = 0;
  for (uint32_t i = x; i < y; ++i) bits += huf[lits[i]] >> 16;
  // bits after this chunk within its stream (chunks after it: reverse scan)
  uint32_t incl = bits;  // inclusive scan from the stream's last chunk
  for (uint32_t dd = 1; dd < lps; dd <<= 1) {
    const uint32_t v = __shfl_down(incl, dd);
    if (r + dd < lps) incl += v;
  }
  const uint32_t after = incl - bits;
  const uint32_t stream_bits = __shfl(incl, sid * lps);  // the stream's total
  uint32_t sz[4];
#pragma unroll
  for (uint32_t k = 0; k < 4; ++k)
    sz[k] = k < ns ? (uni(__shfl(stream_bits, k * lps)) + 8u) >> 3 : 0u;
  const uint32_t jump = single ? 0u : 6u;
  const uint32_t total = hsize + jump + sz[0] + sz[1] + sz[2] + sz[3];
  if (total >= n - 1u) return raw_literals(out, lits, n, lane);  // HUF: not worth it
  if (total >= n - min_gain) return raw_literals(out, lits, n, lane);
  zcstamp(stamp, 11);
  // pack: zero the streams' dwords, OR each chunk's bits in
  const uint32_t s0 = lh + hsize + jump;
  uint32_t* ow = reinterpret_cast<uint32_t*>(out);
  for (uint32_t k = (s0 >> 2) + lane; k < ((lh + total + 3u) >> 2); k += 64) ow[k] = 0;
  lds_sync();
  uint32_t sbase = s0;
#pragma unroll
  for (uint32_t k = 0; k < 4; ++k)
    if (k < sid) sbase += sz[k];
  if (len) {
    uint32_t A = 8u * sbase + after;
    uint32_t D = A >> 5;
    uint64_t acc = 0;
    uint32_t an = A & 31u;
    for (uint32_t i = y; i > x; --i) {
      const uint32_t e = huf[lits[i - 1u]];
      acc |= static_cast<uint64_t>(e & 0xFFFFu) << an;
      an += e >> 16;
      if (an >= 32) {
        atomicOr(&ow[D], static_cast<uint32_t>(acc));
        ++D;
        acc >>= 32;
        an -= 32;
      }
    }
    if (r == 0) {  // the stream's first chunk ends it: the end mark
      acc |= uint64_t{1} << an;
      ++an;
    }
    if (an) atomicOr(&ow[D], static_cast<uint32_t>(acc));
    if (an > 32) atomicOr(&ow[D + 1u], static_cast<uint32_t>(acc >> 32));
  }
  lds_sync();
  // the header, the tree description, the jump table
  if (lane == 0) {
    const uint32_t c_lit = total;
    if (lh == 3) {
      const uint32_t h = 2u + ((single ? 0u : 1u) << 2) + (n << 4) + (c_lit << 14);
      out[0] = static_cast<uint8_t>(h);
      out[1] = static_cast<uint8_t>(h >> 8);
      out[2] = static_cast<uint8_t>(h >> 16);
    } else if (lh == 4) {
      const uint32_t h = 2u + (2u << 2) + (n << 4) + (c_lit << 18);
      out[0] = static_cast<uint8_t>(h);
      out[1] = static_cast<uint8_t>(h >> 8);
      out[2] = static_cast<uint8_t>(h >> 16);
      out[3] = static_cast<uint8_t>(h >> 24);
    } else {
      const uint32_t h = 2u + (3u << 2) + (n << 4) + (c_lit << 22);
      out[0] = static_cast<uint8_t>(h);
      out[1] = static_cast<uint8_t>(h >> 8);
      out[2] = static_cast<uint8_t>(h >> 16);
      out[3] = static_cast<uint8_t>(h >> 24);
      out[4] = static_cast<uint8_t>(c_lit >> 10);
    }
    if (!single) {
      out[lh + hsize + 0] = static_cast<uint8_t>(sz[0]);
      out[lh + hsize + 1] = static_cast<uint8_t>(sz[0] >> 8);
      out[lh + hsize + 2] = static_cast<uint8_t>(sz[1]);
      out[lh + hsize + 3] = static_cast<uint8_t>(sz[1] >> 8);
      out[lh + hsize + 4] = static_cast<uint8_t>(sz[2]);
      out[lh + hsize + 5] = static_cast<uint8_t>(sz[2] >> 8);
    }
  }
  if (fse_form) {
    if (lane == 0) out[lh] = static_cast<uint8_t>(hsize - 1u);
    for (uint32_t k = lane; k + 1u < hsize; k += 64) out[lh + 1u + k] = wbuf[k];
  } else {
    if (lane == 0) out[lh] = static_cast<uint8_t>(128u + (max_sym - 1u));
    // 4-bit weights, two a byte (symbol max_sym's weight taken as 0)
    for (uint32_t k = lane; 2u * k < max_sym; k += 64) {
      const uint32_t s0w = 2u * k, s1w = 2u * k + 1u;
      const uint32_t n0 = huf[s0w] >> 16;
      const uint32_t n1 = s1w < max_sym ? huf[s1w] >> 16 : 0u;
      const uint32_t w0 = n0 ? mb + 1u - n0 : 0u, w1 = n1 ? mb + 1u - n1 : 0u;
      out[lh + 1u + k] = static_cast<uint8_t>((w0 << 4) + w1);
    }
  }
  lds_sync();
  return lh + total;
}

// ---- the sequences section --------------------------------------------------

// ZSTD_selectEncodingType (strategy fast, repeat none): 0 basic, 1 rle, 2 new.
__device__ __forceinline__ uint32_t select_type(uint32_t most, uint32_t nbseq, uint32_t dlog,
                                                bool allowed) {
  if (most == nbseq) return (allowed && nbseq <= 2) ? 0u : 1u;
  if (allowed) {
    const uint32_t dyn_min = ((1u << dlog) * 9u) >> 3;
    if (nbseq < dyn_min || most < (nbseq >> (dlog - 1u))) return 0u;
  }
  return 2u;
}

__device__ __forceinline__ int32_t default_norm(uint32_t table, uint32_t s) {
  // LL_defaultNorm / OF_defaultNorm / ML_defaultNorm
  if (table == 0) {
    if (s >= 32) return -1;
    if (s == 0) return 4;
    if (s == 1 || s == 25) return 3;
    if ((s >= 13 && s <= 15) || s >= 27) return 1;
    return 2;
  }
  if (table == 1) {
    if (s >= 24) return -1;
    return (s >= 6 && s <= 8) ? 2 : 1;
  }
  if (s >= 46) return -1;
  if (s == 0) return 1;
  if (s == 1) return 4;
  if (s == 2) return 3;
  return s <= 8 ? 2 : 1;
}

// One of the three tables: type, description bytes through bw, the CTable.
__device__ __forceinline__ uint32_t seq_table(uint32_t table, const uint8_t* codes, uint32_t nbseq, uint8_t* ent,
                              uint16_t* st, BitW& bw, FseC* t, uint32_t* desc_at, uint32_t lane) {
  uint32_t* cnt = reinterpret_cast<uint32_t*>(ent + kECnt);
  if (lane < 64) cnt[lane] = 0;
  lds_sync();
  for (uint32_t i = lane; i < nbseq; i += 64) atomicAdd(&cnt[codes[i]], 1u);
  lds_sync();
  const uint32_t mx = table == 0 ? 35u : (table == 1 ? 31u : 52u);
  uint32_t c = lane <= mx ? cnt[lane] : 0u;
  const uint64_t nz = __ballot(c != 0);
  const uint32_t max_sym = 63u - __builtin_clzll(nz);
  uint32_t most = c;
  for (uint32_t dd = 32; dd >= 1; dd >>= 1) {
    const uint32_t o = __shfl_xor(most, dd);
    most = o > most ? o : most;
  }
  most = uni(most);
  const uint32_t dlog = table == 1 ? 5u : 6u;
  const bool allowed = table == 1 ? max_sym <= 28u : true;
  const uint32_t type = select_type(most, nbseq, dlog, allowed);
  t->st = st;
  *desc_at = 0xFFFFFFFFu;
  if (type == 1) {  // FSE_buildCTable_rle: one state, no bits
    const uint32_t sym = uni(codes[0]);
    bw_add(bw, sym, 8, lane);
    bw_flush(bw, lane);
    if (lane == 0) st[0] = 0;
    t->dnb = 0;
    t->dfs = 0;
    t->log = 0;
    lds_sync();
    fse_regs(*t, lane);
    return type;
  }
  uint32_t tl, ms;
  int32_t normv;
  if (type == 0) {
    tl = dlog;
    ms = table == 0 ? 35u : (table == 1 ? 28u : 52u);
    normv = lane <= ms ? default_norm(table, lane) : 0;
  } else {
    const uint32_t fse_log = table == 1 ? 8u : 9u;
    tl = fse_opt_log(fse_log, nbseq, max_sym, 2);
    const uint32_t last = uni(codes[nbseq - 1u]);
    uint32_t n1 = nbseq;
    const uint32_t cl = uni(__builtin_amdgcn_readlane(c, last));
    if (cl > 1) {
      if (lane == last) c -= 1u;
      --n1;
    }
    normv = fse_normalize(c, tl, n1, max_sym, n1 >= 2048, lane);
    *desc_at = bw_end(bw);
    fse_write_ncount(normv, max_sym, tl, bw, lane);
    // (the description ends on a byte: the next starts on a fresh one)
    const uint32_t pad = (8u - (bw.n & 7u)) & 7u;
    bw_add(bw, 0, pad, lane);
    ms = max_sym;
  }
  bw_flush(bw, lane);
  lds_sync();
  fse_build_ctable(normv, ms, tl, st, ent, lane, &t->dnb, &t->dfs);
  t->log = tl;
  lds_sync();
  fse_regs(*t, lane);
  return type;
}

// ---- the block --------------------------------------------------------------

// A frame's header (ZSTD_writeFrameHeader): content size, single segment
// when the window covers it. Returns its bytes (written by lane 0 to g).
__device__ __forceinline__ uint32_t frame_header(uint8_t* g, uint32_t wlog, uint32_t n, uint32_t lane) {
  const uint32_t single = (1u << wlog) >= n ? 1u : 0u;
  const uint32_t fcs = (n >= 256u) + (n >= 65536u + 256u);
  uint32_t p = 0;
  uint8_t h[12];
  h[p++] = 0x28;
  h[p++] = 0xB5;
  h[p++] = 0x2F;
  h[p++] = 0xFD;
  h[p++] = static_cast<uint8_t>((single << 5) + (fcs << 6));
  if (!single) h[p++] = static_cast<uint8_t>((wlog - 10u) << 3);
  if (fcs == 0) {
    if (single) h[p++] = static_cast<uint8_t>(n);
  } else if (fcs == 1) {
    h[p++] = static_cast<uint8_t>(n - 256u);
    h[p++] = static_cast<uint8_t>((n - 256u) >> 8);
  } else {
    h[p++] = static_cast<uint8_t>(n);
    h[p++] = static_cast<uint8_t>(n >> 8);
    h[p++] = static_cast<uint8_t>(n >> 16);
    h[p++] = static_cast<uint8_t>(n >> 24);
  }
  if (lane < p) {
    uint8_t v = h[0];
#pragma unroll
    for (uint32_t k = 1; k < 12; ++k)
      if (k == lane) v = h[k];
    g[lane] = v;
  }
  return p;
}

__device__ __forceinline__ uint32_t zhash(const uint8_t* in, uint32_t p, uint32_t hlog, uint32_t mls) {
  if (mls == 4) return (ld32(in, p) * 2654435761u) >> (32u - hlog);
  const uint64_t prime = mls == 5 ? 889523592379ull : (mls == 6 ? 227718039650203ull : 58295818150454627ull);
  const uint64_t v = ld64(in, p) << (64u - 8u * mls);
  return static_cast<uint32_t>((v * prime) >> (64u - hlog));
}

// a / b for a, b < 2^16, b > 0: a float reciprocal and one correction (the
// estimate is within one), not the ~35-instruction integer division
__device__ __forceinline__ uint32_t udiv16(uint32_t a, uint32_t b) {
  uint32_t q = static_cast<uint32_t>(static_cast<float>(a) * __builtin_amdgcn_rcpf(static_cast<float>(b)));
  if (q * b > a) --q;
  else if ((q + 1u) * b <= a) ++q;
  return q;
}

// ip0 - anchor after j steps from d0 (step = d >> 7 + ss)
__device__ __forceinline__ uint32_t step_pos(uint32_t d, uint32_t k, uint32_t ss) {
  while (k) {
    const uint32_t q = d >> 7, st = q + ss;
    const uint32_t rem = ((q + 1u) << 7) - d;
    const uint32_t nseg = udiv16(rem + st - 1u, st);
    if (k <= nseg) {
      d += k * st;
      break;
    }
    d += nseg * st;
    k -= nseg;
  }
  return d;
}

// matches bytes in[a + k] == in[b + k] for a + k < lim: the count (wave)
__device__ __forceinline__ uint32_t zcount(const uint8_t* in, uint32_t a, uint32_t b, uint32_t lim,
                                           uint32_t lane) {
  uint32_t m = 0;
  for (;;) {
    const uint32_t pa = a + m + lane;
    const bool diff = pa >= lim || in[pa] != in[b + m + lane];
    const uint64_t bal = __ballot(diff);
    if (bal != 0) return m + static_cast<uint32_t>(__builtin_ctzll(bal));
    m += 64;
  }
}

struct Seqs {
  uint8_t* lits;  // the match finder's: the block's frame slot in HBM (kLitStage)
  uint32_t* sll;  // litLength | mlBase << 16
  uint16_t* sof;  // offset code + 1 (<= max_len + 3)
  uint32_t nlit, nseq;
};

__device__ __forceinline__ void store_seq(Seqs& s, const uint8_t* in, uint32_t anchor, uint32_t litlen,
                                          uint32_t offcode, uint32_t mlbase, uint32_t lane) {
  for (uint32_t k = lane; k < litlen; k += 64) s.lits[s.nlit + k] = in[anchor + k];
  if (lane == 0) {
    s.sll[s.nseq] = litlen | (mlbase << 16);
    s.sof[s.nseq] = static_cast<uint16_t>(offcode + 1u);
  }
  s.nlit += litlen;
  s.nseq += 1u;
}

// ZSTD_compressBlock_fast_generic over the whole frame in[0, n) (one block:
// n <= the window), 64 steps a window.
template <typename TIdx>
__device__ __forceinline__ void match_block(const uint8_t* in, uint32_t n, TIdx* table, uint32_t* tags,
                            const ZParams& zp, Seqs& sq, uint32_t lane) {
  const uint32_t hlog = zp.hlog, mls = zp.mls;
  const uint32_t ss = zp.tl + (zp.tl ? 0u : 1u) + 1u;
  const int32_t ilimit = static_cast<int32_t>(n) - 8;
  const uint64_t below = (uint64_t{1} << lane) - 1u;
  uint32_t anchor = 0;
  uint32_t ip0 = 1;  // (istart == prefixStart: the first position is skipped)
  // repcodes 1, 4, 8; maxRep = 1 at ip0 = 1: offset_2 (4) is set aside
  uint32_t off1 = 1, off2 = 0;
  uint32_t d0 = ip0 - anchor;
  // (every window moves ip0 forward; the bound only guards the grid's exit)
  for (uint32_t guard = 0; guard <= n; ++guard) {
    const uint32_t d = step_pos(d0, lane, ss);
    const uint32_t p0 = anchor + d, p1 = p0 + 1u;
    const bool valid = static_cast<int32_t>(p1) < ilimit;
    const uint64_t vmask = __ballot(valid);
    if (vmask == 0) break;
    const uint32_t q0 = valid ? p0 : 0u;
    const uint32_t h0 = zhash(in, q0, hlog, mls), h1 = zhash(in, q0 + 1u, hlog, mls);
    const uint32_t v0 = ld32(in, q0), v1 = ld32(in, q0 + 1u);
    const bool rep = valid && off1 > 0 && ld32(in, q0 + 2u - off1) == ld32(in, q0 + 2u);
    const uint32_t c0 = valid ? static_cast<uint32_t>(table[h0]) : 0u;
    const uint32_t c1 = valid ? static_cast<uint32_t>(table[h1]) : 0u;
    const bool sm0 = valid && c0 > 1u && ld32(in, c0 - 1u) == v0;
    const bool sm1 = valid && c1 > 1u && ld32(in, c1 - 1u) == v1;
    const uint32_t t0 = h0 & (kTags - 1u), t1 = h1 & (kTags - 1u);
    const uint32_t w0 = 2u * lane;
    if (valid) {
      atomicMin(&tags[t0], w0);
      atomicMin(&tags[t1], w0 + 1u);
    }
    lds_sync();
    const uint32_t f0 = valid ? tags[t0] : 0xFFFFFFFFu;
    const uint32_t f1 = valid ? tags[t1] : 0xFFFFFFFFu;
    lds_sync();
    if (valid) {
      tags[t0] = 0;
      tags[t1] = 0;
    }
    lds_sync();
    const bool sus0 = valid && f0 < w0, sus1 = valid && f1 < w0;
    const uint64_t sure = __ballot(rep || (sm0 && !sus0) || (sm1 && !sus1));
    uint32_t J = sure ? static_cast<uint32_t>(__builtin_ctzll(sure)) : 64u;
    // kind: 1 rep, 2 first position, 3 second position
    uint32_t kind = 0, cand = 0;
    if (J < 64) {
      const uint64_t br = __ballot(rep), b0 = __ballot(sm0 && !sus0);
      kind = ((br >> J) & 1u) ? 1u : (((b0 >> J) & 1u) ? 2u : 3u);
    }
    // the suspect reads up to J, in order
    uint64_t sl = __ballot(sus0 || sus1);
    const uint64_t s0m = __ballot(sus0), s1m = __ballot(sus1), sm0m = __ballot(sm0),
                   sm1m = __ballot(sm1);
    bool resolved = false;
    while (sl) {
      const uint32_t dl = static_cast<uint32_t>(__builtin_ctzll(sl));
      sl &= sl - 1u;
      if (dl > J) break;
      if (dl == J && kind != 3) break;  // rep or a sure first read wins
      const uint64_t bl = (uint64_t{1} << dl) - 1u;
      for (uint32_t slot = 0; slot < 2; ++slot) {
        if (slot == 1 && dl == J) break;  // (kind 3 at J: its second read is sure)
        const bool is_s = ((slot == 0 ? s0m : s1m) >> dl) & 1u;
        bool hit;
        uint32_t cpos = 0;
        if (is_s) {
          const uint32_t hd = uni(__builtin_amdgcn_readlane(slot == 0 ? h0 : h1, dl));
          const uint64_t m0w = __ballot(valid && h0 == hd) & bl;
          const uint64_t m1w = __ballot(valid && h1 == hd) & bl;
          const int32_t i0 = m0w ? 63 - __builtin_clzll(m0w) : -1;
          const int32_t i1 = m1w ? 63 - __builtin_clzll(m1w) : -1;
          const uint32_t vd = uni(__builtin_amdgcn_readlane(slot == 0 ? v0 : v1, dl));
          if (i0 < 0 && i1 < 0) {  // another hash in the slot: the old entry stands
            hit = ((slot == 0 ? sm0m : sm1m) >> dl) & 1u;
            cpos = uni(__builtin_amdgcn_readlane(slot == 0 ? c0 : c1, dl)) - 1u;
          } else if (2 * i0 > 2 * i1 + 1) {
            cpos = uni(__builtin_amdgcn_readlane(p0, static_cast<uint32_t>(i0)));
            hit = uni(__builtin_amdgcn_readlane(v0, static_cast<uint32_t>(i0))) == vd;
          } else {
            cpos = uni(__builtin_amdgcn_readlane(p1, static_cast<uint32_t>(i1)));
            hit = uni(__builtin_amdgcn_readlane(v1, static_cast<uint32_t>(i1))) == vd;
          }
        } else {
          hit = false;  // (a sure hit there would have set J)
        }
        if (hit) {
          J = dl;
          kind = slot == 0 ? 2u : 3u;
          cand = cpos;
          resolved = true;
          break;
        }
      }
      if (resolved) break;
    }
    if (J < 64 && !resolved && kind != 1) {
      cand = uni(__builtin_amdgcn_readlane(kind == 2 ? c0 : c1, J)) - 1u;
    }
    const uint32_t ki = ~vmask ? static_cast<uint32_t>(__builtin_ctzll(~vmask)) : 64u;
    const bool end = ki < 64 && J >= ki;  // the loop runs past ilimit before a hit
    // the window's table writes: steps 0..min(J, 63), each hash's last
    const uint32_t Jw = J < 64 ? J : 63u;
    const bool part = valid && lane <= Jw;
    if (part) {
      atomicMax(&tags[t0], w0 + 1u);
      atomicMax(&tags[t1], w0 + 2u);
    }
    lds_sync();
    const uint32_t l0 = valid ? tags[t0] : 0u, l1 = valid ? tags[t1] : 0u;
    lds_sync();
    if (valid) {
      tags[t0] = 0xFFFFFFFFu;
      tags[t1] = 0xFFFFFFFFu;
    }
    bool fin0 = part && l0 == w0 + 1u, fin1 = part && l1 == w0 + 2u;
    uint64_t wsus = __ballot(part && (!fin0 || !fin1));
    const uint64_t pm = __ballot(part);
    while (wsus) {
      const uint32_t dl = static_cast<uint32_t>(__builtin_ctzll(wsus));
      wsus &= wsus - 1u;
      const uint64_t ab = pm & ~((uint64_t{2} << dl) - 1u);  // later steps
      for (uint32_t slot = 0; slot < 2; ++slot) {
        const bool f = __builtin_amdgcn_readlane(slot == 0 ? (fin0 ? 1u : 0u) : (fin1 ? 1u : 0u), dl);
        if (f) continue;
        const uint32_t hd = uni(__builtin_amdgcn_readlane(slot == 0 ? h0 : h1, dl));
        bool later = ((__ballot(h0 == hd) | __ballot(h1 == hd)) & ab) != 0;
        if (slot == 0) later = later || uni(__builtin_amdgcn_readlane(h1, dl)) == hd;
        if (!later && lane == dl) {
          if (slot == 0) fin0 = true;
          else fin1 = true;
        }
      }
    }
    if (fin0) table[h0] = static_cast<TIdx>(p0 + 1u);
    if (fin1) table[h1] = static_cast<TIdx>(p1 + 1u);
    lds_sync();
    if (end) break;
    if (J == 64) {  // no hit in 64 steps: the next window
      d0 = uni(step_pos(__shfl(d, 63), 1, ss));
      continue;
    }
    // the hit (step J)
    const uint32_t hp0 = uni(__builtin_amdgcn_readlane(p0, J));
    uint32_t ip, m0, ml, offcode;
    if (kind == 1) {
      const uint32_t q2 = hp0 + 2u, rm = q2 - off1;
      const uint32_t e = uni(in[q2 - 1u]) == uni(in[rm - 1u]) ? 1u : 0u;
      ip = q2 - e;
      m0 = rm - e;
      ml = 4u + e;
      offcode = 0;
    } else {
      ip = kind == 2 ? hp0 : hp0 + 1u;
      m0 = cand;
      off2 = off1;
      off1 = ip - m0;
      offcode = off1 + 2u;
      ml = 4;
      // backward: while ip > anchor && m0 > 0 && in[ip-1] == in[m0-1]
      const uint32_t lim = (ip - anchor) < m0 ? ip - anchor : m0;
      uint32_t k = 0;
      for (;;) {
        const uint32_t kk = k + lane;
        const bool stop = kk >= lim || in[ip - 1u - kk] != in[m0 - 1u - kk];
        const uint64_t bal = __ballot(stop);
        if (bal) {
          k += static_cast<uint32_t>(__builtin_ctzll(bal));
          break;
        }
        k += 64;
      }
      ip -= k;
      m0 -= k;
      ml += k;
    }
    ml += zcount(in, ip + ml, m0 + ml, n, lane);
    store_seq(sq, in, anchor, ip - anchor, offcode, ml - 3u, lane);
    ip += ml;
    anchor = ip;
    if (static_cast<int32_t>(ip) <= ilimit) {
      const uint32_t ha = zhash(in, hp0 + 2u, hlog, mls);
      const uint32_t hb = zhash(in, ip - 2u, hlog, mls);
      if (lane == 0) table[ha] = static_cast<TIdx>(hp0 + 3u);
      lds_sync();
      if (lane == 0) table[hb] = static_cast<TIdx>(ip - 1u);
      lds_sync();
      if (off2 > 0) {
        while (static_cast<int32_t>(ip) <= ilimit && uni(ld32(in, ip)) == uni(ld32(in, ip - off2))) {
          const uint32_t rl = 4u + zcount(in, ip + 4u, ip + 4u - off2, n, lane);
          const uint32_t tmp = off2;
          off2 = off1;
          off1 = tmp;
          const uint32_t hr = zhash(in, ip, hlog, mls);
          if (lane == 0) table[hr] = static_cast<TIdx>(ip + 1u);
          lds_sync();
          store_seq(sq, in, anchor, 0, 0, rl - 3u, lane);
          ip += rl;
          anchor = ip;
        }
      }
    }
    d0 = 0;
  }
  // the last literals
  for (uint32_t k = lane; k < n - anchor; k += 64) sq.lits[sq.nlit + k] = in[anchor + k];
  sq.nlit += n - anchor;
  lds_sync();
  (void)below;
}

template <typename TIdx>
__global__ void __launch_bounds__(64) zstd_compress_kernel(ZcArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t b = blockIdx.x;
  if (b >= a.nblocks) return;
  const uint32_t lane = threadIdx.x;
  const uint32_t n = a.src_len[b];
  const uint8_t* src = a.src + a.src_off[b];
  uint8_t* g = a.dst + (a.dst_off ? a.dst_off[b] : b * a.dst_stride);
  auto finish = [&](uint32_t st, uint32_t len) {
    if (lane == 0) {
      a.dst_len[b] = len;
      a.status[b] = static_cast<uint8_t>(st);
    }
  };
#ifdef LVKV_PROBE_BUILD
  __shared__ uint64_t stamp_lds[16];
  uint64_t* stamp = stamp_lds;
#else
  uint64_t* stamp = nullptr;
#endif
  zcstamp(stamp, 0);
  const ZParams zp = zstd_port_params(a.level, n);
  if (!zp.ok) return finish(LVKV_ZSTD_UNSUPPORTED, 0);
  if (n > a.max_len) return finish(LVKV_ZSTD_TOO_LARGE, 0);
  const uint32_t fh = frame_header(g, zp.wlog, n, lane);
  if (n == 0) {
    if (lane < 3) g[fh + lane] = lane == 0 ? 1 : 0;  // the last (empty) raw block
    return finish(LVKV_ZSTD_OK, fh + 3u);
  }
  auto raw_block = [&]() {
    const uint32_t bh = 1u + (n << 3);
    if (lane < 3) g[fh + lane] = static_cast<uint8_t>(bh >> (8u * lane));
    for (uint32_t k = lane; k < n; k += 64) g[fh + 3u + k] = src[k];
    finish(LVKV_ZSTD_OK, fh + 3u + n);
  };
  if (n < 7) return raw_block();  // (MIN_CBLOCK_SIZE + header + 1)
  uint8_t* in = smem;
  TIdx* table = reinterpret_cast<TIdx*>(smem + a.o_tbl);
  uint32_t* tags = reinterpret_cast<uint32_t*>(smem + a.o_tag);
  Seqs sq;
  // the literals go to the block's own frame slot in HBM while the table is
  // in use (room: ZSTD_compressBound(n) - n >= kLitStage + 22 for n <=
  // LVKV_ZSTD_COMPRESS_MAX_BLOCK), then into the dead table's LDS for the
  // entropy stage: one LDS region less, one more workgroup a CU
  sq.lits = g + kLitStage;
  sq.sll = reinterpret_cast<uint32_t*>(smem + a.o_sll);
  sq.sof = reinterpret_cast<uint16_t*>(smem + a.o_sof);
  sq.nlit = 0;
  sq.nseq = 0;
  stage(in, src, n, 16, lane);
  {
    const uint32_t tw = ((sizeof(TIdx) << zp.hlog) + 3u) >> 2;
    uint32_t* tz = reinterpret_cast<uint32_t*>(table);
    for (uint32_t k = lane; k < tw; k += 64) tz[k] = 0;
    for (uint32_t k = lane; k < kTags; k += 64) tags[k] = 0xFFFFFFFFu;
  }
  lds_sync();
  zcstamp(stamp, 1);
  match_block<TIdx>(in, n, table, tags, zp, sq, lane);
  {
    __builtin_amdgcn_s_waitcnt(0);  // (every lane's literal stores have landed)
    uint8_t* lits = smem + a.o_lit;
    for (uint32_t k = lane; k < sq.nlit; k += 64) lits[k] = g[kLitStage + k];
    sq.lits = lits;
    lds_sync();
  }
  zcstamp(stamp, 2);
  // ---- entropy (the input region becomes the block's staging buffer)
  uint8_t* out = in;
  uint8_t* ent = reinterpret_cast<uint8_t*>(table);
  HNode* nodes = reinterpret_cast<HNode*>(tags);
  const uint32_t nseq = sq.nseq;
  const uint32_t limit = n - ((n >> 6) + 2u);  // a body at least this long: raw
  uint32_t pos = compress_literals(out, sq.lits, sq.nlit, zp.tl > 0, ent, nodes, lane, stamp);
  zcstamp(stamp, 3);
  if (pos + 1u >= limit) return raw_block();  // (the smallest body: + the count byte)
  // sequences header
  if (lane == 0) {
    if (nseq < 128) {
      out[pos] = static_cast<uint8_t>(nseq);
    } else if (nseq < 0x7F00) {
      out[pos] = static_cast<uint8_t>((nseq >> 8) + 0x80u);
      out[pos + 1] = static_cast<uint8_t>(nseq);
    } else {
      out[pos] = 0xFF;
      out[pos + 1] = static_cast<uint8_t>(nseq - 0x7F00u);
      out[pos + 2] = static_cast<uint8_t>((nseq - 0x7F00u) >> 8);
    }
  }
  pos += nseq < 128 ? 1u : (nseq < 0x7F00 ? 2u : 3u);
  lds_sync();
  if (nseq > 0) {
    uint8_t* llc = ent + kECodes;
    uint8_t* ofc = llc + round16(a.smax);
    uint8_t* mlc = ofc + round16(a.smax);
    for (uint32_t i = lane; i < nseq; i += 64) {
      const uint32_t v = sq.sll[i];
      const uint32_t ll = v & 0xFFFFu, mlb = v >> 16;
      llc[i] = static_cast<uint8_t>(ll_code(ll));
      ofc[i] = static_cast<uint8_t>(hibit(sq.sof[i]));
      mlc[i] = static_cast<uint8_t>(ml_code(mlb));
    }
    lds_sync();
    const uint32_t seq_head = pos++;
    BitW bw;
    bw_init(bw, out, pos);
    FseC tll, tof, tml;
    uint32_t at_ll, at_of, at_ml;
    const uint32_t ty_ll = seq_table(0, llc, nseq, ent, reinterpret_cast<uint16_t*>(ent + kEStLL),
                                     bw, &tll, &at_ll, lane);
    const uint32_t ty_of = seq_table(1, ofc, nseq, ent, reinterpret_cast<uint16_t*>(ent + kEStOF),
                                     bw, &tof, &at_of, lane);
    const uint32_t ty_ml = seq_table(2, mlc, nseq, ent, reinterpret_cast<uint16_t*>(ent + kEStML),
                                     bw, &tml, &at_ml, lane);
    uint32_t last_nc = at_ml != 0xFFFFFFFFu ? at_ml : (at_of != 0xFFFFFFFFu ? at_of : at_ll);
    zcstamp(stamp, 4);
    if (lane == 0) out[seq_head] = static_cast<uint8_t>((ty_ll << 6) + (ty_of << 4) + (ty_ml << 2));
    lds_sync();
    // the backward bitstream (ZSTD_encodeSequences)
    const uint32_t bs_start = bw_end(bw);
    bw_init(bw, out, bs_start);
    // the sequences 64 at a time in registers (lane k: sequence base + k),
    // read by the serial coder with v_readlane
    uint32_t base = (nseq - 1u) & ~63u;
    uint32_t rv = 0, ro = 0, rc = 0;
    auto load = [&](uint32_t b0) {
      const uint32_t k = b0 + lane;
      rv = k < nseq ? sq.sll[k] : 0u;
      ro = k < nseq ? sq.sof[k] : 0u;
      rc = k < nseq ? (llc[k] | (static_cast<uint32_t>(ofc[k]) << 8) |
                       (static_cast<uint32_t>(mlc[k]) << 16))
                    : 0u;
    };
    load(base);
    uint32_t i = nseq - 1u;
    uint32_t v = __builtin_amdgcn_readlane(rv, i - base), of = __builtin_amdgcn_readlane(ro, i - base);
    uint32_t cc = __builtin_amdgcn_readlane(rc, i - base);
    uint32_t cl = cc & 255u, co = (cc >> 8) & 255u, cm = cc >> 16;
    uint32_t sm = fse_init(tml, cm), so = fse_init(tof, co), sl = fse_init(tll, cl);
    bw_add(bw, v & 0xFFFFu, ll_bits(cl), lane);
    bw_add(bw, v >> 16, ml_bits(cm), lane);
    bw_add(bw, of, co, lane);
    bool over = false;
    while (i > 0) {
      --i;
      if (i < base) {
        base -= 64u;
        load(base);
      }
      v = __builtin_amdgcn_readlane(rv, i - base);
      of = __builtin_amdgcn_readlane(ro, i - base);
      cc = __builtin_amdgcn_readlane(rc, i - base);
      cl = cc & 255u;
      co = (cc >> 8) & 255u;
      cm = cc >> 16;
      so = fse_enc(tof, so, co, bw, lane);
      sm = fse_enc(tml, sm, cm, bw, lane);
      sl = fse_enc(tll, sl, cl, bw, lane);
      bw_add(bw, v & 0xFFFFu, ll_bits(cl), lane);
      bw_add(bw, v >> 16, ml_bits(cm), lane);
      bw_add(bw, of, co, lane);
      if (4u * bw.d >= limit) {
        over = true;
        break;
      }
    }
    if (over) return raw_block();
    zcstamp(stamp, 5);
    bw_add(bw, sm, tml.log, lane);
    bw_add(bw, so, tof.log, lane);
    bw_add(bw, sl, tll.log, lane);
    bw_add(bw, 1u, 1, lane);
    bw_flush(bw, lane);
    pos = bw_end(bw);
    // (zstd <= 1.3.4's decoder: a last table description within 4 bytes of
    // the end makes the block raw)
    if (last_nc != 0xFFFFFFFFu && pos - last_nc < 4u) return raw_block();
  }
  if (pos >= limit) return raw_block();
  lds_sync();
  const uint32_t bh = 1u + (2u << 1) + (pos << 3);
  if (lane < 3) g[fh + lane] = static_cast<uint8_t>(bh >> (8u * lane));
  for (uint32_t k = lane; k < pos; k += 64) g[fh + 3u + k] = out[k];
  finish(LVKV_ZSTD_OK, fh + 3u + pos);
  zcstamp(stamp, 6);
#ifdef LVKV_PROBE_BUILD
  lds_sync();
  if (a.stamps != nullptr && lane < 16) a.stamps[16u * b + lane] = stamp[lane];
#endif
}

}  // namespace

struct ZstdCompressPlan {
  uint32_t lds, o_tbl, o_tag, o_lit, o_sll, o_sof, smax;
};

// The LDS plan for blocks up to max_len at `level`: the staged block (+ room
// for a body that runs past it before the raw decision), the hash table (the
// largest hash log any size up to max_len gets; u16 entries; after the match
// finder, the entropy scratch and the literals), the window slots (then the
// Huffman nodes) and the sequences. 31.3 KB for 4 KiB blocks: 5 workgroups
// a CU.
ZstdCompressPlan zstd_compress_plan(uint32_t max_len, int level) {
  ZstdCompressPlan p{};
  uint32_t hmax = 6;
  for (uint32_t k = 0; k <= 17; ++k) {
    for (uint32_t n : {1u << k, (1u << k) + 1u}) {
      const ZParams z = zstd_port_params(level, n < max_len ? n : max_len);
      if (z.ok && z.hlog > hmax) hmax = z.hlog;
    }
  }
  p.smax = max_len / 4u + 2u;
  // the table region: the hash table, then (entropy stage) the scratch and
  // after it the literals
  const uint32_t ent = kECodes + 3u * round16(p.smax);
  const uint32_t ent_lits = ent + round16(max_len + 16u);
  const uint32_t tbl = (2u << hmax) > ent_lits ? (2u << hmax) : ent_lits;
  uint32_t o = round16(max_len + 512u);
  p.o_tbl = o;
  p.o_lit = o + ent;
  o += round16(tbl);
  p.o_tag = o;
  o += 4u * kTags;
  p.o_sll = o;
  o += 4u * round16(p.smax);
  p.o_sof = o;
  o += 2u * round16(p.smax);
  p.lds = o;
  return p;
}

uint32_t zstd_compress_lds(uint32_t max_len, int level) {
  return zstd_compress_plan(max_len < 16u ? 16u : max_len, level).lds;
}

uint64_t* g_zstdc_stamps = nullptr;  // lvkv_debug_zstdc_stamps (tools/probe)

hipError_t launch_zstd_compress(const uint8_t* src, const uint64_t* src_off, const uint32_t* src_len,
                                uint8_t* dst, const uint64_t* dst_off, uint32_t* dst_len,
                                uint8_t* status, uint32_t nblocks, uint32_t max_len, int level,
                                uint64_t dst_stride, hipStream_t stream) {
  const uint32_t cap = max_len < 16u ? 16u : max_len;
  const ZstdCompressPlan p = zstd_compress_plan(cap, level);
  ZcArgs a{src, src_off, src_len, dst, dst_off, dst_len, status, nblocks, level, max_len,
           dst_stride, p.o_tbl, p.o_tag, p.o_lit, p.o_sll, p.o_sof, p.smax, g_zstdc_stamps};
  hipLaunchKernelGGL(zstd_compress_kernel<uint16_t>, dim3(nblocks), dim3(64), p.lds, stream, a);
  return hipGetLastError();
}

}  // namespace lvkv
