// Zstd frame decoder on the device (the read side of
// kZstdCompression): what port::Zstd_GetUncompressedLength / Zstd_Uncompress
// (port/port_stdcxx.h:163-199) do in ReadBlock (table/format.cc:138-155).
// The frames are RFC 8878's, decoded the way libzstd 1.4.9 decodes them
// (oracle/zstd_oracle.py is the restatement it is tested against, and that
// is pinned to the library). The compressor stays the library's: its bytes
// depend on zstd's match finder and entropy heuristics, which this project
// does not restate.
//
// One wave per frame (64-thread workgroups), the frame staged in LDS. The
// frame is a chain (headers, a Huffman tree, FSE tables, backward
// bitstreams, sequences whose matches read earlier output), so control flow
// is wave-uniform and the serial chains run on the scalar unit from
// registers (uni(), RegBits); the lanes build the decode tables, decode the
// Huffman streams in self-synchronising segments, and copy literals and
// matches.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lvkv_snappy.h"
#include "lvkv_zstd_tables.h"

namespace lvkv {
namespace {

constexpr uint32_t kMagic = 0xFD2FB528u;
constexpr uint32_t kBlockMax = 128u * 1024u;

// failure sites (the debug detail array; 0 = none)
enum : uint32_t {
  kFOk = 0, kFHeader, kFDict, kFBlockHdr, kFBlockType, kFBlockSize, kFCap, kFLitHdr,
  kFLitSize, kFHufHdr, kFHufWeights, kFHufTable, kFHufStream, kFJump, kFSeqHdr, kFNcount,
  kFFseSpread, kFRle, kFRepeat, kFSeqBits, kFLitOverrun, kFOffset, kFContentSize, kFChecksum,
  kFTrailing, kFSkippable, kFEmpty
};

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

// Wave-uniform reads. The parser's values are the same in every lane; an
// LDS or global load still lands in a VGPR, and everything computed from it
// would run as divergent code (exec masks, VALU), so the loads that steer
// control flow go through v_readfirstlane into SGPRs.
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint32_t ldb(const uint8_t* b, uint32_t p) { return uni(b[p]); }
__device__ __forceinline__ uint32_t ld32u(const uint8_t* b, uint32_t p) { return uni(ld32(b, p)); }
__device__ __forceinline__ uint64_t ld64u(const uint8_t* b, uint32_t p) {
  const uint64_t v = ld64(b, p);
  return (static_cast<uint64_t>(uni(static_cast<uint32_t>(v >> 32))) << 32) |
         uni(static_cast<uint32_t>(v));
}

// Global -> LDS (4-aligned), as the Snappy kernels stage (aligned dword loads
// at any source alignment, nothing read past the block's last dword).
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

// ---- backward bitstreams (RFC 8878 §4.1.1.1) ------------------------------
// Bits [0, pos) of a stream, read from the top down; bits below 0 read as
// zeros. The Huffman lanes cache a 64-bit window each (huf_run); the wave's
// scalar readers use a register-held window (RegBits).

// The sequences' bitstream, read by the scalar unit from a window of 248
// staged bytes held a dword a lane and reloaded from LDS when a read leaves
// it (about every 60 sequences): a read is two v_readlane and a 64-bit
// shift, with no LDS round trip to wait on. Bits below the stream's start
// read as zeros (the window's lanes there hold zeros).
struct RegBits {
  const uint8_t* in;
  uint32_t start;  // the stream's first byte in `in`
  int32_t pos;     // bits left
  int32_t wlo;     // the window's first bit (stream-relative, a multiple of 32)
  uint32_t d;      // lane k: the stream's bits [wlo + 32 k, wlo + 32 k + 32)
};
__device__ __forceinline__ void rb_load(RegBits& r, int32_t top, uint32_t lane) {
  r.wlo = ((top + 31) & ~31) - 1984;  // top - wlo <= 2015: lanes q >> 5 and + 1 <= 63
  const int32_t b = (r.wlo >> 3) + 4 * static_cast<int32_t>(lane);
  r.d = b < 0 ? 0u : ld32(r.in, r.start + static_cast<uint32_t>(b));
  __builtin_amdgcn_s_waitcnt(0xc07f);
}
// false: no end marker (br_init)
__device__ __forceinline__ bool rb_init(RegBits& r, const uint8_t* in, uint32_t lo, uint32_t hi,
                                        uint32_t lane) {
  r.in = in;
  r.start = lo;
  if (hi <= lo) return false;
  const uint32_t last = ldb(in, hi - 1);
  if (last == 0) return false;
  r.pos = static_cast<int32_t>(8u * (hi - lo - 1u) + (31u - __builtin_clz(last)));
  rb_load(r, r.pos, lane);
  return true;
}
// n <= 32 bits
__device__ __forceinline__ uint32_t rb_read(RegBits& r, uint32_t n, uint32_t lane) {
  r.pos -= static_cast<int32_t>(n);
  if (r.pos < r.wlo) rb_load(r, r.pos + static_cast<int32_t>(n), lane);
  const uint32_t q = static_cast<uint32_t>(r.pos - r.wlo);
  // (readlane returns int: widen through uint32_t, not by sign)
  const uint32_t w0 = __builtin_amdgcn_readlane(r.d, q >> 5);
  const uint32_t w1 = __builtin_amdgcn_readlane(r.d, (q >> 5) + 1u);
  const uint64_t x = (static_cast<uint64_t>(w1) << 32) | w0;
  return static_cast<uint32_t>((x >> (q & 31u)) & ((uint64_t{1} << n) - 1u));
}

// ---- FSE tables (RFC 8878 §4.1; FSE_readNCount / FSE_buildDTable) --------
// Decode entries: symbol | nbBits << 8 | baseline << 16.

// 256 staged bytes from in[a] (a 4-aligned) held across the wave, a dword a
// lane, so that the serial header and weight decoders read them with
// v_readlane (a few cycles) instead of an LDS round trip each.
struct RegBytes {
  const uint8_t* in;
  uint32_t a;
  uint32_t d;
};
__device__ __forceinline__ RegBytes reg_bytes(const uint8_t* in, uint32_t p, uint32_t lane) {
  RegBytes r;
  r.in = in;
  r.a = p & ~3u;
  r.d = reinterpret_cast<const uint32_t*>(in + r.a)[lane];
  return r;
}
// 32 bits at in[p] (p >= r.a)
__device__ __forceinline__ uint32_t rb32(const RegBytes& r, uint32_t p) {
  const uint32_t b = p - r.a;
  if (b + 8u > 256u) return ld32u(r.in, p);
  const uint32_t w0 = __builtin_amdgcn_readlane(r.d, b >> 2);
  const uint32_t w1 = __builtin_amdgcn_readlane(r.d, (b >> 2) + 1u);
  return __builtin_amdgcn_alignbyte(w1, w0, b & 3u);
}

// The table description at in[p, end): false when malformed. Scalar code.
__device__ bool read_ncount(const uint8_t* in, uint32_t p, uint32_t end, uint32_t max_sym,
                            uint32_t max_log, int16_t* counts, uint32_t* nsym, uint32_t* log_out,
                            uint32_t* used, uint32_t lane) {
  if (end <= p) return false;
  const uint32_t len = end - p;
  const RegBytes rg = reg_bytes(in, p, lane);
  // 32 bits at byte offset i of the description, zeros past its end
  auto rd32 = [&](uint32_t i) -> uint32_t {
    if (i >= len) return 0u;
    const uint32_t v = rb32(rg, p + i);
    return i + 4u <= len ? v : v & ((1u << (8u * (len - i))) - 1u);
  };
  uint32_t ip = 0;
  uint32_t bits = rd32(0);
  const uint32_t log = (bits & 0xFu) + 5u;
  if (log > max_log) return false;
  bits >>= 4;
  int32_t bit_count = 4;
  int32_t nb = static_cast<int32_t>(log) + 1;
  int32_t remaining = (1 << log) + 1;
  int32_t threshold = 1 << log;
  bool prev0 = false;
  uint32_t s = 0;
  while (remaining > 1 && s <= max_sym) {
    if (prev0) {
      uint32_t n0 = s;
      while ((bits & 0xFFFFu) == 0xFFFFu) {
        n0 += 24;
        ip += 2;
        bits = rd32(ip) >> bit_count;
      }
      while ((bits & 3u) == 3u) {
        n0 += 3;
        bits >>= 2;
        bit_count += 2;
      }
      n0 += bits & 3u;
      bit_count += 2;
      if (n0 > max_sym) return false;
      while (s < n0) counts[s++] = 0;
      ip += static_cast<uint32_t>(bit_count >> 3);
      bit_count &= 7;
      bits = rd32(ip) >> bit_count;
    }
    const int32_t mx = (2 * threshold - 1) - remaining;
    int32_t count;
    if (static_cast<int32_t>(bits & static_cast<uint32_t>(threshold - 1)) < mx) {
      count = static_cast<int32_t>(bits & static_cast<uint32_t>(threshold - 1));
      bit_count += nb - 1;
    } else {
      count = static_cast<int32_t>(bits & static_cast<uint32_t>(2 * threshold - 1));
      if (count >= threshold) count -= mx;
      bit_count += nb;
    }
    count -= 1;
    remaining -= count < 0 ? -count : count;
    counts[s++] = static_cast<int16_t>(count);
    prev0 = count == 0;
    while (remaining < threshold) {
      nb -= 1;
      threshold >>= 1;
    }
    ip += static_cast<uint32_t>(bit_count >> 3);
    bit_count &= 7;
    bits = rd32(ip) >> bit_count;
  }
  if (remaining != 1 || bit_count > 32) return false;
  const uint32_t u = ip + static_cast<uint32_t>((bit_count + 7) >> 3);
  if (u > len) return false;
  *nsym = s;
  *log_out = log;
  *used = u;
  return true;
}

// A decode entry as the table keeps it, symbol | nextState << 6 (u16:
// symbols < 64, next states < 1024), expanded to symbol | nbBits << 8 |
// baseline << 16: nbBits = log - highbit(nextState), baseline = (nextState
// << nbBits) - (1 << log) (FSE_buildDTable's own formulas).
__device__ __forceinline__ uint32_t fse_entry(uint32_t e16, uint32_t log) {
  const uint32_t ns = e16 >> 6;
  const uint32_t nb = log - (31u - __builtin_clz(ns));
  return (e16 & 63u) | (nb << 8) | (((ns << nb) - (1u << log)) << 16);
}

// Spread and decode entries for counts[0, nsym) at accuracy `log` into
// table (1 << log u16 entries, <= 512). `nxt` holds the per-symbol next state,
// `syms` (>= 512 bytes) the symbols in spread order.
//
// FSE_buildDTable walks the positions p_j = j * step mod size, skipping the
// low-probability slots at the top, and gives the k-th position it keeps to
// the k-th symbol of the counts laid end to end. Here every j at once: its
// rank among the kept positions (ballot), the symbol of that rank (the
// symbols' first ranks marked, then a running max), one scatter.
__device__ bool build_fse(const int16_t* counts, uint32_t nsym, uint32_t log, uint16_t* table,
                          uint16_t* nxt, uint8_t* syms, uint32_t lane) {
  const uint32_t size = 1u << log;
  const uint64_t below = (uint64_t{1} << lane) - 1u;
  for (uint32_t r = lane; r < size; r += 64) syms[r] = 0;
  __builtin_amdgcn_s_waitcnt(0xc07f);
  // symbols with count -1 at the top, in order; next states start at the
  // count (1 for those); each positive count's first rank marked
  uint32_t nlow = 0, cum = 0;
  for (uint32_t g = 0; g < nsym; g += 64) {
    const uint32_t s = g + lane;
    const int32_t c = s < nsym ? counts[s] : 0;
    const bool low = c == -1;
    const uint64_t m = __ballot(low);
    if (low) table[size - 1u - (nlow + __popcll(m & below))] = s;
    nlow += __popcll(m);
    const uint32_t pc = c > 0 ? static_cast<uint32_t>(c) : 0u;
    uint32_t incl = pc;
    for (uint32_t d = 1; d < 64; d <<= 1) {
      const uint32_t v = __shfl_up(incl, d);
      if (lane >= d) incl += v;
    }
    if (s < nsym) nxt[s] = static_cast<uint16_t>(low ? 1 : c);
    if (pc != 0 && cum + incl - pc < size) syms[cum + incl - pc] = static_cast<uint8_t>(s);
    cum += uni(__shfl(incl, 63));
  }
  const uint32_t kept = size - nlow;  // (high + 1)
  if (nlow > size || cum != kept) return false;
  __builtin_amdgcn_s_waitcnt(0xc07f);
  // symbol of every rank: the running max of the marks (symbols ascend)
  uint32_t carry = 0;
  for (uint32_t r0 = 0; r0 < kept; r0 += 64) {
    const uint32_t r = r0 + lane;
    uint32_t v = r < kept ? syms[r] : 0u;
    v = v > carry ? v : carry;
    for (uint32_t d = 1; d < 64; d <<= 1) {
      const uint32_t o = __shfl_up(v, d);
      if (lane >= d && o > v) v = o;
    }
    if (r < kept) syms[r] = static_cast<uint8_t>(v);
    carry = uni(__shfl(v, 63));
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);
  const uint32_t step = (size >> 1) + (size >> 3) + 3u;
  const uint32_t mask = size - 1u;
  uint32_t rank = 0;
  for (uint32_t j0 = 0; j0 < size; j0 += 64) {
    const uint32_t j = j0 + lane;
    const uint32_t t = (j * step) & mask;
    const bool keep = j < size && t < kept;
    const uint64_t m = __ballot(keep);
    if (keep) table[t] = syms[rank + __popcll(m & below)];
    rank += __popcll(m);
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);
  // decode entries in table order: symbol s's k-th entry gets state
  // nxt[s] + k. 64 entries a step: a lane's rank among the step's entries of
  // its symbol (the lanes sharing its symbol, one ballot per distinct
  // symbol); the last of each symbol carries nxt[s] on.
  for (uint32_t c = 0; c < size; c += 64) {
    const uint32_t u = c + lane;
    const bool in = u < size;
    const uint32_t s = in ? (table[u] & 63u) : 0x1000u;
    uint64_t todo = __ballot(in), peers = 0;
    while (todo) {
      const uint32_t sl = __builtin_amdgcn_readlane(s, static_cast<uint32_t>(__builtin_ctzll(todo)));
      const uint64_t m = __ballot(s == sl);
      if (s == sl) peers = m;
      todo &= ~m;
    }
    const uint32_t before = __popcll(peers & below);
    const bool last = (peers >> lane) == 1u;
    const uint32_t ns = (in ? nxt[s] : 1u) + before;
    __builtin_amdgcn_s_waitcnt(0xc07f);  // every lane has read nxt before it moves
    if (in) {
      table[u] = static_cast<uint16_t>(s | (ns << 6));  // (fse_entry expands it)
      if (last) nxt[s] = static_cast<uint16_t>(ns + 1u);
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
  }
  return true;
}

// Baselines and extra bits of the LL / ML codes (RFC 8878 §3.1.1.3.2.1)
__constant__ uint32_t kLLBase[36] = {0,    1,    2,    3,     4,     5,     6,    7,    8,
                                     9,    10,   11,   12,    13,    14,    15,   16,   18,
                                     20,   22,   24,   28,    32,    40,    48,   64,   128,
                                     256,  512,  1024, 2048,  4096,  8192,  16384, 32768, 65536};
__constant__ uint8_t kLLBits[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  0,  0,  1,  1,
                                    1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
__constant__ uint32_t kMLBase[53] = {3,  4,  5,  6,  7,  8,  9,  10,  11,  12,   13,   14,   15,  16,
                                     17, 18, 19, 20, 21, 22, 23, 24,  25,  26,   27,   28,   29,  30,
                                     31, 32, 33, 34, 35, 37, 39, 41,  43,  47,   51,   59,   67,  83,
                                     99, 131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771, 65539};
__constant__ uint8_t kMLBits[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  0,  0,  0,
                                    0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1,  1,  1,  1,
                                    2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};

// ---- LDS layout -----------------------------------------------------------

struct Lds {
  uint8_t* in;      // the staged frame (+16 zero bytes)
  uint8_t* out;     // the frame's output
  uint16_t* huf;    // Huffman decode table: symbol | nbBits << 8 (2048; a 12-bit
                    // tree in split form, huf_table)
  uint8_t* hside;   // a 12-bit tree's second symbols of its split entries (128)
  uint16_t* ll;     // FSE tables: 512 / 256 / 512 entries, and 64 for weights
  uint16_t* of;     // (u16: symbol | nextState << 6, fse_entry)
  uint16_t* ml;
  uint16_t* wt;
  int16_t* cnt;     // normalized counts scratch (256: the weights' FSE may name 256)
  uint16_t* nxt;    // FSE next-state scratch (256)
  uint8_t* sym;     // FSE spread scratch (512)
};

constexpr uint32_t kHufEntries = 2048, kFseLL = 512, kFseOF = 256, kFseML = 512, kFseW = 64;

__host__ __device__ constexpr uint32_t zstd_in_cap(uint32_t out_cap) {
  // ZSTD_compressBound(out_cap) (1.4.9): every frame the library writes
  return out_cap + (out_cap >> 8) + (out_cap < (128u << 10) ? ((128u << 10) - out_cap) >> 11 : 0u);
}
__host__ __device__ constexpr uint32_t round16(uint32_t x) { return (x + 15u) & ~15u; }
constexpr uint32_t kTabBytes =
    2u * kHufEntries + 128u + 2u * (kFseLL + kFseOF + kFseML + kFseW) + 512u + 512u + 512u;
__host__ __device__ constexpr uint32_t zstd_lds_bytes(uint32_t out_cap) {
  return round16(zstd_in_cap(out_cap) + 16u + 4u) + round16(out_cap) + kTabBytes;
}
// The HBM-output kernel's input window: a compressed block (< 128 KiB) from
// any 4-aligned start, + slack for the register-window reads past its end.
constexpr uint32_t kZWin = (128u << 10) + 64u, kZWinBytes = kZWin + 512u, kZBigChunk = 32;
constexpr uint32_t kZBigLds = kZWinBytes + kTabBytes;

// in_bytes of input staging, then out_bytes of output (0: the output is in
// HBM), then the tables
__device__ __forceinline__ Lds lds_layout(uint8_t* smem, uint32_t in_bytes, uint32_t out_bytes) {
  Lds L;
  uint32_t o = 0;
  L.in = smem;
  o += in_bytes;
  L.out = smem + o;
  o += out_bytes;
  L.huf = reinterpret_cast<uint16_t*>(smem + o);
  o += 2u * kHufEntries;
  L.hside = smem + o;
  o += 128u;
  L.ll = reinterpret_cast<uint16_t*>(smem + o);
  o += 2u * kFseLL;
  L.of = reinterpret_cast<uint16_t*>(smem + o);
  o += 2u * kFseOF;
  L.ml = reinterpret_cast<uint16_t*>(smem + o);
  o += 2u * kFseML;
  L.wt = reinterpret_cast<uint16_t*>(smem + o);
  o += 2u * kFseW;
  L.cnt = reinterpret_cast<int16_t*>(smem + o);
  o += 512u;
  L.nxt = reinterpret_cast<uint16_t*>(smem + o);
  o += 512u;
  L.sym = smem + o;
  return L;
}

// ---- Huffman (RFC 8878 §4.2; HUF_readStats / HUF_readDTableX1) -----------

// s_memtime into a frame's stamp slot k (probe build only: a vector store
// from every lane, the same value, so that no lane-dependent branch splits
// the parser's uniform control flow)
__device__ __forceinline__ void zstamp(uint64_t* slot, uint32_t k, uint32_t) {
#ifdef LVKV_PROBE_BUILD
  if (slot != nullptr) slot[k] = __builtin_amdgcn_s_memtime();
#else
  (void)slot;
  (void)k;
#endif
}

// The tree description at in[p, end): the weights in registers (symbol
// 64 g + lane's in w[g], zeros past the last; with the implied last), *nw =
// symbols, *maxbits, *used. Uniform control flow; no LDS stores in the
// serial loop (a store there would make every step wait on lgkmcnt).
__device__ bool huf_weights(const Lds& L, uint32_t p, uint32_t end, uint32_t (&w)[4],
                            uint32_t* nw, uint32_t* maxbits, uint32_t* used, uint32_t lane,
                            uint32_t* fail, uint64_t* stamp) {
  zstamp(stamp, 8, lane);
  if (p >= end) return *fail = kFHufHdr, false;
  const uint32_t hb = ldb(L.in, p);
  uint32_t n = 0;
#pragma unroll
  for (uint32_t g = 0; g < 4; ++g) w[g] = 0;
  // weight v of symbol i (uniform i): one lane of one register
  auto put = [&](uint32_t i, uint32_t v) {
    const bool me = lane == (i & 63u);
#pragma unroll
    for (uint32_t g = 0; g < 4; ++g)
      if ((i >> 6) == g) w[g] = me ? v : w[g];
  };
  if (hb >= 128) {  // direct 4-bit weights
    n = hb - 127u;
    const uint32_t nbytes = (n + 1u) >> 1;
    if (p + 1u + nbytes > end) return *fail = kFHufHdr, false;
#pragma unroll
    for (uint32_t g = 0; g < 4; ++g) {
      const uint32_t i = 64u * g + lane;
      if (i < n) {
        const uint32_t b = L.in[p + 1u + (i >> 1)];
        w[g] = (i & 1u) ? (b & 15u) : (b >> 4);
      }
    }
    *used = 1u + nbytes;
  } else {  // FSE-compressed weights, two interleaved states
    if (hb == 0 || p + 1u + hb > end) return *fail = kFHufHdr, false;
    uint32_t nsym, log, nc;
    if (!read_ncount(L.in, p + 1u, p + 1u + hb, 255u, 6u, L.cnt, &nsym, &log, &nc, lane))
      return *fail = kFNcount, false;
    zstamp(stamp, 9, lane);
    if (!build_fse(L.cnt, nsym, log, L.wt, L.nxt, L.sym, lane)) return *fail = kFFseSpread, false;
    zstamp(stamp, 10, lane);
    // the <= 64-entry table and the <= 127-byte stream in registers: each
    // step is a readlane, a shift and an add (both states share the stream)
    const uint32_t lo = p + 1u + nc, hi = p + 1u + hb;
    if (hi <= lo || ldb(L.in, hi - 1) == 0) return *fail = kFHufWeights, false;
    const uint32_t treg = fse_entry(L.wt[lane], log);
    // lane k + 1 holds the stream's dword k, lane 0 zeros: bit x of the
    // stream is bit x + 32 of the lanes' concatenation, and the bits below
    // its start (x < 0, at most 12 of them) read as zeros with no test
    const uint32_t sd = lane == 0 ? 0u : ld32(L.in, lo + 4u * (lane - 1u));
    __builtin_amdgcn_s_waitcnt(0xc07f);
    int32_t pos = static_cast<int32_t>(8u * (hi - lo - 1u) +
                                       (31u - __builtin_clz(ldb(L.in, hi - 1))));
    auto rd = [&](uint32_t nb) -> uint32_t {  // br_read on the registers (nb <= 6)
      pos -= static_cast<int32_t>(nb);
      const uint32_t q = static_cast<uint32_t>(pos + 32);
      // (readlane returns int: widen through uint32_t, not by sign)
      const uint32_t w0 = __builtin_amdgcn_readlane(sd, q >> 5);
      const uint32_t w1 = __builtin_amdgcn_readlane(sd, (q >> 5) + 1u);
      const uint64_t x = (static_cast<uint64_t>(w1) << 32) | w0;
      return static_cast<uint32_t>(x >> (q & 31u)) & ((1u << nb) - 1u);
    };
    auto entry = [&](uint32_t s) -> uint32_t { return __builtin_amdgcn_readlane(treg, s); };
    // (lane 0 stores the weights into the spread scratch, free again: one
    // ds_write a weight, nothing waits on it inside the loop)
    uint8_t* ws = L.sym;
    uint32_t s1 = rd(log), s2 = rd(log);
    for (;;) {
      if (n > 253u) return *fail = kFHufWeights, false;
      uint32_t e = entry(s1);
      if (lane == 0) ws[n] = static_cast<uint8_t>(e);
      ++n;
      s1 = (e >> 16) + rd((e >> 8) & 255u);
      if (pos < 0) {
        if (lane == 0) ws[n] = static_cast<uint8_t>(entry(s2));
        ++n;
        break;
      }
      if (n > 253u) return *fail = kFHufWeights, false;
      e = entry(s2);
      if (lane == 0) ws[n] = static_cast<uint8_t>(e);
      ++n;
      s2 = (e >> 16) + rd((e >> 8) & 255u);
      if (pos < 0) {
        if (lane == 0) ws[n] = static_cast<uint8_t>(entry(s1));
        ++n;
        break;
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
#pragma unroll
    for (uint32_t g = 0; g < 4; ++g) {
      const uint32_t i = 64u * g + lane;
      w[g] = i < n ? ws[i] : 0u;
    }
    *used = 1u + hb;
    zstamp(stamp, 11, lane);
  }
  // total weight, the implied last weight, and rank 1's count
  uint32_t total = 0, bad = 0;
#pragma unroll
  for (uint32_t g = 0; g < 4; ++g) {
    bad |= w[g] > 11u;
    total += (1u << (w[g] & 15u)) >> 1;
  }
  for (uint32_t d = 32; d >= 1; d >>= 1) {
    total += __shfl_xor(total, d);
    bad |= __shfl_xor(bad, d);
  }
  total = uni(total);
  bad = uni(bad);
  if (bad || total == 0) return *fail = kFHufWeights, false;
  const uint32_t mb = 32u - __builtin_clz(total);  // highbit(total) + 1
  // HUF_TABLELOG_MAX: a tree of up to 12 bits decodes (1.4.9's DTable holds 12)
  if (mb > 12u) return *fail = kFHufWeights, false;
  const uint32_t rest = (1u << mb) - total;
  if (rest & (rest - 1u)) return *fail = kFHufWeights, false;
  put(n++, 32u - __builtin_clz(rest));
  uint32_t r1 = 0;
#pragma unroll
  for (uint32_t g = 0; g < 4; ++g) r1 += w[g] == 1u ? 1u : 0u;
  for (uint32_t d = 32; d >= 1; d >>= 1) r1 += __shfl_xor(r1, d);
  r1 = uni(r1);
  if (r1 < 2u || (r1 & 1u)) return *fail = kFHufWeights, false;
  *nw = n;
  *maxbits = mb;
  return true;
}

// Decode table: symbols by weight, then by symbol value, each over
// 2^(w-1) entries of 2^maxbits.
// A level at a time: its symbols listed in order (ballot ranks, into the
// nxt scratch), then its entries filled 64 at a time from the list.
// A 12-bit tree (HUF_TABLELOG_MAX) keeps 2048 entries indexed by the top 11
// bits: its weight-1 symbols (12-bit codes, an even count, first in the
// table) pair up into split entries (nbBits field 15; the symbol of the
// 12th bit 0 in the entry, of bit 1 in hside), every other level fills
// 2^(w-2) entries with its real bit count.
__device__ void huf_table(const Lds& L, const uint32_t (&w)[4], uint32_t mb, uint32_t lane) {
  uint8_t* list = reinterpret_cast<uint8_t*>(L.nxt);
  const uint64_t below = (uint64_t{1} << lane) - 1u;
  const bool wide = mb == 12u;
  uint32_t pos = 0, lpos = 0;
  for (uint32_t wgt = 1; wgt <= mb; ++wgt) {
    const uint32_t lpos0 = lpos;
#pragma unroll
    for (uint32_t g = 0; g < 4; ++g) {
      const bool mine = w[g] == wgt;
      const uint64_t m = __ballot(mine);
      if (mine) list[lpos + __popcll(m & below)] = static_cast<uint8_t>(64u * g + lane);
      lpos += __popcll(m);
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    const uint32_t cnt = lpos - lpos0;
    if (wide && wgt == 1u) {  // pairs of 12-bit codes
      for (uint32_t k = lane; 2u * k < cnt; k += 64) {
        L.huf[k] = static_cast<uint16_t>(list[lpos0 + 2u * k] | (15u << 8));
        L.hside[k] = list[lpos0 + 2u * k + 1u];
      }
      pos += cnt >> 1;
      continue;
    }
    const uint32_t sh = wide ? wgt - 2u : wgt - 1u;  // log2 of a symbol's span
    const uint32_t n = cnt << sh;
    const uint32_t e = (mb + 1u - wgt) << 8;
    for (uint32_t k = lane; k < n; k += 64)
      L.huf[pos + k] = static_cast<uint16_t>(list[lpos0 + (k >> sh)] | e);
    pos += n;
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);
}

// Symbols that start above bit `floor`, from bit position `pos` down (one
// lane's segment of a stream at in[lo, ...)): the exit position; *count
// symbols, the first `lim` of them written at dst (when dst is set).
template <bool Wide>
__device__ __forceinline__ int32_t huf_run(const Lds& L, uint32_t lo, int32_t pos, int32_t floor,
                                           uint32_t mb, uint8_t* dst, uint32_t lim,
                                           uint32_t* count) {
  int32_t wlo = 0x7fffffff;
  uint64_t win = 0;
  const uint32_t mask = (1u << mb) - 1u;
  uint32_t c = 0;
  while (pos > floor) {
    // the window holds bits [wlo, wlo + 64): refilled so that it covers the
    // next four symbols (<= 48 bits); near the stream's start it is the
    // first 64 bits and an index below bit 0 shifts up, zeros below
    if (pos - 4 * static_cast<int32_t>(mb) < wlo && wlo > 0) {
      int32_t cb = ((pos + 7) >> 3) - 8;
      if (cb < 0) cb = 0;
      wlo = 8 * cb;
      win = ld64(L.in, lo + static_cast<uint32_t>(cb));
    }
    // four symbols without a branch: a lane past its floor reads and drops
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const bool live = pos > floor;
      const int32_t d = pos - static_cast<int32_t>(mb) - wlo;
      const uint32_t idx = static_cast<uint32_t>(d >= 0 ? win >> d : win << -d) & mask;
      uint32_t e;
      if (Wide) {  // 2048 entries by the top 11 of 12 bits; split entries
        e = L.huf[idx >> 1];
        if ((e >> 8) == 15u) e = ((idx & 1u) ? L.hside[idx >> 1] : (e & 255u)) | (12u << 8);
      } else {
        e = L.huf[idx];
      }
      if (dst != nullptr && live && c < lim) dst[c] = static_cast<uint8_t>(e & 255u);
      pos -= live ? static_cast<int32_t>(e >> 8) : 0;
      c += live ? 1u : 0u;
    }
  }
  *count = c;
  return pos;
}
__device__ __forceinline__ int32_t huf_run_any(const Lds& L, uint32_t lo, int32_t pos,
                                               int32_t floor, uint32_t mb, uint8_t* dst,
                                               uint32_t lim, uint32_t* count) {
  return mb == 12u ? huf_run<true>(L, lo, pos, floor, mb, dst, lim, count)
                   : huf_run<false>(L, lo, pos, floor, mb, dst, lim, count);
}

// ---- a frame --------------------------------------------------------------

struct Frame {
  uint32_t hsize;   // header bytes
  uint64_t csize;   // content size (~0 unknown)
  uint32_t single, checksum, dict;
  bool ok;
};

// RFC 8878 §3.1.1.1 at g[0, n) (any memory); ok = false when malformed.
template <typename Rd>
__device__ Frame frame_header(Rd rd, uint32_t n) {
  Frame f{};
  f.ok = false;
  f.csize = ~uint64_t{0};
  if (n < 5) return f;
  const uint32_t magic = rd(0) | rd(1) << 8 | rd(2) << 16 | rd(3) << 24;
  if (magic != kMagic) return f;
  const uint32_t fhd = rd(4);
  if (fhd & 8u) return f;
  const uint32_t fcs_flag = fhd >> 6;
  f.single = (fhd >> 5) & 1u;
  f.checksum = (fhd >> 2) & 1u;
  const uint32_t did = (fhd & 3u) == 3u ? 4u : (fhd & 3u);
  uint32_t p = 5;
  if (!f.single) {
    if (p >= n) return f;
    if (10u + (rd(p) >> 3) > 31u) return f;
    ++p;
  }
  const uint32_t fcs_size = fcs_flag == 0 ? f.single : (1u << fcs_flag);
  if (p + did + fcs_size > n) return f;
  uint32_t d = 0;
  for (uint32_t k = 0; k < did; ++k) d |= rd(p + k) << (8 * k);
  f.dict = d;
  p += did;
  if (fcs_size) {
    uint64_t v = 0;
    for (uint32_t k = 0; k < fcs_size; ++k) v |= static_cast<uint64_t>(rd(p + k)) << (8 * k);
    if (fcs_size == 2) v += 256;
    f.csize = v;
  }
  p += fcs_size;
  f.hsize = p;
  f.ok = true;
  return f;
}

struct ZArgs {
  const uint8_t* src;
  const uint64_t* src_off;
  const uint32_t* src_len;
  uint8_t* dst;
  const uint64_t* dst_off;
  const uint32_t* dst_cap;  // nullptr: lengths only
  uint32_t* out_len;
  uint8_t* status;
  uint32_t* detail;  // debug: the failure site per block (nullptr: none)
  uint32_t nblocks;
  uint32_t out_cap;
  uint32_t block_mode;  // ReadBlock mode: handles, type byte 2 only, LVKV_READ_*
  const uint8_t* vstatus;
  uint64_t* stamps;  // probe build: 16 clock stamps a frame (nullptr: none)
};


// One compressed block's literals at the end of the frame's output space
// (out_end - n: the output, which grows from the front, reaches a literal
// only once it is consumed; any block that would overrun fails its size
// checks first); *nlit, *used. Uniform.
__device__ bool literals(const Lds& L, uint32_t p, uint32_t end, uint32_t cap, uint8_t* out_end,
                         bool* have_tree, uint32_t* mb_tree, uint32_t* nlit, uint32_t* used,
                         uint32_t lane, uint32_t* fail, uint64_t* stamp) {
  if (end - p < 3u) return *fail = kFLitHdr, false;  // MIN_CBLOCK_SIZE
  const uint32_t b0 = ldb(L.in, p);
  const uint32_t type = b0 & 3u, sf = (b0 >> 2) & 3u;
  if (type <= 1u) {  // raw / RLE
    uint32_t n, hs;
    if (sf == 0 || sf == 2) {
      n = b0 >> 3;
      hs = 1;
    } else if (sf == 1) {
      n = (b0 >> 4) + (ldb(L.in, p + 1) << 4);
      hs = 2;
    } else {
      n = (b0 >> 4) + (ldb(L.in, p + 1) << 4) + (ldb(L.in, p + 2) << 12);
      hs = 3;
    }
    if (n > kBlockMax) return *fail = kFLitSize, false;
    if (n > cap) return *fail = kFCap, false;
    if (type == 0) {
      if (p + hs + n > end) return *fail = kFLitSize, false;
      uint8_t* lits = out_end - n;
      for (uint32_t k = lane; k < n; k += 64) lits[k] = L.in[p + hs + k];
      *used = hs + n;
    } else {
      if (p + hs + 1u > end) return *fail = kFLitSize, false;
      const uint8_t v = static_cast<uint8_t>(ldb(L.in, p + hs));
      uint8_t* lits = out_end - n;
      for (uint32_t k = lane; k < n; k += 64) lits[k] = v;
      *used = hs + 1u;
    }
    *nlit = n;
    return true;
  }
  const uint32_t hs = sf == 0 ? 3u : sf == 1 ? 3u : sf == 2 ? 4u : 5u;
  if (p + hs > end) return *fail = kFLitHdr, false;
  uint64_t hv = 0;
  for (uint32_t k = 0; k < hs; ++k) hv |= static_cast<uint64_t>(ldb(L.in, p + k)) << (8 * k);
  const uint32_t bits = sf <= 1u ? 10u : sf == 2 ? 14u : 18u;
  const uint32_t n = static_cast<uint32_t>(hv >> 4) & ((1u << bits) - 1u);
  const uint32_t csize = static_cast<uint32_t>(hv >> (4 + bits)) & ((1u << bits) - 1u);
  if (n > kBlockMax) return *fail = kFLitSize, false;
  if (p + hs + csize > end) return *fail = kFLitSize, false;
  if (n > cap) return *fail = kFCap, false;
  uint32_t q = p + hs;
  const uint32_t qend = p + hs + csize;
  if (type == 2) {
    uint32_t w[4], nw, mb, u;
    if (!huf_weights(L, q, qend, w, &nw, &mb, &u, lane, fail, stamp)) return false;
    zstamp(stamp, 6, lane);
    huf_table(L, w, mb, lane);
    zstamp(stamp, 7, lane);
    *have_tree = true;
    *mb_tree = mb;
    q += u;
  } else if (!*have_tree) {
    return *fail = kFHufHdr, false;
  }
  const uint32_t mb = *mb_tree;
  // the streams' bounds: one stream on 64 lanes, or four on 16 lanes each
  const uint32_t S = sf == 0 ? 64u : 16u;
  const uint32_t sid = lane / S, k = lane % S;
  uint32_t slo = q, shi = qend, scnt = n, sbase = 0;
  if (sf != 0) {
    if (qend - q < 10u) return *fail = kFJump, false;
    const uint32_t s1 = ldb(L.in, q) | ldb(L.in, q + 1) << 8;
    const uint32_t s2 = ldb(L.in, q + 2) | ldb(L.in, q + 3) << 8;
    const uint32_t s3 = ldb(L.in, q + 4) | ldb(L.in, q + 5) << 8;
    const uint32_t a = q + 6u, b = a + s1, c = b + s2, d = c + s3;
    if (d > qend) return *fail = kFJump, false;
    const uint32_t seg = (n + 3u) >> 2;
    if (3u * seg > n) return *fail = kFJump, false;
    slo = sid == 0 ? a : sid == 1 ? b : sid == 2 ? c : d;
    shi = sid == 0 ? b : sid == 1 ? c : sid == 2 ? d : qend;
    scnt = sid == 3 ? n - 3u * seg : seg;
    sbase = sid * seg;
  }
  bool good = shi > slo && L.in[shi - 1] != 0;  // the end marker (br_init)
  if (__ballot(!good)) return *fail = kFHufStream, false;
  const int32_t P = static_cast<int32_t>(8u * (shi - slo - 1u) +
                                         (31u - __builtin_clz(static_cast<uint32_t>(L.in[shi - 1]))));
  // Self-synchronising parallel decode: lane k of a stream takes the symbols
  // that start in bits (floor, top] of its segment. Pass A starts from the
  // segment's top (a guess), then each lane redoes its segment from the
  // exit of the lane before until no exit moves (the first lane's entry is
  // exact, so a pass in which nothing moves has exact entries everywhere),
  // then the symbols are written at their prefix-summed offsets.
  const int32_t seglen = (P + static_cast<int32_t>(S) - 1) / static_cast<int32_t>(S);
  const int32_t top = P - static_cast<int32_t>(k) * seglen;
  int32_t floor = P - static_cast<int32_t>(k + 1u) * seglen;
  if (floor < 0) floor = 0;
  uint32_t cnt = 0;
  int32_t x = huf_run_any(L, slo, top, floor, mb, nullptr, 0, &cnt);
  for (uint32_t it = 0; it < S; ++it) {
    int32_t entry = __shfl_up(x, 1, static_cast<int>(S));
    if (k == 0) entry = P;
    uint32_t c2 = 0;
    const int32_t x2 = huf_run_any(L, slo, entry, floor, mb, nullptr, 0, &c2);
    const bool moved = x2 != x;
    x = x2;
    cnt = c2;
    if (!__ballot(moved)) break;
  }
  uint32_t incl = cnt;
  for (uint32_t d = 1; d < S; d <<= 1) {
    const uint32_t v = __shfl_up(incl, d, static_cast<int>(S));
    if (k >= d) incl += v;
  }
  const uint32_t off = incl - cnt;
  const uint32_t total = __shfl(incl, static_cast<int>(S - 1u), static_cast<int>(S));
  const int32_t last = __shfl(x, static_cast<int>(S - 1u), static_cast<int>(S));
  int32_t entry = __shfl_up(x, 1, static_cast<int>(S));
  if (k == 0) entry = P;
  uint32_t c3 = 0;
  huf_run_any(L, slo, entry, floor, mb, out_end - n + sbase + off, scnt > off ? scnt - off : 0u,
          &c3);
  // the sequential decoder's verdict: exactly scnt symbols ending at bit 0
  good = total == scnt && last == 0;
  if (__ballot(!good)) return *fail = kFHufStream, false;
  __builtin_amdgcn_s_waitcnt(0xc07f);
  *nlit = n;
  *used = hs + csize;
  return true;
}

// A sequence table by mode into `table`; *log, *used. Uniform.
__device__ bool seq_table(const Lds& L, uint32_t p, uint32_t end, uint32_t mode,
                          const uint32_t* dflt, uint32_t dlog, uint32_t max_sym,
                          uint32_t max_log, uint16_t* table, bool* have, uint32_t* log,
                          uint32_t* used, uint32_t lane, uint32_t* fail) {
  *used = 0;
  if (mode == 0) {  // the predefined table (tools/gen_zstd_tables.py)
    for (uint32_t u = lane; u < (1u << dlog); u += 64) {  // (to the u16 form)
      const uint32_t e = dflt[u], nb = (e >> 8) & 255u;
      table[u] = static_cast<uint16_t>((e & 255u) | ((((e >> 16) + (1u << dlog)) >> nb) << 6));
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    *log = dlog;
  } else if (mode == 1) {
    if (p >= end) return *fail = kFRle, false;
    const uint32_t s = ldb(L.in, p);
    if (s > max_sym) return *fail = kFRle, false;
    if (lane == 0) table[0] = static_cast<uint16_t>(s | (1u << 6));  // (log 0: nextState 1)
    __builtin_amdgcn_s_waitcnt(0xc07f);
    *log = 0;
    *used = 1;
  } else if (mode == 2) {
    uint32_t nsym, lg, u;
    if (!read_ncount(L.in, p, end, max_sym, max_log, L.cnt, &nsym, &lg, &u, lane))
      return *fail = kFNcount, false;
    if (!build_fse(L.cnt, nsym, lg, table, L.nxt, L.sym, lane)) return *fail = kFFseSpread, false;
    *log = lg;
    *used = u;
  } else if (!*have) {
    return *fail = kFRepeat, false;
  }
  *have = true;
  return true;
}

struct SeqState {
  uint64_t* stamp;  // probe stamps of this frame, or nullptr
  // the LL / ML codes' baselines and extra bits, lane c holding code c's
  // (base | bits << 24): a v_readlane a sequence instead of constant-memory
  // loads (the u8 bit counts would be vector loads, waited on each time)
  uint32_t llcode, mlcode;
  bool have_ll, have_of, have_ml, have_tree;
  uint32_t ll_log, of_log, ml_log, mb_tree;
  uint32_t rep0, rep1, rep2;
  uint32_t flushed;  // HBM-output mode: every output byte below it has landed
};

// Copies n bytes from LDS `from` to out[op, ...): lanes 64 at a time. An
// overlapping match (off < n) repeats its first `off` bytes.
__device__ __forceinline__ void lds_copy(uint8_t* dst, const uint8_t* from, uint32_t n,
                                         uint32_t off, uint32_t lane) {
  if (off != 0 && off < n) {
    for (uint32_t k = lane; k < n; k += 64) dst[k] = from[k % off];
  } else {
    for (uint32_t k = lane; k < n; k += 64) dst[k] = from[k];
  }
}

// The block's tables as the sequence loop reads them: the first 64 entries
// in registers, and which tables fit there.
struct Tabs {
  uint32_t ll, of, ml;
  bool sll, sof, sml;
};

// The nseq sequences of a block (RFC 8878 §3.1.1.4-5): decode, execute, and
// the literals left after the last. Small: every table fits in registers.
template <bool Small, bool Global>
__device__ __forceinline__ bool sequences(const Lds& L, RegBits& r, SeqState& S, const Tabs& T,
                                          uint32_t nseq, uint32_t nlit, const uint8_t* lits,
                                          uint32_t* op, uint32_t frame_start, uint32_t cap,
                                          uint32_t lane, uint32_t* fail) {
  auto entry = [&](bool small, uint32_t reg, const uint16_t* t, uint32_t lg, uint32_t s) -> uint32_t {
    if (Small || small) return __builtin_amdgcn_readlane(reg, s);
    return fse_entry(uni(t[s]), lg);
  };
  uint32_t sl = rb_read(r, S.ll_log, lane), so = rb_read(r, S.of_log, lane),
           sm = rb_read(r, S.ml_log, lane);
  uint32_t lp = 0;
  for (uint32_t i = 0; i < nseq; ++i) {
    const uint32_t el = entry(T.sll, T.ll, L.ll, S.ll_log, sl),
                   eo = entry(T.sof, T.of, L.of, S.of_log, so),
                   em = entry(T.sml, T.ml, L.ml, S.ml_log, sm);
    const uint32_t llc = el & 255u, ofc = eo & 255u, mlc = em & 255u;
    const uint32_t lc = __builtin_amdgcn_readlane(S.llcode, llc);
    const uint32_t mc = __builtin_amdgcn_readlane(S.mlcode, mlc);
    const uint32_t mlb = mc >> 24, llb = lc >> 24;
    // the extra bits: offset, then ML and LL in one read (<= 16 + 16)
    const uint32_t ofx = rb_read(r, ofc, lane);
    const uint32_t mlx_llx = rb_read(r, mlb + llb, lane);
    const uint32_t llx = mlx_llx & ((1u << llb) - 1u), mlx = mlx_llx >> llb;
    const uint32_t ofv = (1u << ofc) + ofx;
    const uint32_t ml = (mc & 0xFFFFFFu) + mlx;
    const uint32_t ll = (lc & 0xFFFFFFu) + llx;
    uint32_t off;
    if (ofv > 3u) {
      off = ofv - 3u;
      S.rep2 = S.rep1;
      S.rep1 = S.rep0;
      S.rep0 = off;
    } else {
      const uint32_t idx = ofv - 1u + (ll == 0 ? 1u : 0u);
      if (idx == 0) {
        off = S.rep0;
      } else if (idx == 1) {
        off = S.rep1;
        S.rep1 = S.rep0;
        S.rep0 = off;
      } else if (idx == 2) {
        off = S.rep2;
        S.rep2 = S.rep1;
        S.rep1 = S.rep0;
        S.rep0 = off;
      } else {
        off = S.rep0 - 1u;
        S.rep2 = S.rep1;
        S.rep1 = S.rep0;
        S.rep0 = off;
      }
      if (off == 0) off = S.rep0 = 1;  // (1.4.9 forces a zero repeat offset to 1)
    }
    // the states, LL then ML then OF (also after the last sequence)
    {  // (<= 9 + 9 + 8 bits: one read)
      const uint32_t nl = (el >> 8) & 255u, nm = (em >> 8) & 255u, no = (eo >> 8) & 255u;
      const uint32_t v = rb_read(r, nl + nm + no, lane);
      sl = (el >> 16) + (v >> (nm + no));
      sm = (em >> 16) + ((v >> no) & ((1u << nm) - 1u));
      so = (eo >> 16) + (v & ((1u << no) - 1u));
    }
    if (ll > nlit - lp) return *fail = kFLitOverrun, false;
    if (ll + ml > cap - *op) return *fail = kFCap, false;
    lds_copy(L.out + *op, lits + lp, ll, 0, lane);
    lp += ll;
    *op += ll;
    if (off > *op - frame_start) return *fail = kFOffset, false;
    // (HBM output: a match that reads bytes whose stores may still be in
    // flight waits for them; recent offsets do, far ones mostly do not)
    if (Global && *op - off + (ml < off ? ml : off) > S.flushed) {
      __builtin_amdgcn_s_waitcnt(0);
      S.flushed = *op;
    }
    lds_copy(L.out + *op, L.out + (*op - off), ml, off, lane);
    *op += ml;
  }
  if (r.pos > 0) return *fail = kFSeqBits, false;
  zstamp(S.stamp, 4, lane);
  const uint32_t rest = nlit - lp;
  if (rest > cap - *op) return *fail = kFCap, false;
  lds_copy(L.out + *op, lits + lp, rest, 0, lane);
  *op += rest;
  return true;
}


// A compressed block at in[p, end): output appended at out[*op, ...).
// Global: out is the HBM destination (the literals' stores land before
// the sequences read them).
template <bool Global>
__device__ bool comp_block(const Lds& L, uint32_t p, uint32_t end, uint32_t* op,
                           uint32_t frame_start, uint32_t cap, SeqState& S, uint32_t lane,
                           uint32_t* fail) {
  uint32_t nlit, used;
  if (!literals(L, p, end, cap - *op, L.out + cap, &S.have_tree, &S.mb_tree, &nlit, &used, lane,
                fail, S.stamp))
    return false;
  if (Global) __builtin_amdgcn_s_waitcnt(0);
  const uint8_t* lits = L.out + (cap - nlit);
  zstamp(S.stamp, 2, lane);
  uint32_t q = p + used;
  if (q >= end) return *fail = kFSeqHdr, false;
  const uint32_t b0 = ldb(L.in, q);
  uint32_t nseq;
  if (b0 == 0) {
    nseq = 0;
    q += 1;
  } else if (b0 < 128) {
    nseq = b0;
    q += 1;
  } else if (b0 < 255) {
    if (q + 2 > end) return *fail = kFSeqHdr, false;
    nseq = ((b0 - 128u) << 8) + ldb(L.in, q + 1);
    q += 2;
  } else {
    if (q + 3 > end) return *fail = kFSeqHdr, false;
    nseq = ldb(L.in, q + 1) + (ldb(L.in, q + 2) << 8) + 0x7F00u;
    q += 3;
  }
  if (nseq == 0) {
    if (q != end) return *fail = kFSeqHdr, false;
    if (nlit > cap - *op) return *fail = kFCap, false;
    lds_copy(L.out + *op, lits, nlit, 0, lane);
    *op += nlit;
    return true;
  }
  if (q >= end) return *fail = kFSeqHdr, false;
  const uint32_t modes = ldb(L.in, q);
  ++q;
  uint32_t u;
  if (!seq_table(L, q, end, modes >> 6, kPredefLL, kPredefLLLog, 35, 9, L.ll, &S.have_ll, &S.ll_log,
                 &u, lane, fail))
    return false;
  q += u;
  if (!seq_table(L, q, end, (modes >> 4) & 3u, kPredefOF, kPredefOFLog, 31, 8, L.of, &S.have_of,
                 &S.of_log, &u, lane, fail))
    return false;
  q += u;
  if (!seq_table(L, q, end, (modes >> 2) & 3u, kPredefML, kPredefMLLog, 52, 9, L.ml, &S.have_ml,
                 &S.ml_log, &u, lane, fail))
    return false;
  q += u;
  zstamp(S.stamp, 3, lane);
  RegBits r;
  if (!rb_init(r, L.in, q, end, lane)) return *fail = kFSeqBits, false;
  // tables of <= 64 entries (the predefined ones, RLE, small FSE: a small
  // block's) are read from registers (v_readlane), larger ones from LDS; the
  // loop is built twice so that the common all-small case carries no
  // per-table branch (and no flags to spill)
  const uint32_t tll = fse_entry(L.ll[lane], S.ll_log), tof = fse_entry(L.of[lane], S.of_log),
                 tml = fse_entry(L.ml[lane], S.ml_log);
  __builtin_amdgcn_s_waitcnt(0xc07f);
  const Tabs T{tll, tof, tml, S.ll_log <= 6u, S.of_log <= 6u, S.ml_log <= 6u};
  if (T.sll && T.sof && T.sml)
    return sequences<true, Global>(L, r, S, T, nseq, nlit, lits, op, frame_start, cap, lane, fail);
  return sequences<false, Global>(L, r, S, T, nseq, nlit, lits, op, frame_start, cap, lane, fail);
}

// XXH64 of out[0, n) (seed 0): the frame checksum. Scalar, from LDS.
__device__ uint64_t rotl64(uint64_t x, uint32_t r) { return (x << r) | (x >> (64 - r)); }
__device__ __forceinline__ uint64_t xxh_merge(uint64_t h, uint64_t v, uint64_t P1, uint64_t P2,
                                              uint64_t P4) {
  h ^= rotl64(v * P2, 31) * P1;
  return h * P1 + P4;
}
// (base 4-aligned; the bytes are base[o, o + n))
__device__ __forceinline__ uint64_t xxh64(const uint8_t* base, uint32_t o, uint32_t n) {
  const uint64_t P1 = 11400714785074694791ull, P2 = 14029467366897019727ull,
                 P3 = 1609587929392839161ull, P4 = 9650029242287828579ull,
                 P5 = 2870177450012600261ull;
  uint32_t i = 0;
  uint64_t h;
  if (n >= 32) {
    uint64_t v1 = P1 + P2, v2 = P2, v3 = 0, v4 = 0 - P1;
    for (; i + 32 <= n; i += 32) {
      v1 = rotl64(v1 + ld64u(base, o + i) * P2, 31) * P1;
      v2 = rotl64(v2 + ld64u(base, o + i + 8) * P2, 31) * P1;
      v3 = rotl64(v3 + ld64u(base, o + i + 16) * P2, 31) * P1;
      v4 = rotl64(v4 + ld64u(base, o + i + 24) * P2, 31) * P1;
    }
    h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
    h = xxh_merge(h, v1, P1, P2, P4);
    h = xxh_merge(h, v2, P1, P2, P4);
    h = xxh_merge(h, v3, P1, P2, P4);
    h = xxh_merge(h, v4, P1, P2, P4);
  } else {
    h = P5;
  }
  h += n;
  for (; i + 8 <= n; i += 8) {
    h ^= rotl64(ld64u(base, o + i) * P2, 31) * P1;
    h = rotl64(h, 27) * P1 + P4;
  }
  if (i + 4 <= n) {
    h ^= static_cast<uint64_t>(ld32u(base, o + i)) * P1;
    h = rotl64(h, 23) * P2 + P3;
    i += 4;
  }
  for (; i < n; ++i) {
    h ^= ldb(base, o + i) * P5;
    h = rotl64(h, 11) * P1;
  }
  h ^= h >> 33;
  h *= P2;
  h ^= h >> 29;
  h *= P3;
  h ^= h >> 32;
  return h;
}

// XXH64 of p[0, n) in HBM (seed 0; any alignment): 1 KiB a round, four
// aligned dwords a lane (none starting past the end), the next round's
// loads issued before this round's 32 stripes are folded in by v_readlane.
__device__ __forceinline__ uint64_t xxh64_hbm(const uint8_t* p, uint32_t n, uint32_t lane) {
  const uint64_t P1 = 11400714785074694791ull, P2 = 14029467366897019727ull,
                 P3 = 1609587929392839161ull, P4 = 9650029242287828579ull,
                 P5 = 2870177450012600261ull;
  const uint32_t mis = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(p)) & 3u;
  const uint32_t* d = reinterpret_cast<const uint32_t*>(p - mis);
  const uint32_t nd = (mis + n + 3u) >> 2;
  // register j of round c: bytes p[1024 c + 256 j + 4 lane, + 4)
  auto fetch = [&](uint32_t c, uint32_t* w) {
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
      const uint32_t i = 256u * c + 64u * j + lane;
      const uint32_t lo = i < nd ? d[i] : 0u;
      const uint32_t hi = mis != 0 && i + 1u < nd ? d[i + 1u] : 0u;
      w[j] = __builtin_amdgcn_alignbyte(hi, lo, mis);
    }
  };
  auto dw = [&](const uint32_t* w, uint32_t b) -> uint32_t {  // the dword at round byte b
    const uint32_t j = b >> 8;
    const uint32_t v = j == 0 ? w[0] : j == 1 ? w[1] : j == 2 ? w[2] : w[3];
    return static_cast<uint32_t>(__builtin_amdgcn_readlane(v, (b >> 2) & 63u));
  };
  auto qw = [&](const uint32_t* w, uint32_t b) -> uint64_t {
    return static_cast<uint64_t>(dw(w, b + 4u)) << 32 | dw(w, b);
  };
  auto rnd = [&](uint64_t v, uint64_t x) { return rotl64(v + x * P2, 31) * P1; };
  uint32_t w[4], wn[4];
  fetch(0, w);
  uint32_t i = 0, c = 0;
  uint64_t h;
  if (n >= 32) {
    uint64_t v1 = P1 + P2, v2 = P2, v3 = 0, v4 = 0 - P1;
    for (;;) {
      fetch(c + 1u, wn);
      bool more = true;
#pragma unroll
      for (uint32_t s = 0; s < 32; ++s) {
        if (more && i + 32u <= n) {
          v1 = rnd(v1, qw(w, 32u * s));
          v2 = rnd(v2, qw(w, 32u * s + 8u));
          v3 = rnd(v3, qw(w, 32u * s + 16u));
          v4 = rnd(v4, qw(w, 32u * s + 24u));
          i += 32u;
        } else {
          more = false;
        }
      }
      if (!more) break;
#pragma unroll
      for (uint32_t j = 0; j < 4; ++j) w[j] = wn[j];
      ++c;
    }
    h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
    h = xxh_merge(h, v1, P1, P2, P4);
    h = xxh_merge(h, v2, P1, P2, P4);
    h = xxh_merge(h, v3, P1, P2, P4);
    h = xxh_merge(h, v4, P1, P2, P4);
  } else {
    h = P5;
  }
  h += n;
  // the < 32 bytes left, all in round c's registers
  for (; i + 8u <= n; i += 8u) {
    h ^= rotl64(qw(w, i & 1023u) * P2, 31) * P1;
    h = rotl64(h, 27) * P1 + P4;
  }
  if (i + 4u <= n) {
    h ^= static_cast<uint64_t>(dw(w, i & 1023u)) * P1;
    h = rotl64(h, 23) * P2 + P3;
    i += 4u;
  }
  for (; i < n; ++i) {
    h ^= ((dw(w, i & 1020u) >> (8u * (i & 3u))) & 255u) * P5;
    h = rotl64(h, 11) * P1;
  }
  h ^= h >> 33;
  h *= P2;
  h ^= h >> 29;
  h *= P3;
  h ^= h >> 32;
  return h;
}

// One stream b (RFC 8878 frames one after another). LDS mode: the stream
// staged whole, the output built in LDS and copied out; a stream past the
// staging is marked TOO_LARGE. Global (zstd_uncompress_big_kernel, for the
// streams so marked): the input read through a window of one block at a
// time (kZWin), the output written straight into the HBM destination.
template <bool Global>
__device__ __forceinline__ void zstd_stream(const ZArgs& a, uint32_t b, uint8_t* smem,
                                            uint32_t lane) {
  uint32_t n = uni(a.src_len[b]);
  const uint64_t so = a.src_off[b];
  const uint8_t* src =
      a.src + ((static_cast<uint64_t>(uni(static_cast<uint32_t>(so >> 32))) << 32) |
               uni(static_cast<uint32_t>(so)));
  auto finish = [&](uint32_t st, uint32_t ol, uint32_t why) {
    if (lane == 0) {
      a.status[b] = static_cast<uint8_t>(st);
      a.out_len[b] = ol;
      if (a.detail) a.detail[b] = why;
    }
  };
  // status codes: codec (LVKV_SNAPPY_*, shared) or ReadBlock's
  const uint32_t kOK = a.block_mode ? LVKV_READ_OK : LVKV_SNAPPY_OK;
  const uint32_t kLen = a.block_mode ? LVKV_READ_ZSTD_LENGTH : LVKV_SNAPPY_BAD_LENGTH;
  const uint32_t kBad = a.block_mode ? LVKV_READ_ZSTD_CONTENTS : LVKV_SNAPPY_BAD_CONTENTS;
  const uint32_t kCap = a.block_mode ? LVKV_READ_CAPACITY : LVKV_SNAPPY_CAPACITY;
  const uint32_t kBig = a.block_mode ? LVKV_READ_TOO_LARGE : LVKV_SNAPPY_TOO_LARGE;
  if (a.block_mode) {  // only type-2 blocks whose checksum held (the rest are done)
    if (ldb(src, n) != 2) return;
    // (Global: the mark this kernel's LDS pass left is the verdict slot)
    if (!Global && a.vstatus != nullptr && uni(a.vstatus[b]) != 0) return;
  }
  // port::Zstd_GetUncompressedLength: ZSTD_getFrameContentSize, false on 0
  // (a skippable frame reads as 0; a malformed header as ERROR, passed on)
  uint64_t csize;
  {
    // the first 24 bytes (a frame header is at most 18) in one round of
    // aligned dword loads, lanes 0-6; read back by v_readlane, not by a
    // chain of dependent byte loads from global memory
    const uint32_t mis = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(src)) & 3u;
    const uint32_t* s32 = reinterpret_cast<const uint32_t*>(src - mis);
    const uint32_t hd = lane < 7u && 4u * lane < mis + n ? s32[lane] : 0u;
    auto rd = [&](uint32_t i) -> uint32_t {  // byte i < min(n, 24)
      const uint32_t q = i + mis;
      return (static_cast<uint32_t>(__builtin_amdgcn_readlane(hd, q >> 2)) >> (8u * (q & 3u))) & 255u;
    };
    const uint32_t m = n >= 4 ? (rd(0) | rd(1) << 8 | rd(2) << 16 | rd(3) << 24) : 0u;
    if (n >= 4 && (m & 0xFFFFFFF0u) == 0x184D2A50u) {
      csize = n >= 8 ? 0 : ~uint64_t{1};
    } else {
      const Frame f = frame_header(rd, n);
      csize = f.ok ? f.csize : ~uint64_t{1};
    }
  }
  if (csize == 0) return finish(kLen, 0, kFOk);
  if (a.dst_cap == nullptr)  // (unknown, malformed and > 4 GiB sizes: TOO_LARGE)
    return csize > 0xFFFFFFFFull ? finish(kBig, 0xFFFFFFFFu, kFOk)
                                 : finish(kOK, static_cast<uint32_t>(csize), kFOk);
  const uint32_t cap = uni(a.dst_cap[b]);
  if (csize > cap) return finish(kCap, csize > 0xFFFFFFFFull ? 0xFFFFFFFFu : csize, kFOk);
  if (!Global && (csize > a.out_cap || n > zstd_in_cap(a.out_cap)))
    return finish(kBig, csize, kFOk);
  uint8_t* const dst = a.dst + a.dst_off[b];
  Lds L = Global ? lds_layout(smem, kZWinBytes, 0)
                 : lds_layout(smem, round16(zstd_in_cap(a.out_cap) + 16u + 4u), round16(a.out_cap));
  uint8_t* const win = L.in;
  if (Global) L.out = dst;
  uint64_t* stamp = a.stamps != nullptr ? a.stamps + 16u * b : nullptr;
  zstamp(stamp, 0, lane);
  const uint32_t llcode = lane < 36u ? kLLBase[lane] | static_cast<uint32_t>(kLLBits[lane]) << 24 : 0u;
  const uint32_t mlcode = lane < 53u ? kMLBase[lane] | static_cast<uint32_t>(kMLBits[lane]) << 24 : 0u;
  // the staged input: in[wbase, wend) (LDS mode: all of it)
  uint32_t wbase = 0, wend = n;
  auto ensure = [&](uint32_t lo, uint32_t hi) {  // in[lo, min(hi, n)) staged
    if (!Global) return;
    hi = hi < n ? hi : n;
    if (lo >= wbase && hi <= wend) return;
    __builtin_amdgcn_s_waitcnt(0);  // (reads of the old window done)
    wbase = lo & ~3u;
    const uint32_t wl = n - wbase < kZWin ? n - wbase : kZWin;
    wend = wbase + wl;
    stage(win, src + wbase, wl, 16, lane);
    __builtin_amdgcn_s_waitcnt(0);
    L.in = win - wbase;
  };
  if (Global) {
    wend = 0;
    ensure(0, 32);
  } else {
    stage(L.in, src, n, 16, lane);
    __builtin_amdgcn_s_waitcnt(0);
  }
  zstamp(stamp, 1, lane);
  // ZSTD_decompressDCtx(dst, csize, src, n): frames one after another
  const uint32_t ocap = static_cast<uint32_t>(csize);
  uint32_t p = 0, op = 0, fail = kFOk;
  bool ok = true;
  while (ok && p < n) {
    p = uni(p);  // (loop-carried parser state: pinned uniform, see uni())
    op = uni(op);
    const uint32_t rem = n - p;
    if (rem < 5) {  // (ZSTD_startingInputLength: input left over)
      ok = false;
      fail = kFTrailing;
      break;
    }
    ensure(p, p + 32u);
    const uint32_t m = ld32u(L.in, p);
    if ((m & 0xFFFFFFF0u) == 0x184D2A50u) {  // skippable frame
      if (rem < 8) {
        ok = false;
        fail = kFSkippable;
        break;
      }
      const uint32_t sz = ld32u(L.in, p + 4);
      if (sz > rem - 8) {
        ok = false;
        fail = kFSkippable;
        break;
      }
      p += 8 + sz;
      continue;
    }
    if (rem < 9) {
      ok = false;
      fail = kFHeader;
      break;
    }
    auto rd = [&](uint32_t i) -> uint32_t { return ldb(L.in, p + i); };
    const Frame f = frame_header(rd, rem);
    if (!f.ok) {
      ok = false;
      fail = kFHeader;
      break;
    }
    if (f.dict != 0) {
      ok = false;
      fail = kFDict;
      break;
    }
    uint32_t q = p + f.hsize;
    const uint32_t start = op;
    SeqState S{};
    S.stamp = stamp;
    S.llcode = llcode;
    S.mlcode = mlcode;
    S.rep0 = 1;
    S.rep1 = 4;
    S.rep2 = 8;
    S.flushed = start;
    for (;;) {
      q = uni(q);
      op = uni(op);
      if (q + 3 > n) {
        ok = false;
        fail = kFBlockHdr;
        break;
      }
      ensure(q, q + 3u);
      const uint32_t bh = ldb(L.in, q) | ldb(L.in, q + 1) << 8 | ldb(L.in, q + 2) << 16;
      q += 3;
      const uint32_t last = bh & 1u, btype = (bh >> 1) & 3u, bsize = bh >> 3;
      if (btype == 3) {
        ok = false;
        fail = kFBlockType;
        break;
      }
      if (btype == 1) {
        if (q + 1 > n) {
          ok = false;
          fail = kFBlockSize;
          break;
        }
        if (bsize > ocap - op) {
          ok = false;
          fail = kFCap;
          break;
        }
        ensure(q, q + 1u);
        const uint8_t v = static_cast<uint8_t>(ldb(L.in, q));
        for (uint32_t k = lane; k < bsize; k += 64) L.out[op + k] = v;
        op += bsize;
        q += 1;
      } else {
        if (btype == 2 && bsize >= kBlockMax) {
          ok = false;
          fail = kFBlockSize;
          break;
        }
        if (bsize > n - q) {
          ok = false;
          fail = kFBlockSize;
          break;
        }
        if (btype == 0) {
          if (bsize > ocap - op) {
            ok = false;
            fail = kFCap;
            break;
          }
          if (Global) {  // (HBM to HBM; a raw block may pass the window)
            for (uint32_t k = lane; k < bsize; k += 64) L.out[op + k] = src[q + k];
          } else {
            for (uint32_t k = lane; k < bsize; k += 64) L.out[op + k] = L.in[q + k];
          }
          op += bsize;
        } else {
          if (bsize < 3) {
            ok = false;
            fail = kFLitHdr;
            break;
          }
          ensure(q, q + bsize);
          if (!comp_block<Global>(L, q, q + bsize, &op, start, ocap, S, lane, &fail)) {
            ok = false;
            break;
          }
        }
        q += bsize;
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);
      if (last) break;
    }
    if (!ok) break;
    if (f.csize != ~uint64_t{0} && op - start != f.csize) {
      ok = false;
      fail = kFContentSize;
      break;
    }
    if (f.checksum) {
      if (q + 4 > n) {
        ok = false;
        fail = kFChecksum;
        break;
      }
      ensure(q, q + 4u);
      const uint32_t want = ld32u(L.in, q);
      uint64_t h;
      if (Global) {
        __builtin_amdgcn_s_waitcnt(0);
        h = xxh64_hbm(dst + start, op - start, lane);
      } else {
        h = xxh64(L.out, start, op - start);
      }
      if (static_cast<uint32_t>(h) != want) {
        ok = false;
        fail = kFChecksum;
        break;
      }
      q += 4;
    }
    p = q;
  }
  if (Global) __builtin_amdgcn_s_waitcnt(0);
  if (!ok) return finish(kBad, ocap, fail);
  if (op != ocap) return finish(kBad, ocap, kFContentSize);  // (short output)
  if (!Global) {
    uint32_t k0 = 0;
    if ((reinterpret_cast<uintptr_t>(dst) & 3u) == 0) {
      const uint32_t nd = op >> 2;
      for (uint32_t i = lane; i < nd; i += 64)
        reinterpret_cast<uint32_t*>(dst)[i] = reinterpret_cast<const uint32_t*>(L.out)[i];
      k0 = 4u * nd;
    }
    for (uint32_t k = k0 + lane; k < op; k += 64) dst[k] = L.out[k];
  }
  zstamp(stamp, 5, lane);
  finish(kOK, op, kFOk);
}

__global__ void __launch_bounds__(64) zstd_uncompress_kernel(ZArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t b = blockIdx.x;
  if (b >= a.nblocks) return;
  zstd_stream<false>(a, b, smem, threadIdx.x);
}

// The streams zstd_uncompress_kernel marked TOO_LARGE (a frame past the LDS
// staging, ReadBlock's any-size blocks), run after it on the same stream: a
// workgroup per 32 streams, their statuses in one load, the marked ones one
// after another (a batch without one costs a short launch).
__global__ void __launch_bounds__(64) zstd_uncompress_big_kernel(ZArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t lane = threadIdx.x;
  const uint32_t b0 = blockIdx.x * kZBigChunk;
  const uint32_t mark = a.block_mode ? LVKV_READ_TOO_LARGE : LVKV_SNAPPY_TOO_LARGE;
  const bool mine = lane < kZBigChunk && b0 + lane < a.nblocks && a.status[b0 + lane] == mark;
  uint64_t todo = __ballot(mine);
  while (todo) {
    const uint32_t b = b0 + static_cast<uint32_t>(__builtin_ctzll(todo));
    todo &= todo - 1u;
    zstd_stream<true>(a, b, smem, lane);
  }
}

}  // namespace

#ifdef LVKV_PROBE_BUILD
uint64_t* g_zstd_stamps = nullptr;  // lvkv_debug_zstd_stamps (tools/probe)
#endif

uint32_t zstd_lds(uint32_t max_ulen) { return zstd_lds_bytes(max(16u, max_ulen)); }

hipError_t launch_zstd_uncompress(const uint8_t* src, const uint64_t* src_off,
                                  const uint32_t* src_len, uint8_t* dst, const uint64_t* dst_off,
                                  const uint32_t* dst_cap, uint32_t* out_len, uint8_t* status,
                                  uint32_t* detail, uint32_t nblocks, uint32_t max_ulen,
                                  uint32_t block_mode, const uint8_t* vstatus,
                                  hipStream_t stream) {
  ZArgs a{src, src_off, src_len, dst, dst_off, dst_cap, out_len, status, detail, nblocks,
          0, block_mode, vstatus, nullptr};
#ifdef LVKV_PROBE_BUILD
  a.stamps = g_zstd_stamps;
#endif
  a.out_cap = dst_cap == nullptr ? 0u : max(16u, max_ulen);
  const size_t lds = dst_cap == nullptr ? 16u : zstd_lds_bytes(a.out_cap);
  hipLaunchKernelGGL(zstd_uncompress_kernel, dim3(nblocks), dim3(64), lds, stream, a);
  if (dst_cap != nullptr && nblocks != 0)  // (the streams past the LDS staging, any size)
    hipLaunchKernelGGL(zstd_uncompress_big_kernel,
                       dim3((nblocks + kZBigChunk - 1u) / kZBigChunk), dim3(64), kZBigLds,
                       stream, a);
  return hipGetLastError();
}

}  // namespace lvkv
