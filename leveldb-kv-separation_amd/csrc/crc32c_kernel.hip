// Batched CRC32C over many independent blocks — hand-written for gfx950.
//
// Replaces, for batches, the per-call loop of leveldb::crc32c::Extend
// (/root/reference/util/crc32c.cc:276-377) as used by the SST writer/reader
// (table/table_builder.cc:199-203, table/format.cc:92-99) and the WAL
// writer/reader (db/log_writer.cc:94-95, db/log_reader.cc:243-257).
//
// Algorithm (one wavefront per block, all integer, no MFMA):
//
//  * CRC32C is affine over GF(2). With raw(M, s) = the reflected register
//    after feeding M from state s, Extend(init, M) = raw(M, init^~0) ^ ~0,
//    and a 32-bit word w that ends d bytes before the end of the message
//    contributes Z_d(w), where Z_d = "advance the register over d zero bytes".
//  * The block is laid on a grid of 4-byte words that is aligned to the END of
//    the block; the grid is padded at the front with zero words (leading zeros
//    do not change raw(., 0)). The init state is xored into the first 4 data
//    bytes. Grid word idx of row r is handled by lane s = idx mod 64, so every
//    wave-wide load reads 256 contiguous bytes (one row).
//  * Lane s keeps a Horner accumulator S_s = Z_256(S_s) ^ w_r over the rows
//    (Z_256 from four LDS byte tables, 32 bank-private copies, addressed with
//    one v_perm_b32 each). At the end lane s applies its private end shift
//    Z_{256-4s} (eight LDS nibble tables) and the wave xor-reduces:
//       raw = XOR_s Z_{256-4s}(S_s).
//  * Block bytes are read through a buffer resource bounded to the dwords
//    that overlap the block, so front padding, rows past the end and the
//    prefetch of the next item come back as zeros without touching memory.
//    A block whose end is not 4-byte aligned is read as aligned dwords and
//    re-aligned with v_alignbyte (neighbour dword via ds_bpermute).
//
// Persistent grid: one 1024-thread workgroup per CU fills the 160 KiB LDS
// image once, then each wave walks blocks gw, gw + nwaves, ... in 4 KiB
// chunks with a two-stage register double buffer (issue chunk k+1 while
// consuming chunk k).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_device_common.h"
#include "lvkv_kernel_args.h"

namespace lvkv {
namespace {


// Cache policy of the block loads: nt (non-temporal). Block bytes are read
// exactly once; streaming them with nt keeps the 36 KiB of tables that every
// workgroup reloads at kernel start resident in the XCD's L2 across launches
// (without it the table loads miss and queue behind the whole batch in HBM).
constexpr int kDataCachePolicy = 2;

// Probe variants (timing experiments only; results are wrong except for 0
// and kProbeShflReduce). Bits combine.
enum : int {
  kProbeNone = 0,
  kProbeNoCompute = 1,    // loads + xor of the words, no LDS table work
  kProbeNoLoads = 2,      // no global loads, words = lane constants
  kProbeNoFill = 4,       // skip the LDS table fill
  kProbeShflReduce = 8,   // wave reduction via ds_bpermute shuffles
  kProbeEmpty = 16,       // return at once: launch + dispatch cost only
  // Not a probe: the uniform-stride specialisation (every block `length`
  // bytes at base + i*stride, every block END 4-byte aligned, length >= 4,
  // compute mode). All geometry is loop-invariant except the block address.
  kUniformAligned = 32,
  kProbeStamps = 64,      // record s_memrealtime per wave at phase edges
  kProbeLateLoads = 128,  // issue the first round only after the LDS fill
};

// Probe timeline: lane 0 of each wave writes 8 u64 slots (100 MHz realtime
// clock): 0 entry, 1 after the LDS fill barrier, 2.. after each round
// (capped), 7 exit.
template <int V>
__device__ __forceinline__ void stamp(const KernelArgs& a, uint32_t gw, int slot) {
  if (V & kProbeStamps) {
    const uint64_t t = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63u) == 0) a.stamps[gw * 8u + slot] = t;
  }
}

// Wave-uniform geometry of one block (lives in SGPRs).
// All fields are 32-bit so copies of Item carry no padding (padding bytes
// defeat SROA and end up in scratch).
struct Geo {
  uint32_t b4_lo;     // buffer window [b4, b4 + nrec) = [floor4(ptr), ceil4(end))
  uint32_t b4_hi;
  uint32_t nrec;
  int32_t vb0;        // byte offset of lane 0, row 0, relative to rsrc
  uint32_t rows;      // grid rows (the last chunk may be partial)
  uint32_t nchunks;   // chunks of kRowsPerChunk rows
  uint32_t e;         // grid misalignment vs dwords (0 = aligned)
  uint32_t s0l;       // first lane of row 0 that holds data
  uint32_t delta;     // bytes of front padding inside the first data word
  uint32_t s0;        // init ^ ~0, xored into the first 4 data bytes
  uint32_t spill;     // part of s0 that lands in the second data word
  uint32_t tiny;      // 1: length < 4, computed bitwise; 2: a long block left
                      //    to crc32c_long_kernel (no loads, no store)
  uint32_t len;
  uint32_t ptr_lo;    // absolute address of the first covered byte
  uint32_t ptr_hi;    //   (split: keeps the struct free of padding)
  uint32_t expected;  // verify modes: unmasked stored CRC
  __device__ __forceinline__ uint64_t ptr() const {
    return (static_cast<uint64_t>(ptr_hi) << 32) | ptr_lo;
  }
  // The descriptor inputs go through readfirstlane so the compiler can prove
  // the SRD wave-uniform; otherwise it wraps every buffer load in a
  // waterfall loop (cdna_hip_programming.md T20).
  __device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc() const {
    const uint32_t lo = __builtin_amdgcn_readfirstlane(b4_lo);
    const uint32_t hi = __builtin_amdgcn_readfirstlane(b4_hi);
    const uint32_t n = __builtin_amdgcn_readfirstlane(nrec);
    const uint64_t b = (static_cast<uint64_t>(hi) << 32) | lo;
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(b), 0,
                                             static_cast<int>(n),
                                             kBufferDword3);
  }
};

struct Item {
  uint32_t block;
  uint32_t chunk;
  Geo g;
};

__device__ __forceinline__ Geo null_geo() {
  Geo g;
  g.b4_lo = 0;
  g.b4_hi = 0;
  g.nrec = 0;
  g.vb0 = 0;
  g.rows = 0;
  g.nchunks = 1;
  g.e = 0;
  g.s0l = 0;
  g.delta = 0;
  g.s0 = 0;
  g.spill = 0;
  g.tiny = 1;
  g.len = 0;
  g.ptr_lo = 0;
  g.ptr_hi = 0;
  g.expected = 0;
  return g;
}

template <int V>
__device__ __forceinline__ Geo make_geo(const KernelArgs& a, uint32_t b) {
  if (V & kUniformAligned) {
    // Same shape for every block; only the window base moves.
    Geo g;
    const uint32_t len = a.length;
    const uint32_t q = (len + 3u) >> 2;
    const uint32_t rows = (q + 63u) >> 6;
    g.delta = 4u * q - len;
    g.s0l = 64u * rows - q;
    g.s0 = a.init ^ 0xffffffffu;
    g.spill = g.delta ? (g.s0 >> (32u - 8u * g.delta)) : 0u;
    g.e = 0;
    g.tiny = 0;
    g.len = len;
    g.expected = 0;
    g.nrec = (b < a.nblocks) ? 4u * q : 0u;
    g.vb0 = -4 * static_cast<int32_t>(g.s0l);
    g.rows = rows;
    g.nchunks = (rows + kRowsPerChunk - 1) / kRowsPerChunk;
    const uint64_t ptr = reinterpret_cast<uint64_t>(a.base) +
                         static_cast<uint64_t>(b) * a.stride;
    const uint64_t b4 = ptr - g.delta;  // end-aligned: floor4(ptr)
    g.ptr_lo = static_cast<uint32_t>(ptr);
    g.ptr_hi = static_cast<uint32_t>(ptr >> 32);
    g.b4_lo = static_cast<uint32_t>(b4);
    g.b4_hi = static_cast<uint32_t>(b4 >> 32);
    return g;
  }
  if (b >= a.nblocks) return null_geo();
  const uint64_t base = reinterpret_cast<uint64_t>(a.base);
  uint64_t off;
  uint32_t len, init = a.init, expected = 0;
  if (a.mode == kModeLogVerify || a.mode == kModeLogFill) {
    // Header [masked crc u32][len u16][type u8]; CRC covers type + payload
    // (db/log_reader.cc:217-221, 243-247).
    const uint64_t hoff = sload_u64(a.offsets, b);
    const uint64_t hdr = base + hoff;
    const uint32_t len_type = sload_le(hdr + 4, 3);
    if (a.mode == kModeLogVerify) expected = crc_unmask(sload_le(hdr, 4));
    off = hoff + 6;
    len = 1u + (len_type & 0xffffu);
    init = 0;
  } else if (a.offsets != nullptr) {
    off = sload_u64(a.offsets, b);
    len = sload_u32(a.lengths, b);
    if (a.inits != nullptr) init = sload_u32(a.inits, b);
  } else {
    off = static_cast<uint64_t>(b) * a.stride;
    len = a.length;
  }
  if (a.mode == kModeSstVerify || a.mode == kModeSstFill) {
    // Block contents n bytes + type byte are covered; the masked CRC follows
    // (table/format.cc:92-94, table/table_builder.cc:199-203).
    len += 1;
    init = 0;
    if (a.mode == kModeSstVerify) expected = crc_unmask(sload_le(base + off + len, 4));
  }

  if (a.long_split && len > kLongBytes) {  // crc32c_long_kernel's block
    Geo g = null_geo();
    g.tiny = 2;
    return g;
  }
  Geo g;
  const uint64_t ptr = base + off;
  g.ptr_lo = static_cast<uint32_t>(ptr);
  g.ptr_hi = static_cast<uint32_t>(ptr >> 32);
  g.len = len;
  g.s0 = init ^ 0xffffffffu;
  g.expected = expected;
  if (len < 4) {
    g.b4_lo = 0;
    g.b4_hi = 0;
    g.nrec = 0;
    g.tiny = 1;
    g.vb0 = 0;
    g.rows = 0;
    g.nchunks = 1;
    g.e = 0;
    g.s0l = 0;
    g.delta = 0;
    g.spill = 0;
    return g;
  }
  g.tiny = 0;
  const uint32_t q = (len + 3u) >> 2;        // grid words
  const uint32_t rows = (q + 63u) >> 6;
  g.delta = 4u * q - len;                    // 0..3
  g.s0l = 64u * rows - q;                    // 0..63
  g.spill = g.delta ? (g.s0 >> (32u - 8u * g.delta)) : 0u;
  const uint32_t m = static_cast<uint32_t>(ptr & 3u);
  const int32_t d = static_cast<int32_t>(m) - static_cast<int32_t>(g.delta);
  g.e = static_cast<uint32_t>(d) & 3u;
  const int32_t f = d >> 2;                  // -1 or 0
  const uint64_t b4 = ptr - m;
  const uint64_t end4 = (ptr + len + 3u) & ~uint64_t{3};
  g.b4_lo = static_cast<uint32_t>(b4);
  g.b4_hi = static_cast<uint32_t>(b4 >> 32);
  g.nrec = static_cast<uint32_t>(end4 - b4);
  g.vb0 = 4 * f - 4 * static_cast<int32_t>(g.s0l);
  g.rows = rows;
  g.nchunks = (rows + kRowsPerChunk - 1) / kRowsPerChunk;
  return g;
}

template <int V>
__device__ __forceinline__ Item next_item(const KernelArgs& a, const Item& it,
                                          uint32_t block_stride) {
  Item n;
  if (it.chunk + 1 < it.g.nchunks) {
    n.block = it.block;
    n.chunk = it.chunk + 1;
    n.g = it.g;
  } else {
    n.block = it.block + block_stride;
    n.chunk = 0;
    n.g = make_geo<V>(a, n.block);
  }
  return n;
}

// Issue the 16 row loads of one chunk plus, for lane 0 only, the first dword
// of the row after it (the high neighbour of lane 63 when re-aligning).
template <int V>
__device__ __forceinline__ void issue(uint32_t (&buf)[kRowsPerChunk + 1],
                                      const Item& it) {
  if (V & kProbeNoLoads) {
#pragma unroll
    for (int j = 0; j <= kRowsPerChunk; ++j)
      buf[j] = (lane_id() * 0x9E3779B1u) ^ (j * 0x85EBCA6Bu) ^ it.block;
    return;
  }
  const int32_t row0 =
      it.g.vb0 + kRowBytes * kRowsPerChunk * static_cast<int32_t>(it.chunk);
  const uint32_t lane = lane_id();
  const int32_t vo = row0 + 4 * static_cast<int32_t>(lane);
  const __amdgpu_buffer_rsrc_t rsrc = it.g.rsrc();
  if (row0 >= 0) {
    // Every offset is non-negative: let the compiler fold 256*j into the
    // instruction offset.
#pragma unroll
    for (int j = 0; j < kRowsPerChunk; ++j)
      buf[j] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, vo + 256 * j,
                                                    0, kDataCachePolicy);
  } else {
    // Some lanes start before the block: keep each offset whole so that the
    // bounds check sees the negative (= huge) value.
#pragma unroll
    for (int j = 0; j < kRowsPerChunk; ++j) {
      int32_t o = vo + 256 * j;
      asm volatile("" : "+v"(o));
      buf[j] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, o, 0, kDataCachePolicy);
    }
  }
  int32_t o16 = row0 + 256 * kRowsPerChunk;
  o16 = (lane == 0 && o16 >= 0) ? o16 : static_cast<int32_t>(kOobOffset);
  asm volatile("" : "+v"(o16));
  buf[kRowsPerChunk] =
      __builtin_amdgcn_raw_buffer_load_b32(rsrc, o16, 0, kDataCachePolicy);
}

// Prepare a loaded chunk in place, before any table work (so it overlaps the
// other stream's lookups):
//  * blocks whose end is not 4-byte aligned: re-align every row to the grid
//    (high neighbour of lane s = lane s+1's dword; lane 63 takes lane 0's
//    dword of the next row, the extra slot for the last row);
//  * chunk 0: zero the words before the block, clear the padding bytes of the
//    first data word and xor the init state s0 into the first 4 data bytes;
//    the high part of s0 spills into the next word (row 1, lane 0 when the
//    first data word is lane 63's).
template <int V>
__device__ __forceinline__ void prep_chunk(uint32_t (&buf)[kRowsPerChunk + 1],
                                           const Item& it) {
  const uint32_t lane = lane_id();
  if (!(V & kUniformAligned) && it.g.e != 0) {
    const int nb_addr = static_cast<int>(((lane + 1u) & 63u) * 4u);
#pragma unroll
    for (int j = 0; j < kRowsPerChunk; ++j) {
      const uint32_t src = (lane == 0) ? buf[j + 1] : buf[j];
      const uint32_t hi = static_cast<uint32_t>(
          __builtin_amdgcn_ds_bpermute(nb_addr, static_cast<int>(src)));
      buf[j] = __builtin_amdgcn_alignbyte(hi, buf[j], it.g.e);
    }
  }
  if (it.chunk == 0) {
    const Geo& g = it.g;
    const uint32_t sh = 8u * g.delta;
    uint32_t w = buf[0];
    w = (lane < g.s0l) ? 0u : w;
    w = (lane == g.s0l) ? ((w & (0xffffffffu << sh)) ^ (g.s0 << sh)) : w;
    w = (lane == g.s0l + 1u) ? (w ^ g.spill) : w;
    buf[0] = w;
    if (g.s0l == 63u) buf[1] = (lane == 0) ? (buf[1] ^ g.spill) : buf[1];
  }
}

__device__ __forceinline__ uint32_t tiny_crc(const Geo& g) {
  uint32_t reg = g.s0;
  if (g.len > 0) {
    const uint32_t bytes = sload_le(g.ptr(), g.len);
    for (uint32_t i = 0; i < g.len; ++i) {
      reg ^= (bytes >> (8u * i)) & 0xffu;
#pragma unroll
      for (int k = 0; k < 8; ++k)
        reg = (reg >> 1) ^ (kCastagnoliReflected & (0u - (reg & 1u)));
    }
  }
  return reg ^ 0xffffffffu;
}

template <int V>
__device__ __forceinline__ void store_result(const KernelArgs& a,
                                             const Item& it, uint32_t crc) {
  if (!(V & kUniformAligned) && it.g.tiny == 2) return;
  if (lane_id() == 0) {
    if ((V & kUniformAligned) || a.mode == kModeCompute) {
      a.out_crc[it.block] = a.mask ? crc_mask(crc) : crc;
    } else if (a.mode == kModeSstFill || a.mode == kModeLogFill) {
      // The stored form (Mask, little-endian) into the trailer / header hole:
      // trailer bytes 1..4 follow the covered n+1 bytes; the header CRC sits
      // 6 bytes before the covered type byte.
      const uint64_t ptr = (static_cast<uint64_t>(it.g.ptr_hi) << 32) | it.g.ptr_lo;
      uint8_t* dst = reinterpret_cast<uint8_t*>(a.mode == kModeSstFill ? ptr + it.g.len : ptr - 6);
      const uint32_t m = crc_mask(crc);
#pragma unroll
      for (int k = 0; k < 4; ++k) dst[k] = static_cast<uint8_t>(m >> (8 * k));
      if (a.out_crc != nullptr) a.out_crc[it.block] = crc;
    } else {
      a.out_crc[it.block] = crc;
      if (a.out_status != nullptr) a.out_status[it.block] = (crc != it.g.expected) ? 1 : 0;
    }
  }
}

template <int V>
__device__ __forceinline__ uint32_t finish_value(const uint32_t* lds,
                                                 uint32_t s,
                                                 uint32_t lane_base) {
  if (V & kProbeNoCompute) return wave_xor_dpp(s);
  if (V & kProbeShflReduce)
    return wave_xor_shfl(lane_end_shift(lds, s, lane_base)) ^ 0xffffffffu;
  return wave_xor_dpp(lane_end_shift(lds, s, lane_base)) ^ 0xffffffffu;
}

// One round: the current chunk of stream A and of stream B, two independent
// Horner chains interleaved row by row (latency of one chain hides behind the
// other's LDS lookups). A stream whose block is past the batch is idle.
template <int V>
__device__ __forceinline__ void consume2(
    const KernelArgs& a, const uint32_t* lds,
    uint32_t (&ba)[kRowsPerChunk + 1], const Item& ia, uint32_t& sa,
    uint32_t (&bb)[kRowsPerChunk + 1], const Item& ib, uint32_t& sb,
    uint32_t k0, uint32_t k1, uint32_t lane_base) {
  const bool live_a = ia.block < a.nblocks;
  const bool live_b = ib.block < a.nblocks;
  const bool rows_a = live_a && ((V & kUniformAligned) || !ia.g.tiny);
  const bool rows_b = live_b && ((V & kUniformAligned) || !ib.g.tiny);
  if (V & kProbeNoCompute) {
#pragma unroll
    for (int j = 0; j < kRowsPerChunk; ++j) {
      sa ^= ba[j];
      sb ^= bb[j];
    }
  } else {
    if (rows_a) prep_chunk<V>(ba, ia);
    if (rows_b) prep_chunk<V>(bb, ib);
    const uint32_t na =
        rows_a ? min(static_cast<uint32_t>(kRowsPerChunk),
                     ia.g.rows - kRowsPerChunk * ia.chunk)
               : 0u;
    const uint32_t nb =
        rows_b ? min(static_cast<uint32_t>(kRowsPerChunk),
                     ib.g.rows - kRowsPerChunk * ib.chunk)
               : 0u;
    // Row 0 of the chunk: starts the chain (chunk 0) or continues it.
    if (na != 0) sa = (ia.chunk == 0) ? ba[0] : row_step(lds, sa, ba[0], k0, k1);
    if (nb != 0) sb = (ib.chunk == 0) ? bb[0] : row_step(lds, sb, bb[0], k0, k1);
    if (na == kRowsPerChunk && nb == kRowsPerChunk) {
      // Straight-line body: both chains in one basic block.
#pragma unroll
      for (int j = 1; j < kRowsPerChunk; ++j) {
        sa = row_step(lds, sa, ba[j], k0, k1);
        sb = row_step(lds, sb, bb[j], k0, k1);
      }
    } else {
      // Ragged chunks: both chains up to the shorter one, then the rest of
      // each (three simple loops unroll fully; one three-way loop does not).
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
  const bool fin_a = live_a && ia.chunk + 1 == ia.g.nchunks;
  const bool fin_b = live_b && ib.chunk + 1 == ib.g.nchunks;
  if (fin_a && fin_b && ((V & kUniformAligned) || (!ia.g.tiny && !ib.g.tiny))) {
    const uint32_t ca = finish_value<V>(lds, sa, lane_base);
    const uint32_t cb = finish_value<V>(lds, sb, lane_base);
    store_result<V>(a, ia, ca);
    store_result<V>(a, ib, cb);
  } else {
    if (fin_a)
      store_result<V>(a, ia, (!(V & kUniformAligned) && ia.g.tiny)
                                 ? tiny_crc(ia.g) : finish_value<V>(lds, sa, lane_base));
    if (fin_b)
      store_result<V>(a, ib, (!(V & kUniformAligned) && ib.g.tiny)
                                 ? tiny_crc(ib.g) : finish_value<V>(lds, sb, lane_base));
  }
}

}  // namespace

// Persistent grid, one 1024-thread workgroup per CU (all 160 KiB of LDS).
// Wave gw runs two block streams: A = blocks gw, gw + 2W, ... and
// B = blocks gw + W, gw + 3W, ... (W = waves in the grid); each stream walks
// its blocks in 4 KiB chunks and keeps one chunk in flight while the current
// chunks of both streams are consumed.
template <int V>
__global__ void __launch_bounds__(kGroupThreads, 1)
    crc32c_batch_kernel(KernelArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsBytes / 4];

  if (a.count != nullptr) a.nblocks = min(a.nblocks, sload_u32(a.count, 0));
  if (V & kProbeEmpty) {
    if (a.nblocks == 0xffffffffu) lds[threadIdx.x] = 0;  // keep the LDS request
    return;
  }
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = lane_id();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t nwaves = gridDim.x * kWavesPerGroup;
  const uint32_t gw = blockIdx.x * kWavesPerGroup + wave;
  const uint32_t stream_stride = 2u * nwaves;
  stamp<V>(a, gw, 0);

  // 1. table values for this thread's share of the LDS image (L2 hits).
  constexpr int kRowIters = (kLdsRowRegionBytes * 2 / 16) / kGroupThreads;  // 8
  constexpr int kLaneIters = (kLaneTabDwords / 4) / kGroupThreads;          // 2
  uint32_t rv[kRowIters];
  uint32_t lv[kLaneIters][4];
#pragma unroll
  for (int k = 0; k < kRowIters; ++k) {
    if (V & kProbeNoFill) break;
    const uint32_t dw = (tid + kGroupThreads * k) * 4u;
    const uint32_t t = ((dw >> 14) << 1) | ((dw >> 5) & 1u);
    const uint32_t i = (dw >> 6) & 255u;
    rv[k] = a.row_tab[t * 256u + i];
  }
#pragma unroll
  for (int k = 0; k < kLaneIters; ++k) {
    if (V & kProbeNoFill) break;
    const uint32_t* src = a.lane_tab + 4u * (tid + kGroupThreads * k);
#pragma unroll
    for (int x = 0; x < 4; ++x) lv[k][x] = src[x];
  }
  // Every wave's table loads enter the CU's memory queue before any block
  // load of the workgroup; otherwise they queue behind the batch's block
  // stream and the fill (on every wave's critical path) waits ~5 us.
  __builtin_amdgcn_sched_barrier(0);
  if (!(V & kProbeNoFill)) __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);

  // 2. both streams' first chunk in flight before the LDS fill. Only one
  //    round: the table loads + 34 block loads stay under the 63 loads the
  //    vmcnt counter can track, so the fill waits for its table values only
  //    (with both rounds in flight the wait before the first ds_write would
  //    cover most of the block data).
  uint32_t a0[kRowsPerChunk + 1], a1[kRowsPerChunk + 1];
  uint32_t b0[kRowsPerChunk + 1], b1[kRowsPerChunk + 1];
  Item ia0, ib0;
  ia0.block = gw;
  ia0.chunk = 0;
  ia0.g = make_geo<V>(a, ia0.block);
  ib0.block = gw + nwaves;
  ib0.chunk = 0;
  ib0.g = make_geo<V>(a, ib0.block);
  if (!(V & kProbeLateLoads)) {
    issue<V>(a0, ia0);
    issue<V>(b0, ib0);
  }
  __builtin_amdgcn_sched_barrier(0);

  // 3. LDS fill: row tables replicated 4 copies per ds_write_b128.
  if (!(V & kProbeNoFill)) {
#pragma unroll
    for (int k = 0; k < kRowIters; ++k)
      reinterpret_cast<uint4*>(lds)[tid + kGroupThreads * k] =
          make_uint4(rv[k], rv[k], rv[k], rv[k]);
#pragma unroll
    for (int k = 0; k < kLaneIters; ++k)
      reinterpret_cast<uint4*>(lds + kLdsLaneTabBase / 4)[tid + kGroupThreads * k] =
          make_uint4(lv[k][0], lv[k][1], lv[k][2], lv[k][3]);
  }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  stamp<V>(a, gw, 1);

  if (V & kProbeLateLoads) {
    issue<V>(a0, ia0);
    issue<V>(b0, ib0);
  }
  // 4. second round in flight.
  Item ia1 = next_item<V>(a, ia0, stream_stride);
  Item ib1 = next_item<V>(a, ib0, stream_stride);
  issue<V>(a1, ia1);
  issue<V>(b1, ib1);

  const uint32_t k0 = (lane & 31u) * 4u;
  const uint32_t k1 = k0 | 0x10000u;
  const uint32_t lane_base = kLdsLaneTabBase + lane * 4u;

  uint32_t sa = 0, sb = 0;
  int round = 0;
  while (true) {
    if (ia0.block >= a.nblocks && ib0.block >= a.nblocks) break;
    consume2<V>(a, lds, a0, ia0, sa, b0, ib0, sb, k0, k1, lane_base);
    if (V & kProbeStamps) stamp<V>(a, gw, 2 + min(round++, 4));
    ia0 = next_item<V>(a, ia1, stream_stride);
    ib0 = next_item<V>(a, ib1, stream_stride);
    issue<V>(a0, ia0);
    issue<V>(b0, ib0);
    if (ia1.block >= a.nblocks && ib1.block >= a.nblocks) break;
    consume2<V>(a, lds, a1, ia1, sa, b1, ib1, sb, k0, k1, lane_base);
    if (V & kProbeStamps) stamp<V>(a, gw, 2 + min(round++, 4));
    ia1 = next_item<V>(a, ia0, stream_stride);
    ib1 = next_item<V>(a, ib0, stream_stride);
    issue<V>(a1, ia1);
    issue<V>(b1, ib1);
  }
  stamp<V>(a, gw, 7);
}

#ifdef LVKV_PROBE_BUILD
// Read-bandwidth ceiling: every byte read once with 16 B per lane, grid
// stride; nothing is stored unless the xor of the data hits a magic value, so
// the loads cannot be dropped. Used to state the measured HBM ceiling next to
// the 8 TB/s spec.
// 4 B per lane variant of the same (the batch kernel's load width).
__global__ void __launch_bounds__(256)
    read_bw_dword_kernel(const uint32_t* __restrict__ p, uint64_t n4,
                         uint32_t* out) {
  const uint64_t nth = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  uint32_t acc = 0;
  for (; i + 7 * nth < n4; i += 8 * nth) {
#pragma unroll
    for (int k = 0; k < 8; ++k) acc ^= p[i + k * nth];
  }
  for (; i < n4; i += nth) acc ^= p[i];
  if (acc == 0x9E3779B9u) out[0] = acc;
}

__global__ void __launch_bounds__(256)
    read_bw_kernel(const uint4* __restrict__ p, uint64_t n16, uint32_t* out) {
  const uint64_t nth = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (; i + 3 * nth < n16; i += 4 * nth) {
    const uint4 x0 = p[i], x1 = p[i + nth], x2 = p[i + 2 * nth], x3 = p[i + 3 * nth];
    acc.x ^= x0.x ^ x1.x ^ x2.x ^ x3.x;
    acc.y ^= x0.y ^ x1.y ^ x2.y ^ x3.y;
    acc.z ^= x0.z ^ x1.z ^ x2.z ^ x3.z;
    acc.w ^= x0.w ^ x1.w ^ x2.w ^ x3.w;
  }
  for (; i < n16; i += nth) {
    const uint4 x = p[i];
    acc.x ^= x.x; acc.y ^= x.y; acc.z ^= x.z; acc.w ^= x.w;
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9E3779B9u) out[0] = acc.x;
}

#endif  // LVKV_PROBE_BUILD

// Host-side launchers (compiled in this TU so the kernel symbols stay local).
hipError_t launch_crc32c_batch(const KernelArgs& args, bool uniform_aligned,
                               int num_groups, hipStream_t stream) {
  if (uniform_aligned) {
    hipLaunchKernelGGL(crc32c_batch_kernel<kUniformAligned>, dim3(num_groups),
                       dim3(kGroupThreads), 0, stream, args);
  } else {
    hipLaunchKernelGGL(crc32c_batch_kernel<kProbeNone>, dim3(num_groups),
                       dim3(kGroupThreads), 0, stream, args);
  }
  return hipGetLastError();
}

#ifdef LVKV_PROBE_BUILD
hipError_t launch_crc32c_probe(const KernelArgs& args, int variant,
                               int num_groups, hipStream_t stream) {
  switch (variant) {
#define LVKV_PROBE_CASE(v)                                                  \
  case v:                                                                   \
    hipLaunchKernelGGL(crc32c_batch_kernel<v>, dim3(num_groups),            \
                       dim3(kGroupThreads), 0, stream, args);               \
    break;
    LVKV_PROBE_CASE(0)
    LVKV_PROBE_CASE(1)
    LVKV_PROBE_CASE(2)
    LVKV_PROBE_CASE(3)
    LVKV_PROBE_CASE(4)
    LVKV_PROBE_CASE(5)
    LVKV_PROBE_CASE(6)
    LVKV_PROBE_CASE(8)
    LVKV_PROBE_CASE(16)
    LVKV_PROBE_CASE(32)
    LVKV_PROBE_CASE(33)
    LVKV_PROBE_CASE(34)
    LVKV_PROBE_CASE(38)
    LVKV_PROBE_CASE(96)
    LVKV_PROBE_CASE(97)
    LVKV_PROBE_CASE(160)
    LVKV_PROBE_CASE(224)
#undef LVKV_PROBE_CASE
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_read_bw(const void* p, uint64_t bytes, uint32_t* out,
                          int num_groups, hipStream_t stream) {
  if (num_groups < 0) {  // negative: the dword-per-lane variant
    hipLaunchKernelGGL(read_bw_dword_kernel, dim3(-num_groups), dim3(256), 0,
                       stream, static_cast<const uint32_t*>(p), bytes / 4, out);
  } else {
    hipLaunchKernelGGL(read_bw_kernel, dim3(num_groups), dim3(256), 0, stream,
                       static_cast<const uint4*>(p), bytes / 16, out);
  }
  return hipGetLastError();
}

#endif  // LVKV_PROBE_BUILD

}  // namespace lvkv
