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

#include "lvkv_kernel_args.h"

namespace lvkv {
namespace {

typedef __attribute__((address_space(4))) const uint32_t ConstU32;

constexpr uint32_t kBufferDword3 = 0x00020000u;  // gfx9 raw buffer config
constexpr uint32_t kOobOffset = 0x80000000u;     // >= any num_records

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

typedef __attribute__((address_space(4))) const uint64_t ConstU64;

// Wave-uniform dword load through the scalar cache. `addr` must be 4-aligned.
__device__ __forceinline__ uint32_t sload32(uint64_t addr) {
  return *reinterpret_cast<ConstU32*>(addr);
}
// Wave-uniform element loads of the descriptor arrays (s_load, lgkmcnt).
__device__ __forceinline__ uint32_t sload_u32(const uint32_t* p, uint32_t i) {
  return reinterpret_cast<ConstU32*>(reinterpret_cast<uint64_t>(p))[i];
}
__device__ __forceinline__ uint64_t sload_u64(const uint64_t* p, uint32_t i) {
  return reinterpret_cast<ConstU64*>(reinterpret_cast<uint64_t>(p))[i];
}

// Wave-uniform little-endian load of n (1..4) bytes at any address, touching
// only the dwords that contain [addr, addr + n).
__device__ __forceinline__ uint32_t sload_le(uint64_t addr, uint32_t n) {
  const uint64_t a0 = addr & ~uint64_t{3};
  const uint64_t a1 = (addr + n - 1) & ~uint64_t{3};
  const uint32_t lo = sload32(a0);
  const uint32_t hi = (a1 != a0) ? sload32(a1) : 0u;
  const uint32_t sh = static_cast<uint32_t>(addr & 3u) * 8u;
  const uint64_t v = (static_cast<uint64_t>(hi) << 32) | lo;
  uint32_t r = static_cast<uint32_t>(v >> sh);
  if (n < 4) r &= (1u << (8u * n)) - 1u;
  return r;
}

__device__ __forceinline__ uint32_t crc_mask(uint32_t c) {
  return ((c >> 15) | (c << 17)) + kMaskDelta;
}
__device__ __forceinline__ uint32_t crc_unmask(uint32_t m) {
  const uint32_t r = m - kMaskDelta;
  return (r >> 17) | (r << 15);
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
  uint32_t tiny;      // 1: length < 4, computed bitwise
  uint32_t len;
  uint32_t ptr_lo;    // absolute address of the first covered byte
  uint32_t ptr_hi;    //   (split: keeps the struct free of padding)
  uint32_t expected;  // verify modes: unmasked stored CRC
  __device__ __forceinline__ uint64_t ptr() const {
    return (static_cast<uint64_t>(ptr_hi) << 32) | ptr_lo;
  }
  __device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc() const {
    const uint64_t b = (static_cast<uint64_t>(b4_hi) << 32) | b4_lo;
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(b), 0,
                                             static_cast<int>(nrec),
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

__device__ __forceinline__ Geo make_geo(const KernelArgs& a, uint32_t b) {
  if (b >= a.nblocks) return null_geo();
  const uint64_t base = reinterpret_cast<uint64_t>(a.base);
  uint64_t off;
  uint32_t len, init = a.init, expected = 0;
  if (a.mode == kModeLogVerify) {
    // Header [masked crc u32][len u16][type u8]; CRC covers type + payload
    // (db/log_reader.cc:217-221, 243-247).
    const uint64_t hoff = sload_u64(a.offsets, b);
    const uint64_t hdr = base + hoff;
    const uint32_t len_type = sload_le(hdr + 4, 3);
    expected = crc_unmask(sload_le(hdr, 4));
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
  if (a.mode == kModeSstVerify) {
    // Block contents n bytes + type byte are covered; the masked CRC follows
    // (table/format.cc:92-94, table/table_builder.cc:199-203).
    len += 1;
    init = 0;
    expected = crc_unmask(sload_le(base + off + len, 4));
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

__device__ __forceinline__ Item next_item(const KernelArgs& a, const Item& it,
                                          uint32_t nwaves) {
  Item n;
  if (it.chunk + 1 < it.g.nchunks) {
    n.block = it.block;
    n.chunk = it.chunk + 1;
    n.g = it.g;
  } else {
    n.block = it.block + nwaves;
    n.chunk = 0;
    n.g = make_geo(a, n.block);
  }
  return n;
}

// Issue the 16 row loads of one chunk plus, for lane 0 only, the first dword
// of the row after it (the high neighbour of lane 63 when re-aligning).
__device__ __forceinline__ void issue(uint32_t (&buf)[kRowsPerChunk + 1],
                                      const Item& it) {
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
                                                    0, 0);
  } else {
    // Some lanes start before the block: keep each offset whole so that the
    // bounds check sees the negative (= huge) value.
#pragma unroll
    for (int j = 0; j < kRowsPerChunk; ++j) {
      int32_t o = vo + 256 * j;
      asm volatile("" : "+v"(o));
      buf[j] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, o, 0, 0);
    }
  }
  int32_t o16 = row0 + 256 * kRowsPerChunk;
  o16 = (lane == 0 && o16 >= 0) ? o16 : static_cast<int32_t>(kOobOffset);
  asm volatile("" : "+v"(o16));
  buf[kRowsPerChunk] =
      __builtin_amdgcn_raw_buffer_load_b32(rsrc, o16, 0, 0);
}

__device__ __forceinline__ uint32_t lds_ld(const uint32_t* lds,
                                           uint32_t byte_addr) {
  return *reinterpret_cast<const uint32_t*>(
      reinterpret_cast<const char*>(lds) + byte_addr);
}

// S -> Z_256(S): one bank-private LDS lookup per byte of S.
// k0 = (lane & 31) * 4, k1 = k0 | 0x10000. v_perm_b32 builds
// {k.byte0, S.byte_t, k.byte2, 0} = S.byte_t * 256 + copy*4 + region.
__device__ __forceinline__ uint32_t row_advance(const uint32_t* lds,
                                                uint32_t s, uint32_t k0,
                                                uint32_t k1) {
  const uint32_t a0 = __builtin_amdgcn_perm(s, k0, 0x0C020400u);
  const uint32_t a1 = __builtin_amdgcn_perm(s, k0, 0x0C020500u);
  const uint32_t a2 = __builtin_amdgcn_perm(s, k1, 0x0C020600u);
  const uint32_t a3 = __builtin_amdgcn_perm(s, k1, 0x0C020700u);
  return lds_ld(lds, a0) ^ lds_ld(lds, a1 + 128u) ^ lds_ld(lds, a2) ^
         lds_ld(lds, a3 + 128u);
}

// S -> Z_{256-4s}(S) for this lane s: eight lane-private nibble lookups.
__device__ __forceinline__ uint32_t lane_end_shift(const uint32_t* lds,
                                                   uint32_t s,
                                                   uint32_t lane_base) {
  uint32_t r = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint32_t nib = (s >> (4 * k)) & 15u;
    r ^= lds_ld(lds, (lane_base | (nib << 8)) + 4096u * k);
  }
  return r;
}

__device__ __forceinline__ uint32_t wave_xor(uint32_t v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v ^= __shfl_xor(v, m, 64);
  return v;
}

// Word j of a chunk, re-aligned to the grid when the block end is not
// 4-byte aligned (the high neighbour of lane s is lane s+1's dword; lane 63
// takes lane 0's dword of the next row).
template <bool kMisaligned>
__device__ __forceinline__ uint32_t grid_word(
    const uint32_t (&buf)[kRowsPerChunk + 1], int j, uint32_t lane,
    uint32_t nb_addr, uint32_t e) {
  if (!kMisaligned) return buf[j];
  const uint32_t src = (lane == 0) ? buf[j + 1] : buf[j];
  const uint32_t hi = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(
      static_cast<int>(nb_addr), static_cast<int>(src)));
  return __builtin_amdgcn_alignbyte(hi, buf[j], e);
}

// Row 0 of a block: zero the words before the block, clear the padding bytes
// of the first data word and xor in the init state (s0) at the first data
// byte; the high part of s0 spills into the next word.
__device__ __forceinline__ uint32_t fix_row0(uint32_t w, const Geo& g,
                                            uint32_t lane) {
  const uint32_t sh = 8u * g.delta;
  w = (lane < g.s0l) ? 0u : w;
  w = (lane == g.s0l) ? ((w & (0xffffffffu << sh)) ^ (g.s0 << sh)) : w;
  w = (lane == g.s0l + 1u) ? (w ^ g.spill) : w;
  return w;
}

template <bool kMisaligned>
__device__ __forceinline__ uint32_t consume_rows(
    const uint32_t* lds, const uint32_t (&buf)[kRowsPerChunk + 1],
    const Item& it, uint32_t s, uint32_t k0, uint32_t k1) {
  const uint32_t lane = lane_id();
  const uint32_t nb_addr = ((lane + 1u) & 63u) * 4u;
  const uint32_t e = it.g.e;
  const uint32_t left = it.g.rows - kRowsPerChunk * it.chunk;  // >= 1
  uint32_t w = grid_word<kMisaligned>(buf, 0, lane, nb_addr, e);
  if (it.chunk == 0) {
    s = fix_row0(w, it.g, lane);
  } else {
    s = row_advance(lds, s, k0, k1) ^ w;
  }
  if (left > 1) {
    w = grid_word<kMisaligned>(buf, 1, lane, nb_addr, e);
    if (it.chunk == 0 && it.g.s0l == 63u) w = (lane == 0) ? (w ^ it.g.spill) : w;
    s = row_advance(lds, s, k0, k1) ^ w;
  }
#pragma unroll
  for (int j = 2; j < kRowsPerChunk; ++j) {
    if (static_cast<uint32_t>(j) < left) {  // wave-uniform
      w = grid_word<kMisaligned>(buf, j, lane, nb_addr, e);
      s = row_advance(lds, s, k0, k1) ^ w;
    }
  }
  return s;
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

__device__ __forceinline__ void finish_block(const KernelArgs& a,
                                             const uint32_t* lds,
                                             const Item& it, uint32_t s,
                                             uint32_t lane_base) {
  uint32_t crc;
  if (it.g.tiny) {
    crc = tiny_crc(it.g);
  } else {
    crc = wave_xor(lane_end_shift(lds, s, lane_base)) ^ 0xffffffffu;
  }
  if (lane_id() == 0) {
    if (a.mode == kModeCompute) {
      a.out_crc[it.block] = a.mask ? crc_mask(crc) : crc;
    } else {
      a.out_crc[it.block] = crc;
      a.out_status[it.block] = (crc != it.g.expected) ? 1 : 0;
    }
  }
}

__device__ __forceinline__ uint32_t consume(const KernelArgs& a,
                                           const uint32_t* lds,
                                           const uint32_t (&buf)[kRowsPerChunk + 1],
                                           const Item& it, uint32_t s,
                                           uint32_t k0, uint32_t k1,
                                           uint32_t lane_base) {
  if (!it.g.tiny) {
    if (it.g.e == 0)
      s = consume_rows<false>(lds, buf, it, s, k0, k1);
    else
      s = consume_rows<true>(lds, buf, it, s, k0, k1);
  }
  if (it.chunk + 1 == it.g.nchunks) finish_block(a, lds, it, s, lane_base);
  return s;
}

}  // namespace

__global__ void __launch_bounds__(kGroupThreads, 1)
    crc32c_batch_kernel(KernelArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsBytes / 4];

  const uint32_t tid = threadIdx.x;
  const uint32_t lane = lane_id();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t nwaves = gridDim.x * kWavesPerGroup;
  const uint32_t gw = blockIdx.x * kWavesPerGroup + wave;

  // 1. table values for this thread's share of the LDS image (L2 hits).
  constexpr int kRowIters = (kLdsRowRegionBytes * 2 / 16) / kGroupThreads;  // 8
  constexpr int kLaneIters = (kLaneTabDwords / 4) / kGroupThreads;          // 2
  uint32_t rv[kRowIters];
  uint32_t lv[kLaneIters][4];
#pragma unroll
  for (int k = 0; k < kRowIters; ++k) {
    const uint32_t dw = (tid + kGroupThreads * k) * 4u;
    const uint32_t t = ((dw >> 14) << 1) | ((dw >> 5) & 1u);
    const uint32_t i = (dw >> 6) & 255u;
    rv[k] = a.row_tab[t * 256u + i];
  }
#pragma unroll
  for (int k = 0; k < kLaneIters; ++k) {
    const uint32_t* src = a.lane_tab + 4u * (tid + kGroupThreads * k);
#pragma unroll
    for (int x = 0; x < 4; ++x) lv[k][x] = src[x];
  }
  __builtin_amdgcn_sched_barrier(0);

  // 2. first two pipeline stages in flight before the LDS fill.
  uint32_t bufA[kRowsPerChunk + 1], bufB[kRowsPerChunk + 1];
  Item ia;
  ia.block = gw;
  ia.chunk = 0;
  ia.g = make_geo(a, gw);
  issue(bufA, ia);
  Item ib = next_item(a, ia, nwaves);
  issue(bufB, ib);
  __builtin_amdgcn_sched_barrier(0);

  // 3. LDS fill: row tables replicated 4 copies per ds_write_b128.
#pragma unroll
  for (int k = 0; k < kRowIters; ++k)
    reinterpret_cast<uint4*>(lds)[tid + kGroupThreads * k] =
        make_uint4(rv[k], rv[k], rv[k], rv[k]);
#pragma unroll
  for (int k = 0; k < kLaneIters; ++k)
    reinterpret_cast<uint4*>(lds + kLdsLaneTabBase / 4)[tid + kGroupThreads * k] =
        make_uint4(lv[k][0], lv[k][1], lv[k][2], lv[k][3]);
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");

  const uint32_t k0 = (lane & 31u) * 4u;
  const uint32_t k1 = k0 | 0x10000u;
  const uint32_t lane_base = kLdsLaneTabBase + lane * 4u;

  uint32_t s = 0;
  while (true) {
    if (ia.block >= a.nblocks) break;
    s = consume(a, lds, bufA, ia, s, k0, k1, lane_base);
    ia = next_item(a, ib, nwaves);
    issue(bufA, ia);
    if (ib.block >= a.nblocks) break;
    s = consume(a, lds, bufB, ib, s, k0, k1, lane_base);
    ib = next_item(a, ia, nwaves);
    issue(bufB, ib);
  }
}

// Host-side launcher (compiled in this TU so the kernel symbol stays local).
hipError_t launch_crc32c_batch(const KernelArgs& args, int num_groups,
                               hipStream_t stream) {
  hipLaunchKernelGGL(crc32c_batch_kernel, dim3(num_groups),
                     dim3(kGroupThreads), 0, stream, args);
  return hipGetLastError();
}

}  // namespace lvkv
