// Snappy block codec on the device: the codec
// LevelDB calls around the block CRC when a table is written or read with
// kSnappyCompression -- port::Snappy_Compress / Snappy_GetUncompressedLength /
// Snappy_Uncompress (port/port_stdcxx.h:90-133) behind TableBuilder::
// WriteBlock (table/table_builder.cc:151-168) and ReadBlock
// (table/format.cc:120-136). The as-built reference has HAVE_SNAPPY=0; the
// codec is google/snappy, restated from the published algorithm of the
// version in this image (snappy 1.1.8, /opt/conda/lib): the compressor emits
// the same bytes as snappy::RawCompress 1.1.8, the decompressor accepts and
// rejects exactly what snappy::RawUncompress does (oracle/snappy_oracle.py,
// tests/test_snappy.py).
//
// One wave per block (a 64-thread workgroup), its bytes staged in LDS
// (dynamic, sized from the caller's largest block): the codec is a serial
// chain per block (each element's place depends on the one before), so the
// wave runs it with wave-uniform control flow, and its 64 lanes copy
// literals, extend matches 64 bytes at a time (a ballot finds the first
// difference) and write the result out. Blocks are independent: the grid is
// one workgroup per block.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lvkv_snappy.h"

namespace lvkv {
namespace {

constexpr uint32_t kFrag = 1u << 16;       // kBlockSize: fragments compressed alone
constexpr uint32_t kMaxTable = 1u << 14;   // kMaxHashTableSize
constexpr uint32_t kMul = 0x1e35a7bdu;

// Offsets of the literal search's probes after a reset (skip = 32, step =
// skip >> 5, skip += step), clamped at 0xffff: any later probe lies past
// every ip_limit. 267 offsets reach past 64 KiB; the table holds 5 windows.
constexpr uint32_t kProbes = 5 * 64 + 1;
struct ProbeOffsets {
  uint16_t v[kProbes + 7];
  constexpr ProbeOffsets() : v() {
    uint32_t off = 0, skip = 32;
    for (uint32_t i = 0; i < kProbes + 7; ++i) {
      v[i] = static_cast<uint16_t>(off < 0xffffu ? off : 0xffffu);
      if (off < 0xffffu) {
        off += skip >> 5;
        skip += skip >> 5;
      }
    }
  }
};
__constant__ ProbeOffsets kProbe;

__device__ __forceinline__ uint32_t table_size(uint32_t n) {
  uint32_t t = 256;
  while (t < kMaxTable && t < n) t <<= 1;
  return t;
}

// Little-endian dword at byte p of an LDS buffer (4-byte aligned base, padded
// by 8 bytes): two aligned reads.
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

// Block b's bytes [0, n) from global memory into LDS (4-aligned), zero
// padding after them. Aligned dword loads at any source alignment: LDS
// dword i = alignbyte of source dwords i and i+1 (the second only where it
// holds bytes of the block, so nothing past the block's last dword is read).
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
  for (uint32_t i = n + lane; i < n + pad; i += 64) dst[i] = 0;  // (pad >= 3)
}

// ---- compression (snappy::RawCompress 1.1.8) ------------------------------

struct Out {
  uint8_t* p;  // the block's output
  uint32_t n;  // bytes written
};

// A literal: tag (+ 1-4 length bytes) by lane 0, the bytes by every lane.
__device__ __forceinline__ void emit_literal(Out& o, const uint8_t* in, uint32_t from,
                                             uint32_t len, uint32_t lane) {
  const uint32_t n = len - 1;
  uint32_t h;
  if (n < 60) {
    if (lane == 0) o.p[o.n] = static_cast<uint8_t>(n << 2);
    h = 1;
  } else {
    const uint32_t count = ((31u - __builtin_clz(n)) >> 3) + 1u;
    if (lane == 0) {
      o.p[o.n] = static_cast<uint8_t>((59u + count) << 2);
      for (uint32_t k = 0; k < count; ++k) o.p[o.n + 1 + k] = static_cast<uint8_t>(n >> (8 * k));
    }
    h = 1 + count;
  }
  for (uint32_t k = lane; k < len; k += 64) o.p[o.n + h + k] = in[from + k];
  o.n += h + len;
}

__device__ __forceinline__ void emit_copy_at_most_64(Out& o, uint32_t off, uint32_t len, bool lt12,
                                                     uint32_t lane) {
  if (lt12 && off < 2048) {
    if (lane == 0) {
      o.p[o.n] = static_cast<uint8_t>(1u + ((len - 4u) << 2) + ((off >> 3) & 0xe0u));
      o.p[o.n + 1] = static_cast<uint8_t>(off);
    }
    o.n += 2;
  } else {
    const uint32_t u = 2u + ((len - 1u) << 2) + (off << 8);
    if (lane == 0) {
      o.p[o.n] = static_cast<uint8_t>(u);
      o.p[o.n + 1] = static_cast<uint8_t>(u >> 8);
      o.p[o.n + 2] = static_cast<uint8_t>(u >> 16);
    }
    o.n += 3;
  }
}

__device__ __forceinline__ void emit_copy(Out& o, uint32_t off, uint32_t len, uint32_t lane) {
  if (len < 12) {
    emit_copy_at_most_64(o, off, len, true, lane);
    return;
  }
  while (len >= 68) {
    emit_copy_at_most_64(o, off, 64, false, lane);
    len -= 64;
  }
  if (len > 64) {
    emit_copy_at_most_64(o, off, 60, false, lane);
    len -= 60;
  }
  emit_copy_at_most_64(o, off, len, len < 12, lane);
}

// Bytes matching from a + 4 and b + 4 (b > a), b + 4 + result <= n: the
// wave compares 64 bytes a step and the ballot of differences stops it.
__device__ __forceinline__ uint32_t match_length(const uint8_t* in, uint32_t a, uint32_t b,
                                                 uint32_t n, uint32_t lane) {
  uint32_t m = 4;
  for (;;) {
    const uint32_t pb = b + m + lane;
    const bool diff = pb >= n || in[a + m + lane] != in[pb];
    const uint64_t bal = __ballot(diff);
    if (bal != 0) return m + static_cast<uint32_t>(__builtin_ctzll(bal));
    m += 64;
  }
}

__device__ __forceinline__ uint32_t hash32(uint32_t v, uint32_t shift) {
  return (v * kMul) >> shift;
}

// The literal search of CompressFragment (the loop that hashes ip, swaps it
// into the table and compares 4 bytes with the old entry, stepping by
// skip >> 5 with skip += step), 64 probes a step, one a lane. The probe
// positions after a reset do not depend on the data: probe k sits at
// base + probe[k] (kProbe), and is made only if probe k+1 is <= ip_limit.
// Probe k's candidate is the table entry as probes 0..k-1 left it: the
// entry before the step (c0), or the latest earlier lane with the same hash,
// whose 4 bytes are that lane's own v. A 256-slot LDS scratch keeps the
// lowest lane per (hash & 255) (an atomic min): a lane that is lowest in its
// slot is the first of its hash, so its c0 test is exact, and the first
// such match bounds the answer. Only the lanes below it with a lower lane in
// their slot (~4 of 64 on db_bench's data) are resolved one by one. The
// table is written once, after: each hash's last probe at or before the
// match. Returns false at emit_remainder.
__device__ __forceinline__ bool search_probes(const uint8_t* in, uint16_t* table,
                                              uint32_t* slots,
                                              uint32_t base, uint32_t ip_limit, uint32_t shift,
                                              uint32_t lane, uint32_t w0, uint32_t w1,
                                              uint32_t* out_ip, uint32_t* out_cand) {
  for (uint32_t n0 = 0;; n0 += 64) {
    // (the first step's offsets come in registers: most searches end there)
    const uint32_t p = base + (n0 == 0 ? w0 : kProbe.v[n0 + lane]);
    const bool valid = base + (n0 == 0 ? w1 : kProbe.v[n0 + lane + 1]) <= ip_limit;
    const uint64_t vmask = __ballot(valid);
    const uint32_t v = ld32(in, valid ? p : 0u);
    const uint32_t h = hash32(v, shift);
    const uint32_t c0 = valid ? table[h] : 0u;
    uint32_t* slot = slots + (h & 255u);
    *slot = 0xffffffffu;
    if (valid) atomicMin(slot, lane);
    const uint32_t first = *slot;
    const uint32_t vc = ld32(in, valid ? c0 : 0u);
    const uint64_t m0 = __ballot(valid && vc == v);
    const uint64_t dupe = __ballot(valid && first < lane);
    const uint32_t ki = ~vmask ? __builtin_ctzll(~vmask) : 64u;
    const uint64_t sure = m0 & ~dupe;
    uint32_t km = sure ? __builtin_ctzll(sure) : 64u;
    uint32_t kcand = km < 64 ? __builtin_amdgcn_readlane(c0, km) : 0u;
    uint32_t nxt = 64;  // the next lane of this lane's hash, once resolved
    for (uint64_t dl = dupe; dl;) {
      const uint32_t d = __builtin_ctzll(dl);
      if (d >= km) break;
      dl &= dl - 1u;
      const uint32_t hd = __builtin_amdgcn_readlane(h, d);
      const uint64_t g = __ballot(valid && h == hd) & ((uint64_t{1} << d) - 1u);
      if (g == 0) {  // a slot shared by another hash: d is its hash's first
        if ((m0 >> d) & 1u) {
          km = d;
          kcand = __builtin_amdgcn_readlane(c0, d);
        }
        continue;
      }
      const uint32_t prev = 63u - __builtin_clzll(g);
      nxt = lane == prev ? d : nxt;
      if (__builtin_amdgcn_readlane(v, prev) == __builtin_amdgcn_readlane(v, d)) {
        km = d;
        kcand = __builtin_amdgcn_readlane(p, prev);
      }
    }
    if (ki < km) return false;  // the search runs past ip_limit first
    const uint32_t K = km < 64 ? km : 63u;  // the last probe made
    if (valid && lane <= K && nxt > K) table[h] = static_cast<uint16_t>(p);
    if (km < 64) {
      *out_ip = __builtin_amdgcn_readlane(p, km);
      *out_cand = kcand;
      return true;
    }
  }
}

// CompressFragment of frag = in[0, n) (n <= kFrag) with table (u16 x tsize in
// LDS, zeroed here). Control flow is wave-uniform.
__device__ void compress_fragment(const uint8_t* in, uint32_t n, uint16_t* table,
                                  uint32_t* slots, Out& o, uint32_t lane) {
  const uint32_t tsize = table_size(n);
  const uint32_t shift = 32u - (31u - __builtin_clz(tsize));
  for (uint32_t i = lane; i < tsize; i += 64) table[i] = 0;
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the zeroes land first
  uint32_t ip = 0, next_emit = 0;
  if (n >= 15) {
    const uint32_t ip_limit = n - 15;
    ip = 1;
    for (;;) {
      uint32_t cand = 0;
      bool remainder = false;
      if (!search_probes(in, table, slots, ip, ip_limit, shift, lane, kProbe.v[lane],
                         kProbe.v[lane + 1], &ip, &cand))
        break;
      emit_literal(o, in, next_emit, ip - next_emit, lane);
      uint64_t eight = 0;
      for (;;) {
        const uint32_t base = ip;
        const uint32_t m = match_length(in, cand, ip, n, lane);
        ip += m;
        emit_copy(o, base - cand, m, lane);
        next_emit = ip;
        if (ip >= ip_limit) {
          remainder = true;
          break;
        }
        eight = ld64(in, ip - 1);
        const uint32_t prev_hash = hash32(static_cast<uint32_t>(eight), shift);
        table[prev_hash] = static_cast<uint16_t>(ip - 1);
        const uint32_t cur = static_cast<uint32_t>(eight >> 8);
        const uint32_t cur_hash = hash32(cur, shift);
        cand = table[cur_hash];
        const uint32_t cand_bytes = ld32(in, cand);
        table[cur_hash] = static_cast<uint16_t>(ip);
        if (cur != cand_bytes) break;
      }
      if (remainder) break;
      ++ip;
    }
  }
  if (next_emit < n) emit_literal(o, in, next_emit, n - next_emit, lane);
}

struct CompressArgs {
  const uint8_t* src;
  const uint64_t* src_off;
  const uint32_t* src_len;
  uint8_t* dst;
  const uint64_t* dst_off;
  uint32_t* dst_len;
  uint8_t* status;
  uint32_t nblocks;
  uint32_t frag_cap;    // the largest fragment the LDS holds (<= kFrag)
  uint64_t dst_stride;  // dst_off == nullptr: block b's output at b * dst_stride
  uint32_t max_len;     // dst_off == nullptr: the stride's sizing; longer blocks are TOO_LARGE
};

__global__ void __launch_bounds__(64) snappy_compress_kernel(CompressArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t b = blockIdx.x;
  if (b >= a.nblocks) return;
  const uint32_t lane = threadIdx.x;
  const uint32_t len = a.src_len[b];
  const uint8_t* src = a.src + a.src_off[b];
  const uint32_t in_bytes = (a.frag_cap + 16u + 15u) & ~15u;
  uint8_t* in = smem;
  uint32_t* slots = reinterpret_cast<uint32_t*>(smem + in_bytes);  // 256
  uint16_t* table = reinterpret_cast<uint16_t*>(slots + 256);
  // the caller's max_len was too small: the fragment does not fit the LDS,
  // or (fixed stride) the output would run into the next block's slot
  if (min(len, kFrag) > a.frag_cap || (a.dst_off == nullptr && len > a.max_len)) {
    if (lane == 0) {
      a.dst_len[b] = 0;
      a.status[b] = LVKV_SNAPPY_TOO_LARGE;
    }
    return;
  }
  Out o{a.dst + (a.dst_off ? a.dst_off[b] : b * a.dst_stride), 0};
  // varint32 of the uncompressed length
  uint32_t v = len;
  while (v >= 128) {
    if (lane == 0) o.p[o.n] = static_cast<uint8_t>(v | 128u);
    ++o.n;
    v >>= 7;
  }
  if (lane == 0) o.p[o.n] = static_cast<uint8_t>(v);
  ++o.n;
  for (uint32_t s = 0; s < len; s += kFrag) {
    const uint32_t fn = min(kFrag, len - s);
    stage(in, src + s, fn, 16, lane);
    __builtin_amdgcn_s_waitcnt(0);
    compress_fragment(in, fn, table, slots, o, lane);
    __builtin_amdgcn_s_waitcnt(0);
  }
  if (lane == 0) {
    a.dst_len[b] = o.n;
    a.status[b] = LVKV_SNAPPY_OK;
  }
}

// ---- decompression (snappy::GetUncompressedLength / RawUncompress) --------

struct UncompressArgs {
  const uint8_t* src;
  const uint64_t* src_off;
  const uint32_t* src_len;
  uint8_t* dst;
  const uint64_t* dst_off;
  const uint32_t* dst_cap;  // nullptr: lengths only
  uint32_t* out_len;
  uint8_t* status;
  uint32_t nblocks;
  uint32_t out_cap;  // the largest output the LDS holds
  // ReadBlock mode (lvkv_sst_read_blocks_device): src_off/src_len are block
  // handles, the type byte follows the contents, statuses are LVKV_READ_*;
  // vstatus = the checksum verdicts (nullptr: verify_checksums off)
  uint32_t block_mode;
  const uint8_t* vstatus;
};

// snappy::MaxCompressedLength: the longest stream the decompressor stages.
__host__ __device__ constexpr uint32_t snappy_in_cap(uint32_t out_cap) {
  return 32u + out_cap + out_cap / 6u;
}

// The varint32 preamble at in[0, n): its value and size, or size 0 (bad).
__device__ __forceinline__ uint32_t preamble(const uint8_t* in, uint32_t n, uint32_t* value) {
  uint32_t v = 0;
  for (uint32_t i = 0; i < 5 && i < n; ++i) {
    const uint32_t c = in[i];
    if (i == 4 && c >= 16) return 0;  // past 32 bits (or a continuation)
    v |= (c & 127u) << (7 * i);
    if (c < 128) {
      *value = v;
      return i + 1;
    }
  }
  return 0;
}

__global__ void __launch_bounds__(64) snappy_uncompress_kernel(UncompressArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t b = blockIdx.x;
  if (b >= a.nblocks) return;
  const uint32_t lane = threadIdx.x;
  const uint32_t n = a.src_len[b];
  const uint8_t* src = a.src + a.src_off[b];
  // the staging area holds MaxCompressedLength(out_cap) bytes: every stream
  // a snappy encoder writes for out_cap bytes
  const uint32_t in_cap = snappy_in_cap(a.out_cap);
  const uint32_t in_bytes = (in_cap + 16u + 15u) & ~15u;
  uint8_t* in = smem;
  uint8_t* out = smem + in_bytes;
  auto finish_read = [&](uint32_t st, uint32_t ol) {
    if (lane == 0) {
      a.status[b] = static_cast<uint8_t>(st);
      a.out_len[b] = ol;
    }
  };
  // codec status -> ReadBlock status in block mode
  auto finish = [&](uint32_t st, uint32_t ol) {
    constexpr uint8_t kRead[5] = {LVKV_READ_OK, LVKV_READ_SNAPPY_LENGTH, LVKV_READ_SNAPPY_CONTENTS,
                                  LVKV_READ_CAPACITY, LVKV_READ_TOO_LARGE};
    finish_read(a.block_mode ? kRead[st] : st, ol);
  };
  if (a.block_mode) {  // ReadBlock (table/format.cc:90-159): checksum, then the type
    const uint32_t type = src[n];
    if (a.vstatus != nullptr && a.vstatus[b] != 0)
      return finish_read(LVKV_READ_CHECKSUM, 0);  // :95-98
    if (type == 2) return;  // kZstdCompression: the zstd kernel's, launched next
    if (type > 2) return finish_read(LVKV_READ_BAD_TYPE, 0);  // :156-158
    if (type == 0) {  // kNoCompression: the contents as they are (:103-119)
      if (n > a.dst_cap[b]) return finish_read(LVKV_READ_CAPACITY, n);
      uint8_t* dst = a.dst + a.dst_off[b];
      for (uint32_t k = lane; k < n; k += 64) dst[k] = src[k];
      return finish_read(LVKV_READ_OK, n);
    }
  }
  uint32_t ulen = 0, pl;
  const bool staged = a.dst_cap != nullptr && n <= in_cap;
  if (staged) {  // the preamble from LDS, after one round trip for the lot
    stage(in, src, n, 16, lane);
    pl = preamble(in, n, &ulen);
  } else {  // (at most 5 bytes from global memory)
    pl = preamble(src, n, &ulen);
  }
  if (pl == 0) return finish(LVKV_SNAPPY_BAD_LENGTH, 0);  // format.cc:122-124
  if (a.dst_cap == nullptr) return finish(LVKV_SNAPPY_OK, ulen);
  if (ulen > a.dst_cap[b]) return finish(LVKV_SNAPPY_CAPACITY, ulen);
  if (ulen > a.out_cap) return finish(LVKV_SNAPPY_TOO_LARGE, ulen);
  // a longer stream is valid only with padded (non-canonical) elements --
  // no snappy encoder writes one; the caller decodes it on the host
  if (!staged) return finish(LVKV_SNAPPY_TOO_LARGE, ulen);
  uint32_t ip = pl, op = 0;
  bool ok = true;
  while (ip < n) {
    const uint64_t t8 = ld64(in, ip);
    const uint32_t tag = static_cast<uint32_t>(t8) & 255u;
    ++ip;
    if ((tag & 3u) == 0) {
      uint64_t len64 = (tag >> 2) + 1u;
      if (len64 > 60) {
        const uint32_t k = static_cast<uint32_t>(len64) - 60u;
        if (ip + k > n) {
          ok = false;
          break;
        }
        // snappy adds the 1 in uint32: a 4-byte length of 0xffffffff wraps
        // to an empty literal (libsnappy 1.1.8 accepts 03fcffffffff08616263)
        len64 = (((t8 >> 8) & ((uint64_t{1} << (8 * k)) - 1u)) + 1u) & 0xffffffffu;
        ip += k;
      }
      if (len64 > n - ip || len64 > ulen - op) {
        ok = false;
        break;
      }
      const uint32_t len = static_cast<uint32_t>(len64);
      for (uint32_t k = lane; k < len; k += 64) out[op + k] = in[ip + k];
      ip += len;
      op += len;
      continue;
    }
    uint32_t len, off;
    if ((tag & 3u) == 1) {
      if (ip + 1 > n) {
        ok = false;
        break;
      }
      len = ((tag >> 2) & 7u) + 4u;
      off = ((tag >> 5) << 8) | static_cast<uint32_t>((t8 >> 8) & 255u);
      ip += 1;
    } else if ((tag & 3u) == 2) {
      if (ip + 2 > n) {
        ok = false;
        break;
      }
      len = (tag >> 2) + 1u;
      off = static_cast<uint32_t>((t8 >> 8) & 0xffffu);
      ip += 2;
    } else {
      if (ip + 4 > n) {
        ok = false;
        break;
      }
      len = (tag >> 2) + 1u;
      off = static_cast<uint32_t>((t8 >> 8) & 0xffffffffu);
      ip += 4;
    }
    if (off == 0 || off > op || len > ulen - op) {
      ok = false;
      break;
    }
    // len <= 64: one lane a byte; an overlapping copy repeats its last
    // `off` bytes (byte k = out[op - off + k % off])
    if (lane < len) {
      const uint32_t k = off >= len ? lane : lane % off;
      out[op + lane] = out[op - off + k];
    }
    op += len;
  }
  if (!ok || op != ulen) return finish(LVKV_SNAPPY_BAD_CONTENTS, ulen);
  uint8_t* dst = a.dst + a.dst_off[b];
  uint32_t k0 = 0;
  if ((reinterpret_cast<uintptr_t>(dst) & 3u) == 0) {
    const uint32_t nd = ulen >> 2;
    for (uint32_t i = lane; i < nd; i += 64)
      reinterpret_cast<uint32_t*>(dst)[i] = reinterpret_cast<const uint32_t*>(out)[i];
    k0 = 4u * nd;
  }
  for (uint32_t k = k0 + lane; k < ulen; k += 64) dst[k] = out[k];
  finish(LVKV_SNAPPY_OK, ulen);
}

// Blocks the LDS path hands back (TOO_LARGE: a longer output than the
// call's LDS staging, or a stream past MaxCompressedLength of it) decoded
// straight into the HBM output, any size (table/format.cc:120-135 reads
// any block): the stream through an 8 KiB LDS window, the output written to
// the destination as it is produced and its last 32 KiB also kept in an LDS
// ring. A copy from within the ring reads LDS; a farther one reads the
// destination, where every byte that old has landed: the wave waits for
// its stores (vmcnt(0)) each time the output crosses 8 KiB. Runs after
// snappy_uncompress_kernel over the same batch; a block it did not mark
// TOO_LARGE exits at once.
constexpr uint32_t kBigWin = 8192, kBigRing = 32768, kBigChunk = 32;

__device__ __forceinline__ void snappy_big_block(const UncompressArgs& a, uint32_t b, uint8_t* smem, uint32_t lane) {
  const uint32_t n = a.src_len[b];
  const uint8_t* src = a.src + a.src_off[b];
  // (ReadBlock mode: only snappy blocks; a zstd block's status is the zstd
  // kernel's, launched next)
  if (a.block_mode && __builtin_amdgcn_readfirstlane(src[n]) != 1u) return;
  uint8_t* dst = a.dst + a.dst_off[b];
  uint8_t* win = smem;                  // src[wbase, wbase + kBigWin) + 16 zero bytes
  uint8_t* ring = smem + kBigWin + 16;  // out[p] at ring[p % kBigRing]
  auto finish = [&](uint32_t st, uint32_t ol) {
    if (lane == 0) {
      a.status[b] = static_cast<uint8_t>(
          a.block_mode ? (st == LVKV_SNAPPY_OK ? LVKV_READ_OK : LVKV_READ_SNAPPY_CONTENTS) : st);
      a.out_len[b] = ol;
    }
  };
  uint32_t ulen = 0;
  const uint32_t pl = preamble(src, n, &ulen);  // (checked by the LDS path)
  uint32_t wbase = 0, wlen = 0;
  auto window = [&](uint32_t at) {  // the window from at (4-aligned)
    wbase = at & ~3u;
    wlen = n - wbase < kBigWin ? n - wbase : kBigWin;
    stage(win, src + wbase, wlen, 16, lane);
    __builtin_amdgcn_s_waitcnt(0);
  };
  window(pl);
  uint32_t ip = pl, op = 0, flushed_at = 0;
  bool ok = true;
  while (ip < n) {
    if (ip + 5u > wbase + wlen && wbase + wlen < n) window(ip);
    const uint64_t t8 = ld64(win, ip - wbase);
    const uint32_t tag = static_cast<uint32_t>(t8) & 255u;
    ++ip;
    if ((tag & 3u) == 0) {
      uint64_t len64 = (tag >> 2) + 1u;
      if (len64 > 60) {
        const uint32_t k = static_cast<uint32_t>(len64) - 60u;
        if (ip + k > n) {
          ok = false;
          break;
        }
        len64 = (((t8 >> 8) & ((uint64_t{1} << (8 * k)) - 1u)) + 1u) & 0xffffffffu;
        ip += k;
      }
      if (len64 > n - ip || len64 > ulen - op) {
        ok = false;
        break;
      }
      const uint32_t len = static_cast<uint32_t>(len64);
      // the bytes from global memory into the output and the ring
      for (uint32_t k = lane; k < len; k += 64) {
        const uint8_t v = src[ip + k];
        dst[op + k] = v;
        ring[(op + k) & (kBigRing - 1u)] = v;
      }
      ip += len;
      op += len;
    } else {
      uint32_t len, off;
      if ((tag & 3u) == 1) {
        if (ip + 1 > n) {
          ok = false;
          break;
        }
        len = ((tag >> 2) & 7u) + 4u;
        off = ((tag >> 5) << 8) | static_cast<uint32_t>((t8 >> 8) & 255u);
        ip += 1;
      } else if ((tag & 3u) == 2) {
        if (ip + 2 > n) {
          ok = false;
          break;
        }
        len = (tag >> 2) + 1u;
        off = static_cast<uint32_t>((t8 >> 8) & 0xffffu);
        ip += 2;
      } else {
        if (ip + 4 > n) {
          ok = false;
          break;
        }
        len = (tag >> 2) + 1u;
        off = static_cast<uint32_t>((t8 >> 8) & 0xffffffffu);
        ip += 4;
      }
      if (off == 0 || off > op || len > ulen - op) {
        ok = false;
        break;
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);  // (the ring's earlier bytes have landed)
      if (lane < len) {
        const uint32_t k = off >= len ? lane : lane % off;
        const uint32_t from = op - off + k;
        const uint8_t v = off <= kBigRing - 64u ? ring[from & (kBigRing - 1u)] : dst[from];
        dst[op + lane] = v;
        ring[(op + lane) & (kBigRing - 1u)] = v;
      }
      op += len;
    }
    if (op - flushed_at >= kBigWin) {  // every byte before flushed_at is in HBM
      __builtin_amdgcn_s_waitcnt(0);
      flushed_at = op;
    }
  }
  __builtin_amdgcn_s_waitcnt(0);
  if (!ok || op != ulen) return finish(LVKV_SNAPPY_BAD_CONTENTS, ulen);
  finish(LVKV_SNAPPY_OK, ulen);
}

// One workgroup per 32 blocks: their statuses in one load, then the marked
// ones one after another (a batch without big blocks costs a short launch).
__global__ void __launch_bounds__(64) snappy_uncompress_big_kernel(UncompressArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t lane = threadIdx.x;
  const uint32_t b0 = blockIdx.x * kBigChunk;
  const uint32_t mark = a.block_mode ? LVKV_READ_TOO_LARGE : LVKV_SNAPPY_TOO_LARGE;
  const bool mine = lane < kBigChunk && b0 + lane < a.nblocks && a.status[b0 + lane] == mark;
  uint64_t todo = __ballot(mine);
  while (todo) {
    const uint32_t b = b0 + static_cast<uint32_t>(__builtin_ctzll(todo));
    todo &= todo - 1u;
    snappy_big_block(a, b, smem, lane);
  }
}

// ---- TableBuilder::WriteBlock over a batch (table/table_builder.cc:141-209) --

__device__ __forceinline__ uint64_t shfl_up64(uint64_t v, uint32_t d) {
  const uint32_t lo = __shfl_up(static_cast<uint32_t>(v), d);
  const uint32_t hi = __shfl_up(static_cast<uint32_t>(v >> 32), d);
  return (static_cast<uint64_t>(hi) << 32) | lo;
}

// Which form each block keeps and where it lands: the compressed form when
// it is smaller than raw - raw/8 (table_builder.cc:160-168), else raw with
// type kNoCompression; handles are an exclusive scan of size + 5 (the
// trailer, :206) from file_offset. One workgroup, 4 blocks a thread a pass.
__global__ void __launch_bounds__(1024) sst_layout_kernel(const uint32_t* raw_len,
                                                          const uint32_t* clen, const uint8_t* cst,
                                                          uint32_t n, uint64_t file_offset,
                                                          uint64_t* hoff, uint32_t* hsize,
                                                          uint8_t* type, uint64_t* end,
                                                          uint32_t ctype) {
  __shared__ uint64_t wsum[17];
  const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
  uint64_t carry = file_offset;
  for (uint32_t base = 0; base < n; base += 4096) {
    uint32_t sz[4];
    uint8_t ty[4];
    uint64_t local = 0;
    for (uint32_t j = 0; j < 4; ++j) {
      const uint32_t i = base + 4 * t + j;
      sz[j] = 0;
      ty[j] = 0;
      if (i < n) {
        const uint32_t L = raw_len[i];
        const bool c = clen != nullptr && cst[i] == LVKV_SNAPPY_OK && clen[i] < L - L / 8u;
        sz[j] = c ? clen[i] : L;
        ty[j] = c ? static_cast<uint8_t>(ctype) : 0;
        local += sz[j] + 5u;
      }
    }
    uint64_t incl = local;
    for (uint32_t d = 1; d < 64; d <<= 1) {
      const uint64_t y = shfl_up64(incl, d);
      if (lane >= d) incl += y;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    if (w == 0) {
      const uint64_t v = lane < 16 ? wsum[lane] : 0;
      uint64_t s = v;
      for (uint32_t d = 1; d < 16; d <<= 1) {
        const uint64_t y = shfl_up64(s, d);
        if (lane >= d) s += y;
      }
      if (lane < 16) wsum[lane] = s - v;  // exclusive
      if (lane == 15) wsum[16] = s;       // the pass's total
    }
    __syncthreads();
    uint64_t at = carry + wsum[w] + incl - local;
    for (uint32_t j = 0; j < 4; ++j) {
      const uint32_t i = base + 4 * t + j;
      if (i < n) {
        hoff[i] = at;
        hsize[i] = sz[j];
        type[i] = ty[j];
        at += sz[j] + 5u;
      }
    }
    carry += wsum[16];
    __syncthreads();
  }
  if (t == 0) *end = carry;
}

// WriteRawBlock's bytes but the CRC (table_builder.cc:195-204): the kept
// contents at the handle, the type byte after them. The masked CRC is the
// batch CRC kernel's (lvkv_sst_fill_trailers_device) over the same handles.
__global__ void __launch_bounds__(256) sst_place_kernel(const uint8_t* raw, const uint64_t* raw_off,
                                                        const uint8_t* comp, uint64_t comp_stride,
                                                        const uint64_t* hoff, const uint32_t* hsize,
                                                        const uint8_t* type, uint8_t* file) {
  const uint32_t b = blockIdx.x, t = threadIdx.x;
  const uint32_t ty = type[b];
  const uint8_t* src = ty ? comp + b * comp_stride : raw + raw_off[b];
  uint8_t* dst = file + hoff[b];
  const uint32_t n = hsize[b];
  for (uint32_t k = t; k < n; k += 256) dst[k] = src[k];
  if (t == 0) dst[n] = static_cast<uint8_t>(ty);
}

}  // namespace

// A block's compressed scratch slot: room for either codec's bound
// (snappy::MaxCompressedLength, ZSTD_compressBound).
uint64_t snappy_write_stride(uint32_t max_len) {
  const uint64_t zb = uint64_t{max_len} + (max_len >> 8) +
                      (max_len < (128u << 10) ? ((128u << 10) - max_len) >> 11 : 0u);
  const uint64_t sb = snappy_in_cap(max_len);
  return ((sb > zb ? sb : zb) + 15u) & ~uint64_t{15};
}

hipError_t launch_zstd_compress(const uint8_t* src, const uint64_t* src_off, const uint32_t* src_len,
                                uint8_t* dst, const uint64_t* dst_off, uint32_t* dst_len,
                                uint8_t* status, uint32_t nblocks, uint32_t max_len, int level,
                                uint64_t dst_stride, hipStream_t stream);

hipError_t launch_sst_write_blocks(const uint8_t* raw, const uint64_t* raw_off,
                                   const uint32_t* raw_len, uint32_t nblocks, int compression,
                                   uint32_t max_len, uint8_t* scratch, uint8_t* file,
                                   uint64_t file_offset, uint64_t* hoff, uint32_t* hsize,
                                   uint8_t* type, uint64_t* end, int zstd_level,
                                   hipStream_t stream) {
  const uint64_t stride = snappy_write_stride(max_len);
  uint32_t* clen = nullptr;
  uint8_t* cst = nullptr;
  if (compression == 1 && nblocks != 0) {
    clen = reinterpret_cast<uint32_t*>(scratch + stride * nblocks);
    cst = reinterpret_cast<uint8_t*>(clen + nblocks);
    CompressArgs a{raw, raw_off, raw_len, scratch, nullptr, clen, cst, nblocks, 0, stride, max_len};
    a.frag_cap = max(16u, min(max_len, kFrag));
    const uint32_t in_bytes = (a.frag_cap + 16u + 15u) & ~15u;
    uint32_t t = 256;
    while (t < kMaxTable && t < a.frag_cap) t <<= 1;
    const size_t lds = in_bytes + 1024u + 2u * t;
    hipLaunchKernelGGL(snappy_compress_kernel, dim3(nblocks), dim3(64), lds, stream, a);
  } else if (compression == 2 && nblocks != 0) {  // kZstdCompression
    clen = reinterpret_cast<uint32_t*>(scratch + stride * nblocks);
    cst = reinterpret_cast<uint8_t*>(clen + nblocks);
    const hipError_t e = launch_zstd_compress(raw, raw_off, raw_len, scratch, nullptr, clen, cst,
                                              nblocks, max_len, zstd_level, stride, stream);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(sst_layout_kernel, dim3(1), dim3(1024), 0, stream, raw_len, clen, cst,
                     nblocks, file_offset, hoff, hsize, type, end,
                     static_cast<uint32_t>(compression == 2 ? 2 : 1));
  if (nblocks == 0) return hipGetLastError();  // (the layout stored end = file_offset)
  hipLaunchKernelGGL(sst_place_kernel, dim3(nblocks), dim3(256), 0, stream, raw, raw_off,
                     scratch, stride, hoff, hsize, type, file);
  return hipGetLastError();
}

hipError_t launch_sst_read_blocks(const uint8_t* file, const uint64_t* hoff, const uint32_t* hsize,
                                  uint32_t nblocks, uint8_t* out, const uint64_t* out_off,
                                  const uint32_t* out_cap, uint32_t* out_len, uint8_t* status,
                                  const uint8_t* vstatus, uint32_t max_ulen, hipStream_t stream) {
  UncompressArgs a{file, hoff, hsize, out, out_off, out_cap, out_len, status, nblocks, 0, 1,
                   vstatus};
  a.out_cap = max(16u, max_ulen);
  const size_t lds = ((snappy_in_cap(a.out_cap) + 16u + 15u) & ~15u) + ((a.out_cap + 15u) & ~15u);
  hipLaunchKernelGGL(snappy_uncompress_kernel, dim3(nblocks), dim3(64), lds, stream, a);
  hipLaunchKernelGGL(snappy_uncompress_big_kernel, dim3((nblocks + kBigChunk - 1u) / kBigChunk),
                     dim3(64), kBigWin + 16u + kBigRing, stream, a);
  return hipGetLastError();
}

hipError_t launch_snappy_compress(const uint8_t* src, const uint64_t* src_off,
                                  const uint32_t* src_len, uint8_t* dst, const uint64_t* dst_off,
                                  uint32_t* dst_len, uint8_t* status, uint32_t nblocks,
                                  uint32_t max_len, hipStream_t stream) {
  CompressArgs a{src, src_off, src_len, dst, dst_off, dst_len, status, nblocks, 0};
  a.frag_cap = max(16u, min(max_len, kFrag));
  const uint32_t in_bytes = (a.frag_cap + 16u + 15u) & ~15u;
  uint32_t t = 256;
  while (t < kMaxTable && t < a.frag_cap) t <<= 1;
  const size_t lds = in_bytes + 1024u + 2u * t;
  hipLaunchKernelGGL(snappy_compress_kernel, dim3(nblocks), dim3(64), lds, stream, a);
  return hipGetLastError();
}

hipError_t launch_snappy_uncompress(const uint8_t* src, const uint64_t* src_off,
                                    const uint32_t* src_len, uint8_t* dst, const uint64_t* dst_off,
                                    const uint32_t* dst_cap, uint32_t* out_len, uint8_t* status,
                                    uint32_t nblocks, uint32_t max_ulen, hipStream_t stream) {
  UncompressArgs a{src, src_off, src_len, dst, dst_off, dst_cap, out_len, status, nblocks, 0};
  a.out_cap = dst_cap == nullptr ? 0u : max(16u, max_ulen);
  const size_t lds = dst_cap == nullptr ? 16u
                                        : ((snappy_in_cap(a.out_cap) + 16u + 15u) & ~15u) +
                                              ((a.out_cap + 15u) & ~15u);
  hipLaunchKernelGGL(snappy_uncompress_kernel, dim3(nblocks), dim3(64), lds, stream, a);
  if (dst_cap != nullptr)  // (the blocks past the LDS staging, any size)
    hipLaunchKernelGGL(snappy_uncompress_big_kernel,
                       dim3((nblocks + kBigChunk - 1u) / kBigChunk), dim3(64),
                       kBigWin + 16u + kBigRing, stream, a);
  return hipGetLastError();
}

}  // namespace lvkv
