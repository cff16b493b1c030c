// WAL / MANIFEST verify on the device: every physical
// record of a log image, with log::Reader::ReadPhysicalRecord's reporting
// (db/log_reader.cc:189-271, checksum = true, initial_offset = 0).
//
// Headers never straddle a 32 KiB block (the writer pads the tail of a block
// with zeros, db/log_writer.cc:44-55) and the reader drops the REST OF THE
// BLOCK on every error, so each block's verdict depends on that block only.
// One read of the image, two launches:
//
//   log_verify_kernel  one 1024-thread workgroup per CU with TWO block
//                      slots in LDS (32 KiB each) beside the 64 KiB CRC
//                      image. Wave m (m < 2) manages slot m: it claims the
//                      next block with a ticket (an atomic counter, so no
//                      workgroup ever waits on one that has not started,
//                      whatever the residency), copies it into the slot by
//                      LDS-DMA (buffer_load ... lds, no registers), walks its
//                      headers, reserves the block's records a run of the
//                      staging array (an atomic bump), waits for the block's
//                      CRCs and stages the block's results.
//                      The walk is a chain of dependent LDS reads (≈ 80 ns
//                      a header alone, ≈ 200 ns beside the record waves'
//                      traffic, tools/probe/walk_probe.hip and the phase
//                      stamps): it is the kernel's critical path, so a CU
//                      walks two blocks at once. The fourteen other waves
//                      checksum each record as soon as the walker has
//                      published its position (records two at a time, from
//                      any slot). Records over kSegBytes are cut into 4 KiB
//                      segments on the end-aligned grid, checksummed by
//                      several waves and folded with Z_{i·4 KiB} (the zmul
//                      columns). The block's merge (db/log_reader.cc:221-255):
//                      the first mismatch drops the rest of the block; block
//                      status and drop bytes. Nothing waits for a block's
//                      place in file order (that would wait for the slowest
//                      block in flight before it).
//   log_emit_kernel    one wave per block: its first record index (the counts
//                      of the blocks before it, summed by each workgroup), the
//                      staged results moved to their places (and the ReadRecord
//                      event stream); the last workgroup writes the report.
//
// The CRC (same arithmetic as every kernel here): rows of 64
// words folded with Z_256 by four byte lookups in LDS, then each lane's
// Z_{256-4s} end shift, on the compact 64 KiB image (crc32c_compact_common.h).
// Three or four slots with a smaller image (row tables in 16-32 KiB, the end
// shift from columns in registers) walk more blocks at once but make each
// record's CRC dearer, and measured slower (84 and 94 against 76 µs on the
// 66 MB log): the workers, not the walks, then set the pace.
//
// Scratch (lvkv_capi.cpp, one buffer per call in flight): counters left at 0
// by the emit launch of every call, per-block words, the staging array
// and each slot's overflow positions (blocks of more than kPosLds records).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>

#include "crc32c_compact_common.h"
#include "crc32c_device_common.h"
#include "lvkv_crc32c.h"
#include "lvkv_kernel_args.h"
#include "lvkv_log_events.h"

namespace lvkv {
namespace {

constexpr uint64_t kLogBlock = 32768;  // db/log_format.h kBlockSize
constexpr uint32_t kLogHeader = 7;     // db/log_format.h kHeaderSize

constexpr int kVW = 16;  // waves per workgroup
constexpr uint32_t kVThreads = 64 * kVW;
constexpr uint32_t kSlots = 2;  // blocks in LDS per workgroup (one manager wave each)
constexpr uint32_t kMaxRecs = (static_cast<uint32_t>(kLogBlock) + kLogHeader - 1) / kLogHeader;
constexpr uint32_t kPosLds = 4096;  // positions per slot in LDS; the rest in scratch
constexpr uint32_t kPosOver = kMaxRecs - kPosLds;
// a slot holds the block from its 16-byte aligned start: up to 15 bytes before it
constexpr uint32_t kBufBytes = static_cast<uint32_t>(kLogBlock) + 16;
constexpr uint32_t kSegBytes = 4096;  // CRC bytes one wave takes at most
constexpr uint32_t kLog2Seg = 12;
constexpr uint32_t kMaxLong = static_cast<uint32_t>(kLogBlock) / (kSegBytes + 1) + 1;  // 8

struct LogArgs {
  const uint8_t* file;
  uint64_t size;
  uint32_t nblocks, capacity;
  uint64_t* hdr_off;
  uint32_t* actual;
  uint8_t* rec_status;
  uint8_t* block_status;
  uint32_t* block_drop;
  lvkv_log_report* r;
  ulonglong2* info;  // nblocks: {count | good << 32, drop | status << 32}
  uint32_t* stg_off; // nblocks: the block's first entry in `stg`
  uint4* stg;        // capacity: per record {actual, pos | len << 16, type, status}
  uint32_t* over;    // groups x kSlots x kPosOver: positions past kPosLds
  uint32_t* ticket;  // blocks claimed (left at 0 by the emit launch)
  uint32_t* stg_top; // staging entries reserved (left at 0 by the emit launch)
  const uint32_t* zpow;
  const uint32_t* lane_cols;
  uint32_t* events;  // nullable: the ReadRecord event stream (lvkv_log_events.h)
  uint64_t* item_off;  // with events: each item's header offset
  // many blocks: the records before each block (nblocks + 1 entries), scanned
  // by log_scan_kernel for the emit; else nullptr
  unsigned long long* first_of;
  uint64_t* stamps;  // probe build only: 8 u64 per (workgroup, slot, block)
  uint32_t knobs;    // probe build only: bit 0 = workers idle, no CRCs; bits 8-11:
                     // worker waves that sit out (timing)
};

// Manager phase stamps (probe build): 0 claimed, 1 in LDS, 2 walked,
// 3 CRCs done, 4 staged; row (slot 0, k 15) holds the workgroup's own.
__device__ __forceinline__ void log_stamp(const LogArgs& a, uint32_t m, uint32_t k, int slot) {
#ifdef LVKV_PROBE_BUILD
  if (a.stamps != nullptr && lane_id() == 0)
    a.stamps[((static_cast<uint64_t>(blockIdx.x) * kSlots + m) * 16u + min(k, 15u)) * 8u + slot] =
        __builtin_amdgcn_s_memrealtime();
#endif
}

__device__ __forceinline__ uint32_t lds_word(const uint8_t* buf, uint32_t x) {
  const uint32_t* d = reinterpret_cast<const uint32_t*>(buf + (x & ~3u));
  const uint32_t lo = d[0];
  const uint32_t hi = d[1];
  return (x & 3u) ? __builtin_amdgcn_alignbyte(hi, lo, x & 3u) : lo;
}

// ---- record CRCs from LDS ----------------------------------------------

// A lane's constants on the compact image (crc32c_compact_common.h): its
// four lookups' v_perm keys and its nibble-table column.
struct LogLane {
  LaneKeys keys;
  uint32_t lane_base;
};

// CRC32C registers of buf[a, a + n) (LDS, n >= 4) by one wave: the
// end-aligned word grid (grid word j = the 4 bytes ending 4 * (q - 1 - j)
// before the end, lane s of row r holds word 64 r + s), Horner over rows
// with Z_256, lane end shift, xor-reduce. `inj` is xored into the first 4
// data bytes (spilling into the next word): ~0 for a record (the CRC's
// initial state), 0 for a segment after the first; `fin` is xored into the
// result (~0 for a CRC, 0 for a segment's register).
struct LdsRec {
  uint32_t first, s0l, sh, msk, inj, spill;
};

// Geometry of a record of n >= 4 bytes at a on a grid of `rows` rows (at
// least its own; extra rows in front are all-zero words, which leave the
// register at 0, so two records can share one row count).
__device__ __forceinline__ LdsRec lds_rec(uint32_t a, uint32_t n, uint32_t rows, uint32_t inj) {
  LdsRec r;
  const uint32_t q = (n + 3u) >> 2;
  const uint32_t delta = 4u * q - n;
  r.s0l = 64u * rows - q;
  r.sh = 8u * delta;
  r.msk = 0xffffffffu << r.sh;
  r.inj = inj << r.sh;
  r.spill = delta ? (inj >> (32u - r.sh)) : 0u;
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
  w = j == g.s0l ? ((w & g.msk) ^ g.inj) : w;
  return j == g.s0l + 1u ? (w ^ g.spill) : w;
}

// NR records at once. Each row issues every LDS read of every record (the
// two data dwords and the four Z_256 lookups of the running state) before
// any is consumed, so a row costs one LDS round trip for all of them; the
// scheduling barriers keep the compiler from pairing each read with its use.
template <int NR>
__device__ __forceinline__ void lds_record_crcs(const uint8_t* buf, const uint32_t (&at)[NR],
                                                const uint32_t (&n)[NR], const uint32_t (&inj)[NR],
                                                uint32_t fin, const uint32_t* img,
                                                const LogLane& L, uint32_t lane,
                                                uint32_t (&crc)[NR]) {
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
      g[t] = lds_rec(at[t], n[t], rows, inj[t]);
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
        v[t][p] = lds_ld(img, __builtin_amdgcn_perm(st[t], L.keys.kpack, L.keys.sel[p]));
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
      e[t][k] = lds_ld(img, (L.lane_base | (((st[t] >> (4 * k)) & 15u) << 9)) + 8192u * k);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int t = 0; t < NR; ++t) {
    const uint32_t r = xor3(xor3(e[t][0], e[t][1], e[t][2]), xor3(e[t][3], e[t][4], e[t][5]),
                            e[t][6] ^ e[t][7]);
    crc[t] = wave_xor_dpp(r) ^ fin;
  }
}

// Bitwise register update over n (< 4) bytes from `reg` (lane-uniform).
__device__ __forceinline__ uint32_t tiny_reg(const uint8_t* p, uint32_t n, uint32_t reg) {
  for (uint32_t i = 0; i < n; ++i) {
    reg ^= p[i];
#pragma unroll
    for (int k = 0; k < 8; ++k) reg = (reg >> 1) ^ (kCastagnoliReflected & (0u - (reg & 1u)));
  }
  return reg;
}

// ---- the per-slot state in LDS -------------------------------------------
//
// Every word a worker reads to decide what to take carries the slot's
// generation (bumped each time the slot takes a new block), so a worker
// that lags behind a recycled slot sees a foreign generation and backs off.
//   next   (gen << 16) | records claimed by workers (two per claim)
//   prog   (gen << 17) | walk finished << 16 | records walked (published)
//   lclaim (gen << 16) | long-record segments claimed
//   lavail (gen << 16) | long-record segments registered by the walker
constexpr uint32_t kGenShift = 17, kDoneBit = 1u << 16;

struct Slot {
  uint32_t next, prog, lclaim, lavail;
  uint32_t crcd;       // records whose CRC is final (this generation)
  uint32_t first_bad;  // smallest record index whose CRC mismatched
  uint32_t shift;      // the block starts at buf + shift (its 16-byte misalignment)
  uint32_t nlong;
  uint16_t lj[kMaxLong];     // long record: index
  uint16_t lp[kMaxLong];     // position
  uint8_t lseg[kMaxLong];    // segments
  uint8_t lfirst[kMaxLong];  // first segment's index in the slot's segment numbering
  uint32_t lacc[kMaxLong];   // xor of the segments' shifted registers
  uint32_t lrem[kMaxLong];   // segments not yet folded in
};

__device__ __forceinline__ uint32_t lds_load_acq(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_store_rel(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Record j's position in its block: LDS for the first kPosLds, the slot's
// scratch overflow after (stored sc1 by the walker, waited for before it
// published the count).
__device__ __forceinline__ uint32_t pos_of(const uint16_t* pos, const uint32_t* over, uint32_t j) {
  return j < kPosLds ? pos[j]
                     : __hip_atomic_load(&over[j - kPosLds], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void put_pos(uint16_t* pos, uint32_t* over, uint32_t j, uint32_t p) {
  if (j < kPosLds) {
    pos[j] = static_cast<uint16_t>(p);
  } else {
    __hip_atomic_store(&over[j - kPosLds], p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

// Walks one block's headers in LDS, blk[0, n), to the first stop (bad
// length, zero record, end) like ReadPhysicalRecord, publishing the records'
// positions as it goes (8 at a time: positions, then S.prog) and registering
// records longer than kSegBytes for segmented CRCs. Called by the manager
// wave with uniform arguments. Returns the verdict; *count, *stop = the
// records and the block offset after the last one.
//
// Every lane carries the same position in a VGPR (bp, its LDS address), so
// the chain from one header to the next is one LDS round trip and a v_add3:
// the length is an unaligned ds_read_u16 at bp + 4 (the type byte, for the
// zero-record test, a ds_read_u8 beside it). The next header's reads are
// issued before this header's stop test (speculatively: a read past the
// block, about to stop the walk, lands elsewhere in LDS or past the
// allocation and is never used), so the test overlaps the LDS trip. The
// reads are inline asm so the compiler neither sinks the speculative ones
// below the branch nor turns the chain scalar; their registers are tied to
// explicit lgkmcnt waits (an asm load's destination is written late, so it
// must stay live until a wait has seen it land). Positions collect in a
// register (record k in lane k % 64) and are written 8 at a time.
// (Measured against: the block held in an 8 KiB register window, each
// header read by a uniform register index and v_readlane, the chain on the
// scalar unit: 320 shader clocks a header alone against this walk's 193,
// tools/probe/walk_probe.hip variant 5; the cross-unit chain is longer than
// the LDS round trip.)
__device__ __forceinline__ uint8_t walk_block(const uint8_t* blk, uint32_t n, bool eof,
                                              uint16_t* pos, uint32_t* over, Slot& S,
                                              uint32_t gen, uint32_t* count, uint32_t* stop,
                                              const LogArgs& la, uint32_t sm, uint32_t sk) {
  const uint32_t lane = lane_id();
  // (uniform, and seen so: the walk's tests and branches stay scalar)
  const uint32_t base =
      __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(reinterpret_cast<uintptr_t>(blk)));
  const uint32_t end = base + __builtin_amdgcn_readfirstlane(n);
  uint32_t k = 0, bp = base, len = 0, typ = 0;
  uint32_t nseg = 0;  // long-record segments registered
  uint32_t held = 0;  // position of record k in lane k % 64
  if (n >= kLogHeader) {
    uint32_t nlen, ntyp, vlen, vtyp;
    asm volatile("ds_read_u16 %0, %2 offset:4\n\tds_read_u8 %1, %2 offset:6\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(vlen), "=&v"(vtyp)
                 : "v"(bp));
    log_stamp(la, sm, sk, 5);
    // the header's fields as scalars: the tests and the next address on the
    // scalar unit, two v_readfirstlane after each LDS trip
    len = __builtin_amdgcn_readfirstlane(vlen);
    typ = __builtin_amdgcn_readfirstlane(vtyp);
    for (;;) {
      const uint32_t nbp = bp + kLogHeader + len;
      asm volatile("ds_read_u16 %0, %2 offset:4\n\tds_read_u8 %1, %2 offset:6"
                   : "=&v"(nlen), "=&v"(ntyp)
                   : "v"(nbp));
      __builtin_amdgcn_sched_barrier(0);  // the reads issue before the tests below
      // a bad length (:221-232) or a zero record (:234-240) ends the walk
      // (tests as sign bits of 32-bit differences: one scalar compare and
      // branch each, not a chain of selects; offsets and lengths < 2^31)
      const uint32_t left = end - nbp;
      if (((left | ((len | typ) - 1u)) >> 31) != 0) break;
      held = lane == (k & 63u) ? bp - base : held;
      const uint32_t kk = k + 1u;
      // the rare cases behind one test: a record longer than kSegBytes, a
      // batch of 8 positions to publish, a record ending within 7 bytes of
      // the block end
      static_assert(kSegBytes == 4096u && kLogHeader == 7u, "the tests below");
      if (__builtin_expect(((len >> 12) | (((kk & 7u) - 1u) >> 31) | ((left - 7u) >> 31)) != 0, 0)) {
        if (len + 1u > kSegBytes) {
          // a long record: its segments go to the long queue
          const uint32_t m = (len + 1u + kSegBytes - 1u) / kSegBytes;
          if (lane == 0) {
            const uint32_t e = S.nlong++;
            S.lj[e] = static_cast<uint16_t>(k);
            S.lp[e] = static_cast<uint16_t>(bp - base);
            S.lseg[e] = static_cast<uint8_t>(m);
            S.lfirst[e] = static_cast<uint8_t>(nseg);
            S.lacc[e] = 0;
            S.lrem[e] = m;
          }
          nseg += m;
          if (lane == 0) lds_store_rel(&S.lavail, (gen << 16) | nseg);
        }
        if ((kk & 7u) == 0) {
          // records kk-8 .. kk-1: their lanes write their positions, then the
          // first of them publishes the count (LDS keeps one wave's order; the
          // overflow's sc1 stores are waited for first)
          const uint32_t g0 = (kk - 8u) & 63u;
          if ((lane & ~7u) == g0) {
            put_pos(pos, over, kk - 8u + (lane & 7u), held);
            if (lane == g0) lds_store_rel(&S.prog, (gen << kGenShift) | kk);
          }
        }
        if (left < kLogHeader) {
          k = kk;
          bp = nbp;
          break;
        }
      }
      k = kk;
      bp = nbp;
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(nlen), "+v"(ntyp));
      len = __builtin_amdgcn_readfirstlane(nlen);
      typ = __builtin_amdgcn_readfirstlane(ntyp);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(nlen), "+v"(ntyp));
  }
  log_stamp(la, sm, sk, 6);
  const uint32_t p = __builtin_amdgcn_readfirstlane(bp - base);
  len = __builtin_amdgcn_readfirstlane(len);
  // the last 0-7 positions
  if (lane >= (k & ~7u & 63u) && lane < (k & ~7u & 63u) + (k & 7u))
    put_pos(pos, over, (k & ~7u) + (lane & 7u), held);
  uint8_t v;
  if (n - p < kLogHeader)
    v = (eof && p < n) ? LVKV_LOGBLK_EOF : LVKV_LOGBLK_OK;  // :206-213
  else if (kLogHeader + len > n - p)
    v = eof ? LVKV_LOGBLK_EOF : LVKV_LOGBLK_BAD_LENGTH;
  else
    v = LVKV_LOGBLK_ZERO;
  if (lane == 0) lds_store_rel(&S.prog, (gen << kGenShift) | kDoneBit | k);
  *count = k;
  *stop = p;
  return v;
}

// Writes a record's final CRC into its header's CRC bytes (where the stage
// step reads it back) and notes a mismatch; lane 0.
__device__ __forceinline__ void record_done(const uint8_t* blk, uint32_t p, uint32_t crc,
                                            uint32_t j, Slot& S) {
  uint8_t* hb = const_cast<uint8_t*>(blk) + p;
  if (crc != crc_unmask(lds_word(blk, p))) atomicMin(&S.first_bad, j);
  hb[0] = static_cast<uint8_t>(crc);
  hb[1] = static_cast<uint8_t>(crc >> 8);
  hb[2] = static_cast<uint8_t>(crc >> 16);
  hb[3] = static_cast<uint8_t>(crc >> 24);
}

// Block b into a slot's LDS buffer by LDS-DMA from its 16-byte aligned
// start: full 16-byte lines as dwordx4, the last 0-15 bytes by byte loads
// (a sub-dword LDS-DMA does not land one byte per lane). Issued only: the
// caller waits (vmcnt) before reading the slot. Returns the block's
// misalignment (its first byte is at sbuf + shift).
__device__ __forceinline__ uint32_t dma_block(const LogArgs& a, uint32_t b, uint8_t* sbuf,
                                              uint32_t lane) {
  const uint64_t start = uint64_t{b} * kLogBlock;
  const uint32_t n = static_cast<uint32_t>(min(a.size, start + kLogBlock) - start);
  const uint8_t* src = a.file + start;
  const uint32_t shift = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(src) & 15u);
  const uint32_t nbytes = shift + n;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(src - shift), 0, static_cast<int>(nbytes), kBufferDword3);
  const uint32_t lines = nbytes >> 4;
  for (uint32_t i = 0; i * 64u < lines; ++i) {
    const uint32_t line = i * 64u + lane;
    if (line < lines)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          r, (__attribute__((address_space(3))) void*)(sbuf + 1024u * i), 16, 16u * line, 0, 0, 0);
  }
  if (lane < (nbytes & 15u)) sbuf[16u * lines + lane] = (src - shift)[16u * lines + lane];
  return shift;
}

// ---- the kernel ------------------------------------------------------------

__global__ void __launch_bounds__(kVThreads, 1) log_verify_kernel(LogArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t buf[kSlots][kBufBytes];
  __shared__ __attribute__((aligned(16))) uint32_t img[kCompactLdsBytes / 4];
  __shared__ uint16_t pos[kSlots][kPosLds];
  __shared__ Slot slots[kSlots];
  __shared__ uint32_t fin;

  const uint32_t tid = threadIdx.x;
  const uint32_t lane = lane_id();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (tid < kSlots) {
    Slot& S = slots[tid];
    S.next = 0;
    S.prog = 0;
    S.lclaim = 0;
    S.lavail = 0;
    S.crcd = 0;
    S.first_bad = 0xffffffffu;
    S.nlong = 0;
    S.shift = 0;
  }
  if (tid == 0) fin = 0;
  if (tid == 0) log_stamp(a, 0, 15, 0);
  // the CRC image (build_compact_image's steps); each slot's first block is
  // assigned (workgroup g, slot m: block g * kSlots + m; the tickets count
  // the rest) and its DMA issued before the barrier, once the image's loads
  // have landed (vmcnt is in order), so no ticket round trip comes first
  uint32_t first_shift = 0;
  const uint32_t first_b = blockIdx.x * kSlots + wave;
  {
    RowTabStage<64 * kVW> rt;
    LaneTabGen<kVW> lg;
    rt.load(a.zpow, tid);
    lg.load(a.lane_cols, wave, lane);
    rt.store(img, tid);
    lg.store(img, wave, lane);
    if (wave < kSlots && first_b < a.nblocks) first_shift = dma_block(a, first_b, buf[wave], lane);
    __syncthreads();
  }
  if (tid == 0) log_stamp(a, 0, 15, 1);

  if (wave < kSlots) {
    // ---- manager of slot m ----
    const uint32_t m = wave;
    // the walk is the longest chain of the kernel: its wave issues first
    __builtin_amdgcn_s_setprio(3);
    Slot& S = slots[m];
    uint8_t* sbuf = buf[m];
    uint16_t* spos = pos[m];
    uint32_t* sover = a.over + (static_cast<uint64_t>(blockIdx.x) * kSlots + m) * kPosOver;
    uint32_t gen = 0;  // slot generation (gen 0's block is the first)
    // tickets (after the grid's first kSlots blocks a workgroup): the next
    // block's is claimed as soon as this one is in LDS, so the atomic's round
    // trip overlaps the walk
    const uint32_t tk0 = gridDim.x * kSlots;
    uint32_t tk = first_b;
    for (uint32_t k = 0;; ++k) {
      const uint32_t b = __builtin_amdgcn_readfirstlane(tk);
      if (b >= a.nblocks) break;
      log_stamp(a, m, k, 0);
      const uint64_t start = uint64_t{b} * kLogBlock;
      const uint64_t end = min(a.size, start + kLogBlock);
      const uint32_t n = static_cast<uint32_t>(end - start);
      const bool eof = n < kLogBlock;
      // the block into the slot (the first one's DMA was issued before the
      // image barrier)
      const uint32_t shift = k == 0 ? first_shift : dma_block(a, b, sbuf, lane);
      __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0): the DMA has landed
      if (lane == 0) S.shift = shift;
      if (lane == 0)
        tk = tk0 + __hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      log_stamp(a, m, k, 1);
      const uint8_t* blk = sbuf + S.shift;
      uint32_t c, stop_at;
      const uint8_t walked = walk_block(blk, n, eof, spos, sover, S, gen, &c, &stop_at, a, m, k);
      // the block's run of staging entries (the atomic's round trip overlaps
      // the CRCs: its value is first used by the staging stores)
      uint32_t off = 0;
      if (lane == 0) off = __hip_atomic_fetch_add(a.stg_top, c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      log_stamp(a, m, k, 2);
      // while the workers finish, the next block is pulled into L2 (one
      // dword per 128-byte line), so its DMA is an L2 hit
      uint32_t sink = 0;
      {
        const uint32_t nb = __builtin_amdgcn_readfirstlane(tk);
        if (nb < a.nblocks) {
          const uint64_t ns = uint64_t{nb} * kLogBlock;
#pragma unroll
          for (uint32_t i = 0; i < kLogBlock / 128u / 64u; ++i) {
            const uint64_t at = ns + 128u * (i * 64u + lane);
            if (at < a.size) sink ^= *reinterpret_cast<const uint32_t*>(a.file + (at & ~uint64_t{3}));
          }
        }
      }
      // the block's CRCs (the workers'); the merge (db/log_reader.cc:221-255)
      if (!(a.knobs & 1u))
        while (lds_load_acq(&S.crcd) < c) __builtin_amdgcn_s_sleep(1);
      asm volatile("" ::"v"(sink));
      log_stamp(a, m, k, 3);
      const uint32_t bad = S.first_bad;
      uint8_t status = walked;
      uint64_t drop = 0;
      if (bad != 0xffffffffu) {
        status = LVKV_LOGBLK_CHECKSUM;
        drop = end - (start + pos_of(spos, sover, bad));  // ReportCorruption(buffer_.size(), ...)
      } else if (status == LVKV_LOGBLK_BAD_LENGTH) {
        drop = n - stop_at;  // ReportCorruption(drop_size, "bad record length")
      }
      off = __builtin_amdgcn_readfirstlane(off);
      // the records, staged: the checksum a worker left in the header's CRC
      // bytes; those after the first mismatch were dropped with the buffer
      // (:248-255)
      for (uint32_t j = lane; j < c && off + j < a.capacity; j += 64) {
        const uint32_t p = pos_of(spos, sover, j);
        const uint32_t len =
            static_cast<uint32_t>(blk[p + 4]) | (static_cast<uint32_t>(blk[p + 5]) << 8);
        a.stg[off + j] =
            make_uint4(lds_word(blk, p), p | (len << 16), blk[p + 6],
                       j < bad ? LVKV_REC_OK : j == bad ? LVKV_REC_CHECKSUM : LVKV_REC_DROPPED);
      }
      if (lane == 0) {
        a.block_status[b] = status;
        a.block_drop[b] = static_cast<uint32_t>(drop);
        a.stg_off[b] = off;
        // what the emit launch reads (after this kernel's end: plain stores;
        // device-scope ones are acknowledged late, and the next block's DMA
        // wait, vmcnt being in order, waits for them)
        a.info[b] = make_ulonglong2(uint64_t{c} | (uint64_t{bad != 0xffffffffu ? bad : c} << 32),
                                    drop | (uint64_t{status} << 32));
      }
      log_stamp(a, m, k, 4);
      // recycle the slot: reset, then open the next generation (workers
      // claim through `next` / `lclaim` last, so they see the reset state)
      gen = (gen + 1u) & 0x7fffu;
      if (lane == 0) {
        S.crcd = 0;
        S.first_bad = 0xffffffffu;
        S.nlong = 0;
        // the words workers wait on first, the words they claim through last
        lds_store_rel(&S.lavail, gen << 16);
        lds_store_rel(&S.prog, gen << kGenShift);
        lds_store_rel(&S.lclaim, gen << 16);
        lds_store_rel(&S.next, gen << 16);
      }
    }
    // No more blocks: the slot's open generation is published as walked and
    // empty, so a worker whose claim landed in it (after the last recycle)
    // sees the walk over and drops the claim instead of waiting forever.
    if (lane == 0) {
      lds_store_rel(&S.prog, (gen << kGenShift) | kDoneBit);
      __hip_atomic_fetch_add(&fin, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  } else {
    // ---- workers: records (two per claim) and long-record segments from
    // any slot, as soon as the walker has published them. A claim is an
    // atomic add on `next` / `lclaim`; the generation it returns is the one
    // it belongs to (even if the slot was recycled since it was looked at),
    // and a claim of a generation is waited out until the walker has passed
    // it or stopped, so no record of a generation is ever skipped.
    LogLane L;
    L.keys = lane_keys(lane);
    L.lane_base = compact_lane_base(lane);
    // probe knob bits 8-11: that many worker waves sit out (timing)
    const uint32_t nidle = (a.knobs >> 8) & 15u;
    for (uint32_t idle = 0; wave < static_cast<uint32_t>(kVW) - nidle;) {
      if (a.knobs & 1u) {
        if (lds_load_acq(&fin) == kSlots) break;
        __builtin_amdgcn_s_sleep(127);
        continue;
      }
      bool worked = false;
#pragma unroll 1
      for (uint32_t si = 0; si < kSlots; ++si) {
        const uint32_t s = (wave + si) % kSlots;
        Slot& S = slots[s];
        const uint8_t* sbuf = buf[s];
        const uint32_t* sover = a.over + (static_cast<uint64_t>(blockIdx.x) * kSlots + s) * kPosOver;
        // long-record segments first: they are the long poles
        {
          const uint32_t lav = lds_load_acq(&S.lavail);
          const uint32_t lcl = lds_load_acq(&S.lclaim);
          if ((lav >> 16) == (lcl >> 16) && (lcl & 0xffffu) < (lav & 0xffffu)) {
            uint32_t x = 0;
            if (lane == 0) x = atomicAdd(&S.lclaim, 2u);
            x = __builtin_amdgcn_readfirstlane(x);
            const uint32_t g2 = x >> 16, x0 = x & 0xffffu;
            // wait until both segments are registered or the walk is over
            uint32_t av, pr;
            for (;;) {
              av = lds_load_acq(&S.lavail);
              pr = lds_load_acq(&S.prog);
              if ((av >> 16) != g2 || (pr >> kGenShift) != g2) break;
              if ((pr & kDoneBit) || (av & 0xffffu) > x0 + 1u) break;
              __builtin_amdgcn_s_sleep(1);
            }
            // a foreign generation: this one is finished, the claim was empty
            if ((av >> 16) != g2 || (pr >> kGenShift) != g2) continue;
            av = lds_load_acq(&S.lavail);  // final once the walk is over
            const uint32_t navail = av & 0xffffu;
            if (x0 < navail) {
              worked = true;
              const uint8_t* blk = sbuf + S.shift;
              const uint32_t nl = S.nlong;
              // the two segments: entry e, segment i (0 = the last) of each
              uint32_t ent[2], seg[2], at[2], len[2], inj[2], raw[2];
              bool have[2];
#pragma unroll
              for (int t = 0; t < 2; ++t) {
                const uint32_t xi = x0 + t;
                have[t] = xi < navail;
                ent[t] = 0;
                seg[t] = 0;
                if (have[t]) {
                  for (uint32_t e = 1; e < nl; ++e)
                    if (S.lfirst[e] <= xi) ent[t] = e;
                  const uint32_t e = ent[t];
                  const uint32_t p = S.lp[e];
                  const uint32_t nrec = 1u + (static_cast<uint32_t>(blk[p + 4]) |
                                              (static_cast<uint32_t>(blk[p + 5]) << 8));
                  const uint32_t m = S.lseg[e];
                  seg[t] = m - 1u - (xi - S.lfirst[e]);  // numbered from the record's end
                  const uint32_t segend = p + 6u + nrec - kSegBytes * seg[t];
                  const bool front = seg[t] == m - 1u;
                  at[t] = front ? p + 6u : segend - kSegBytes;
                  len[t] = segend - at[t];
                  inj[t] = front ? 0xffffffffu : 0u;
                } else {  // a copy of the first, computed and dropped
                  at[t] = at[0];
                  len[t] = len[0];
                  inj[t] = inj[0];
                }
              }
              // the shift operators' columns (lanes [0,32): Z_{seg0 S}, [32,64): Z_{seg1 S})
              const uint32_t myseg = lane < 32u ? seg[0] : seg[1];
              const uint32_t colv = myseg ? zmul_cols(a.zpow, kLog2Seg, myseg)[lane & 31u] : 0u;
              if (len[0] >= 4u && len[1] >= 4u) {
                lds_record_crcs<2>(blk, at, len, inj, 0u, img, L, lane, raw);
              } else {
#pragma unroll
                for (int t = 0; t < 2; ++t) {
                  if (len[t] >= 4u) {
                    const uint32_t a1[1] = {at[t]}, n1[1] = {len[t]}, i1[1] = {inj[t]};
                    uint32_t r1[1];
                    lds_record_crcs<1>(blk, a1, n1, i1, 0u, img, L, lane, r1);
                    raw[t] = r1[0];
                  } else {
                    raw[t] = tiny_reg(blk + at[t], len[t], inj[t]);
                  }
                }
              }
#pragma unroll
              for (int t = 0; t < 2; ++t) {
                if (!have[t]) continue;
                // the segment's register, shifted to the record's end
                const uint32_t sh = seg[t] ? apply_lane_cols(colv, raw[t], t, lane) : raw[t];
                if (lane == 0) {
                  const uint32_t e = ent[t];
                  atomicXor(&S.lacc[e], sh);
                  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                  if (atomicSub(&S.lrem[e], 1u) == 1u) {
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                    record_done(blk, S.lp[e], S.lacc[e] ^ 0xffffffffu, S.lj[e], S);
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                    atomicAdd(&S.crcd, 1u);
                  }
                }
              }
            }
            continue;
          }
        }
        // records
        const uint32_t nx = lds_load_acq(&S.next);
        const uint32_t prog = lds_load_acq(&S.prog);
        if ((nx >> 16) != (prog >> kGenShift)) continue;  // being recycled
        const uint32_t walked = prog & 0xffffu;
        if ((nx & 0xffffu) >= walked && ((prog & kDoneBit) || walked == 0)) continue;
        uint32_t v = 0;
        if (lane == 0) v = atomicAdd(&S.next, 2u);
        v = __builtin_amdgcn_readfirstlane(v);
        const uint32_t g2 = v >> 16, j0 = v & 0xffffu;
        // wait until the walker has passed both records or stopped
        uint32_t pr;
        for (;;) {
          pr = lds_load_acq(&S.prog);
          if ((pr >> kGenShift) != g2 || (pr & kDoneBit) || (pr & 0xffffu) > j0 + 1u) break;
          __builtin_amdgcn_s_sleep(1);
        }
        if ((pr >> kGenShift) != g2) continue;  // that generation is over: an empty claim
        const uint32_t total = pr & 0xffffu;
        if (j0 >= total) continue;
        worked = true;
        const uint8_t* blk = sbuf + S.shift;
        uint32_t pp[2], nn[2], at[2], len[2], crc[2];
        bool valid[2], rows_ok[2];
        int lead = -1;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const uint32_t j = j0 + t;
          pp[t] = 0;
          nn[t] = 0;
          valid[t] = false;
          if (j < total) {
            pp[t] = pos_of(pos[s], sover, j);
            nn[t] = 1u + (static_cast<uint32_t>(blk[pp[t] + 4]) |
                          (static_cast<uint32_t>(blk[pp[t] + 5]) << 8));
            valid[t] = nn[t] <= kSegBytes;  // long ones: the segment path
          }
          rows_ok[t] = valid[t] && nn[t] >= 4u;
          if (rows_ok[t] && lead < 0) lead = t;
        }
        if (lead >= 0) {
          // a record that is absent or tiny is replaced by the first real one
          const uint32_t inj[2] = {0xffffffffu, 0xffffffffu};
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            at[t] = rows_ok[t] ? pp[t] + 6 : pp[lead] + 6;
            len[t] = rows_ok[t] ? nn[t] : nn[lead];
          }
          lds_record_crcs<2>(blk, at, len, inj, 0xffffffffu, img, L, lane, crc);
        }
#pragma unroll
        for (int t = 0; t < 2; ++t)
          if (valid[t] && !rows_ok[t])
            crc[t] = tiny_reg(blk + pp[t] + 6, nn[t], 0xffffffffu) ^ 0xffffffffu;
        if (lane == 0) {
          uint32_t ndone = 0;
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            if (!valid[t]) continue;
            record_done(blk, pp[t], crc[t], j0 + t, S);
            ++ndone;
          }
          if (ndone) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            atomicAdd(&S.crcd, ndone);
          }
        }
      }
      if (worked) {
        idle = 0;
        continue;
      }
      if (lds_load_acq(&fin) == kSlots) break;
      if (idle < 8)
        __builtin_amdgcn_s_sleep(1);
      else
        __builtin_amdgcn_s_sleep(4);
      ++idle;
    }
  }

  if (tid == 0) log_stamp(a, 0, 15, 2);
  // Nothing more: the block counts' scan into file order and the report are
  // the emit launch's (every workgroup scans the counts before its blocks),
  // so no workgroup here waits for the last one to finish.
}

constexpr uint32_t kEmitWaves = 16;  // blocks per emit workgroup (one wave each)
// Past this many blocks the emit workgroups no longer sum every count before
// their own (a quadratic total): log_scan_kernel scans them first.
constexpr uint32_t kEmitFoldMax = 4096;
constexpr uint32_t kScanThreads = 1024;

// first_of[b] = the records of the blocks before b, first_of[nblocks] = all
// of them. One workgroup; each thread a contiguous run of blocks.
__global__ void __launch_bounds__(kScanThreads) log_scan_kernel(LogArgs a) {
  __shared__ unsigned long long wtot[kScanThreads / 64];
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = lane_id(), wave = tid >> 6;
  const uint32_t n = a.nblocks;
  const uint32_t per = (n + kScanThreads - 1) / kScanThreads;
  const uint32_t b0 = min(n, tid * per), b1 = min(n, b0 + per);
  unsigned long long mine = 0;
  for (uint32_t b = b0; b < b1; ++b) mine += static_cast<uint32_t>(a.info[b].x);
  const unsigned long long inc = wave_scan_dpp<unsigned long long>(mine, lane);
  if (lane == 63) wtot[wave] = inc;
  __syncthreads();
  unsigned long long run = inc - mine;
  for (uint32_t v = 0; v < wave; ++v) run += wtot[v];
  for (uint32_t b = b0; b < b1; ++b) {
    a.first_of[b] = run;
    run += static_cast<uint32_t>(a.info[b].x);
  }
  if (tid == kScanThreads - 1) a.first_of[n] = run;
}

// The staged results to their places, one wave per block: record j of block
// b is record first[b] + j in file order, first[b] = the counts of the
// blocks before b (each workgroup sums them: 2 loads a thread for a 66 MB
// log, all workgroups at once, instead of one workgroup scanning after the
// verify's last one finished); the block's ReadRecord event follows its
// records (item first[b] + counts[b] + b, lvkv_log_events.h). The last
// workgroup also sums everything into the report; workgroup 0 leaves the
// verify's counters at 0 for the next call (the verify has ended: stream
// order).
__global__ void __launch_bounds__(64 * kEmitWaves) log_emit_kernel(LogArgs a) {
  __shared__ unsigned long long s_cnt[kEmitWaves], s_good[kEmitWaves], s_drop[kEmitWaves];
  __shared__ uint32_t s_corrupt[kEmitWaves], s_first[kEmitWaves];
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = lane_id();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t b0 = blockIdx.x * kEmitWaves;
  const bool last = blockIdx.x + 1 == gridDim.x;
  if (blockIdx.x == 0 && tid == 0) {
    *a.ticket = 0;
    *a.stg_top = 0;
  }
  // counts before b0 (and, in the last workgroup, every block's totals);
  // scanned already when there are many blocks
  const bool scanned = a.first_of != nullptr;
  const uint32_t upto = last ? a.nblocks : scanned ? 0u : min(b0, a.nblocks);
  unsigned long long cnt = 0, good = 0, drop = 0;
  uint32_t corrupt = 0, fb = 0xffffffffu;
  for (uint32_t b = tid; b < upto; b += 64 * kEmitWaves) {
    const ulonglong2 v = a.info[b];
    const uint32_t c = static_cast<uint32_t>(v.x);
    if (b < b0) cnt += c;
    if (last) {
      const uint32_t st = static_cast<uint32_t>(v.y >> 32);
      good += v.x >> 32;
      if (st == LVKV_LOGBLK_CHECKSUM || st == LVKV_LOGBLK_BAD_LENGTH) {
        ++corrupt;
        drop += static_cast<uint32_t>(v.y);
        fb = min(fb, b);
      }
      if (b >= b0) cnt += uint64_t{c} << 32;  // this workgroup's own blocks, kept apart
    }
  }
  cnt = wave_sum_dpp(cnt);
  good = wave_sum_dpp(good);
  drop = wave_sum_dpp(drop);
  corrupt = wave_sum_dpp(corrupt);
  fb = wave_min_dpp(fb);
  if (lane == 0) {
    s_cnt[wave] = cnt;
    s_good[wave] = good;
    s_drop[wave] = drop;
    s_corrupt[wave] = corrupt;
    s_first[wave] = fb;
  }
  __syncthreads();
  unsigned long long before = 0, mine_all = 0;
#pragma unroll
  for (uint32_t w = 0; w < kEmitWaves; ++w) {
    before += s_cnt[w] & 0xffffffffull;
    mine_all += s_cnt[w] >> 32;
  }
  if (scanned && !last) before = a.first_of[b0];
  // (a count is at most kMaxRecs and a log at most 2^32 records: the low
  // halves do not carry into the high ones)
  if (last && tid == 0) {
    unsigned long long g = 0, d = 0;
    uint32_t nc = 0, f = 0xffffffffu;
#pragma unroll
    for (uint32_t w = 0; w < kEmitWaves; ++w) {
      g += s_good[w];
      d += s_drop[w];
      nc += s_corrupt[w];
      f = min(f, s_first[w]);
    }
    const uint64_t total = before + mine_all;
    lvkv_log_report* r = a.r;
    r->status = total > a.capacity ? LVKV_LOG_CAPACITY : LVKV_OK;
    r->nblocks = a.nblocks;
    r->nrecords = static_cast<uint32_t>(total);
    r->ngood = static_cast<uint32_t>(g);
    r->ncorrupt = nc;
    r->first_bad_block = f;
    r->dropped_bytes = d;
    r->count_ = total > a.capacity ? 0u : static_cast<uint32_t>(total);
    r->reserved_ = 0;
  }
  const uint32_t b = b0 + wave;
  if (b >= a.nblocks) return;
  // this wave's place: the counts of the workgroup's blocks before it
  const uint32_t pre = wave_sum_dpp(lane < wave ? static_cast<uint32_t>(a.info[b0 + lane].x) : 0u);
  const uint64_t base = before + pre;
  const uint32_t c = static_cast<uint32_t>(a.info[b].x), off = a.stg_off[b];
  const uint64_t start = uint64_t{b} * kLogBlock;
  for (uint32_t j = lane; j < c; j += 64) {
    const uint64_t gi = base + j;
    if (gi >= a.capacity || off + j >= a.capacity) break;
    const uint4 e = a.stg[off + j];
    const uint64_t ho = start + (e.y & 0xffffu);
    a.hdr_off[gi] = ho;
    a.actual[gi] = e.x;
    a.rec_status[gi] = static_cast<uint8_t>(e.w);
    if (a.events != nullptr) {
      a.events[gi + b] = e.w == LVKV_REC_OK ? log_event(kEvRec, e.z, e.y >> 16)
                                             : log_event(kEvSkip, 0, 0);
      a.item_off[gi + b] = ho;
    }
  }
  if (lane == 0 && a.events != nullptr && base + c <= a.capacity)
    a.events[base + c + b] = log_block_event(a.block_status[b], a.block_drop[b]);
}

// Scratch: [0, 8) unused, [8, 16) the logical layer's counter (not touched
// here), [16, 20) ticket counter, [20, 24) staging counter, then from byte
// 32 info (16 B per block), stg_off (u32 per block) and 4 unused bytes per
// block, first_of (u64 per block, and one), the staging array (16 B per
// record, `capacity` of them) and the slots' overflow positions (u32,
// kPosOver per slot of each of the grid's workgroups).
size_t log_scratch_head(uint64_t nblocks) {
  return (32 + static_cast<size_t>(nblocks) * 32 + 8 + 15) & ~size_t{15};
}

// One workgroup per CU at most (each takes most of a CU's LDS); blocks are
// claimed by ticket, so the grid need not be resident all at once.
uint32_t log_groups(uint64_t nblocks, int cus) {
  return static_cast<uint32_t>(std::max<uint64_t>(
      1, std::min<uint64_t>((nblocks + kSlots - 1) / kSlots, static_cast<uint64_t>(cus))));
}

}  // namespace

#ifdef LVKV_PROBE_BUILD
uint64_t* g_log_stamps = nullptr;  // lvkv_debug_log_stamps
uint32_t g_log_knobs = 0;          // lvkv_debug_log_knobs (LogArgs::knobs)
#endif

size_t log_scratch_bytes(uint64_t size, uint32_t capacity, int cus) {
  const uint64_t nblocks = (size + kLogBlock - 1) / kLogBlock;
  return log_scratch_head(nblocks) + size_t{capacity} * 16 +
         size_t{log_groups(nblocks, cus)} * kSlots * kPosOver * 4;
}

hipError_t launch_log_blocks(const uint8_t* file, uint64_t size, uint64_t* hdr_off,
                             uint32_t* actual, uint8_t* rec_status, uint32_t capacity,
                             uint8_t* block_status, uint32_t* block_drop, lvkv_log_report* r,
                             const uint32_t* zpow, const uint32_t* lane_cols, int cus,
                             void* scratch, uint32_t* events, uint64_t* item_off,
                             hipStream_t stream) {
  const uint32_t nblocks = static_cast<uint32_t>((size + kLogBlock - 1) / kLogBlock);
  LogArgs a;
  memset(&a, 0, sizeof(a));
  a.file = file;
  a.size = size;
  a.nblocks = nblocks;
  a.capacity = capacity;
  a.hdr_off = hdr_off;
  a.actual = actual;
  a.rec_status = rec_status;
  a.block_status = block_status;
  a.block_drop = block_drop;
  a.r = r;
  uint8_t* sb = static_cast<uint8_t*>(scratch);
  a.ticket = reinterpret_cast<uint32_t*>(sb + 16);
  a.stg_top = reinterpret_cast<uint32_t*>(sb + 20);
  a.info = reinterpret_cast<ulonglong2*>(sb + 32);
  a.stg_off = reinterpret_cast<uint32_t*>(a.info + nblocks);
  a.first_of = nblocks > kEmitFoldMax
                   ? reinterpret_cast<unsigned long long*>(sb + 32 + size_t{nblocks} * 24)
                   : nullptr;
  a.stg = reinterpret_cast<uint4*>(sb + log_scratch_head(nblocks));
  a.over = reinterpret_cast<uint32_t*>(a.stg + capacity);
  a.zpow = zpow;
  a.lane_cols = lane_cols;
  a.events = events;
  a.item_off = item_off;
#ifdef LVKV_PROBE_BUILD
  a.stamps = g_log_stamps;
  a.knobs = g_log_knobs;
#endif
  if (nblocks != 0) {
    hipLaunchKernelGGL(log_verify_kernel, dim3(log_groups(nblocks, cus)), dim3(kVThreads), 0,
                       stream, a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  if (a.first_of != nullptr) {
    hipLaunchKernelGGL(log_scan_kernel, dim3(1), dim3(kScanThreads), 0, stream, a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(log_emit_kernel, dim3(std::max<uint32_t>(1, (nblocks + kEmitWaves - 1) / kEmitWaves)),
                     dim3(64 * kEmitWaves), 0, stream, a);
  return hipGetLastError();
}

}  // namespace lvkv
