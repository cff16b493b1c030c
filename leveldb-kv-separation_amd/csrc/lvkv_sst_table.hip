// Whole-SSTable verify on the device, for one table or
// many at once, as TWO launches on one stream whatever the number of tables,
// with no host round trip:
//
//   1. sst_table_kernel     one 1024-thread workgroup per table does what
//                           Table::Open + Table::ReadMeta + the index walk do
//                           (table/table.cc:38-124, table/format.cc:24-160,
//                           table/block.cc:25-75), in LDS where it can:
//                             * the footer (format.cc:43-67): size, magic, the
//                               two BlockHandles, the short-read test;
//                             * the index and metaindex CRCs (contents + type
//                               byte against the stored trailer), 1 KiB
//                               segments over the 16 waves (workgroup_crc);
//                             * the verdicts in ReadBlock's order (short read,
//                               checksum, type byte), Block::Block's restart
//                               array test;
//                             * ReadMeta's exact Seek("filter." + policy name)
//                               over the metaindex staged in LDS;
//                             * its place in the shared per-block arrays: the
//                               entry count of every earlier table (published
//                               by their workgroups, agent-scope 8-byte
//                               atomics, tagged with the call's generation so
//                               no clearing pass is needed);
//                             * every index entry (the index staged in LDS
//                               when it fits): the index is written with
//                               block_restart_interval = 1 (table_builder.cc:35,
//                               :90), so restart point i IS entry i and the
//                               1024 threads decode entries in parallel
//                               (DecodeEntry, block.cc:55-75; BlockHandle
//                               varints, format.cc:24-30).
//   2. crc32c_ragged_kernel SST-table mode over all entries (count read on the
//                           device): the CRC, then stored trailer vs computed
//                           CRC, type byte and parse status -> LVKV_BLOCK_*,
//                           per-table nbad / first_bad (format.cc:92-158).
//
// Bounds: every byte the kernels touch is inside its table image: handles are
// range-checked (in an order that cannot overflow) before anything is read
// through them; a bad one becomes 0/0 with a non-zero status; varints are
// decoded against explicit limits.
//
// BlockHandle sizes near 2^64: ReadBlock computes n + kBlockTrailerSize in
// size_t (format.cc:77-80), so n = 2^64 - 1 reads 4 bytes, passes the
// short-read test and compares Unmask(those 4 bytes) with the CRC of zero
// bytes (0): "block checksum mismatch" (pinned by tests/golden/damage_sst.json
// footer_*_size_max). This path gives the same verdict. n in [2^64-5, 2^64-2]
// makes the reference read before its buffer (undefined); this path reports
// "truncated block read" there.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_compact_common.h"
#include "crc32c_device_common.h"
#include "crc32c_ragged_body.h"
#include "lvkv_crc32c.h"
#include "lvkv_kernel_args.h"

namespace lvkv {

namespace {

constexpr uint64_t kTableMagic = 0xdb4775248b80fb57ull;  // table/format.h:76
constexpr uint64_t kFooterLen = 48;  // table/format.h:53 (2 * 20 + 8)
constexpr uint64_t kTrailer = 5;     // table/format.h:79
constexpr uint32_t kMetaStage = 2048;                // metaindex staged in LDS up to this
constexpr uint32_t kIndexStage = kCompactLdsBytes;   // index staged in the (spent) image
// One-table calls leave an index (contents + type) in this range to
// sst_index_kernel: larger than what the head stages in LDS, and at most 256
// of its largest chunks (kWideChunkMaxLog2).
constexpr uint32_t kWideGroups = 64, kWideWaves = 8;
constexpr uint32_t kWideChunkMinLog2 = 13, kWideChunkMaxLog2 = 19;
constexpr uint64_t kWideIndexMin = kIndexStage;
constexpr uint64_t kWideIndexMax = uint64_t{256} << kWideChunkMaxLog2;

struct Table {  // one image of the batch
  const uint8_t* img;
  uint64_t base;  // offset of the image in d_file
  uint64_t size;
};

__device__ __forceinline__ Table table_of(const uint8_t* file, const uint64_t* toff,
                                          const uint64_t* tsize, uint64_t single_size,
                                          uint32_t t) {
  Table x;
  x.base = toff != nullptr ? toff[t] : 0;
  x.size = tsize != nullptr ? tsize[t] : single_size;
  x.img = file + x.base;
  return x;
}

__device__ __forceinline__ uint32_t ld_le32(const uint8_t* p) {
  return static_cast<uint32_t>(p[0]) | (static_cast<uint32_t>(p[1]) << 8) |
         (static_cast<uint32_t>(p[2]) << 16) | (static_cast<uint32_t>(p[3]) << 24);
}

// GetVarint64Ptr / GetVarint32Ptr (util/coding.cc): bytes consumed, 0 on
// failure (runs past `limit` or longer than the type allows).
__device__ __forceinline__ uint32_t get_varint(const uint8_t* p, const uint8_t* limit, uint32_t max_shift,
                               uint64_t* v) {
  uint64_t result = 0;
  uint32_t i = 0;
  for (uint32_t shift = 0; shift <= max_shift && p + i < limit; shift += 7, ++i) {
    const uint64_t b = p[i];
    if (b & 128) {
      result |= (b & 127) << shift;
    } else {
      *v = result | (b << shift);
      return i + 1;
    }
  }
  return 0;
}

// BlockHandle::DecodeFrom over [p, limit): true and (off, size) on success.
__device__ __forceinline__ bool decode_handle(const uint8_t* p, const uint8_t* limit, uint64_t* off,
                              uint64_t* size, const uint8_t** next) {
  const uint32_t n1 = get_varint(p, limit, 63, off);
  if (n1 == 0) return false;
  const uint32_t n2 = get_varint(p + n1, limit, 63, size);
  if (n2 == 0) return false;
  if (next) *next = p + n1 + n2;
  return true;
}

// ReadBlock's read of size + kBlockTrailerSize bytes at off (format.cc:76-87)
// against an image of file_size bytes, without overflow: kFitOk when block
// and trailer are inside the image (and n + 1 < 4 GiB, the CRC kernels'
// length type), kFitWrap for n = 2^64 - 1 with 4 bytes readable (see the
// header comment), else kFitShort ("truncated block read").
enum Fit : uint32_t { kFitOk, kFitShort, kFitWrap };

__device__ __forceinline__ Fit handle_fit(uint64_t off, uint64_t size, uint64_t file_size) {
  if (off > file_size) return kFitShort;
  const uint64_t avail = file_size - off;
  if (size == ~uint64_t{0}) return avail >= 4 ? kFitWrap : kFitShort;
  if (size > 0xfffffffeull || avail < kTrailer || avail - kTrailer < size) return kFitShort;
  return kFitOk;
}

// LVKV_BLOCK_* of a block that is not kFitOk.
__device__ __forceinline__ uint8_t unfit_status(const uint8_t* img, Fit f, uint64_t off) {
  if (f == kFitWrap && crc_unmask(ld_le32(img + off)) != 0u) return LVKV_BLOCK_CHECKSUM;
  return LVKV_BLOCK_TRUNCATED;  // also kFitWrap whose dword unmasks to 0 (see header)
}

// ReadBlock's verdict for a kFitOk block from its CRC test and type byte.
__device__ __forceinline__ uint8_t read_status(bool crc_ok, uint8_t type) {
  if (!crc_ok) return LVKV_BLOCK_CHECKSUM;
  if (type == 1 || type == 2) return LVKV_BLOCK_COMPRESSED;  // no codec as built
  if (type > 2) return LVKV_BLOCK_BAD_TYPE;
  return LVKV_BLOCK_OK;
}

// DecodeEntry (table/block.cc:55-75): pointer to the key delta or nullptr.
__device__ __forceinline__ const uint8_t* decode_entry(const uint8_t* p, const uint8_t* limit, uint32_t* shared,
                                       uint32_t* non_shared, uint32_t* value_len) {
  if (limit - p < 3) return nullptr;
  uint64_t v;
  uint32_t n;
  if ((n = get_varint(p, limit, 28, &v)) == 0) return nullptr;
  *shared = static_cast<uint32_t>(v);
  p += n;
  if ((n = get_varint(p, limit, 28, &v)) == 0) return nullptr;
  *non_shared = static_cast<uint32_t>(v);
  p += n;
  if ((n = get_varint(p, limit, 28, &v)) == 0) return nullptr;
  *value_len = static_cast<uint32_t>(v);
  p += n;
  if (static_cast<uint64_t>(limit - p) < static_cast<uint64_t>(*non_shared) + *value_len)
    return nullptr;
  return p;
}

// Everything the table's workgroup shares, in LDS.
struct Head {
  int32_t status;
  uint64_t mo, ms, io, is;
  uint32_t ifit, mfit;
  uint8_t index_status, meta_status, itype, mtype;
  uint32_t nr;          // index restart count = data blocks
  uint32_t has_filter;
  uint64_t fo, fs;      // filter handle
  uint8_t filter_status;
  uint32_t nb;          // entries this table contributes
  uint32_t first;
  uint32_t icrc, mcrc;
};

// Footer::DecodeFrom (format.cc:43-67) on the 48 staged footer bytes.
__device__ __forceinline__ void parse_footer(Head& h, const uint8_t* f, uint64_t size) {
  h.status = LVKV_SST_OK;
  h.mo = h.ms = h.io = h.is = 0;
  h.ifit = h.mfit = kFitShort;
  h.index_status = h.meta_status = LVKV_BLOCK_NOT_READ;
  h.itype = h.mtype = 0;
  h.nr = 0;
  h.has_filter = 0;
  h.fo = h.fs = 0;
  h.filter_status = LVKV_BLOCK_OK;
  h.nb = h.first = 0;
  h.icrc = h.mcrc = 0;
  if (size < kFooterLen) {  // table/table.cc:40-42
    h.status = LVKV_SST_TOO_SHORT;
    return;
  }
  const uint64_t magic = static_cast<uint64_t>(ld_le32(f + 40)) |
                         (static_cast<uint64_t>(ld_le32(f + 44)) << 32);
  if (magic != kTableMagic) {  // format.cc:48-55
    h.status = LVKV_SST_BAD_MAGIC;
    return;
  }
  const uint8_t* p = nullptr;
  if (!decode_handle(f, f + kFooterLen, &h.mo, &h.ms, &p) ||
      !decode_handle(p, f + kFooterLen, &h.io, &h.is, nullptr)) {  // format.cc:58-61
    h.status = LVKV_SST_BAD_HANDLE;
    return;
  }
  h.ifit = handle_fit(h.io, h.is, size);
  h.mfit = handle_fit(h.mo, h.ms, size);
}

// Table::ReadMeta's Seek("filter." + name) and exact key test (table.cc:95-102)
// over the staged metaindex m[0, msize) (kNoCompression, CRC verified): a
// linear walk keeping the length of the common prefix of the current key and
// the target, so no key buffer is needed. Sets the filter handle on a match.
// One wave: entries are decoded lane-uniformly; each key's bytes are
// compared 64 at a time, one lane per byte (a ballot gives the prefix).
__device__ __forceinline__ void find_filter(Head& h, const uint8_t* m, uint64_t msize, const uint8_t* key,
                            uint32_t key_len, const Table& tb, uint32_t lane) {
  if (lane == 0) h.has_filter = 0;
  if (key_len == 0 || msize < 4) return;
  const uint32_t nr = ld_le32(m + msize - 4);
  if (nr > (msize - 4) / 4) return;
  const uint8_t* limit = m + (msize - (1 + static_cast<uint64_t>(nr)) * 4);
  uint32_t lcp = 0, klen = 0;
  const uint8_t* p = m;
  while (p < limit) {
    uint32_t sh, ns, vl;
    const uint8_t* q = decode_entry(p, limit, &sh, &ns, &vl);
    if (q == nullptr || sh > klen) return;  // Block::Iter: "bad entry in block"
    uint32_t l = min(sh, lcp);
    if (l == sh) {
      // leading bytes of q[0, ns) equal to key[sh, key_len)
      for (uint32_t i0 = 0; i0 < ns && sh + i0 < key_len; i0 += 64) {
        const uint32_t i = i0 + lane;
        const bool eq = i < ns && sh + i < key_len && q[i] == key[sh + i];
        const uint64_t miss = ~__ballot(eq);
        const uint32_t run = miss ? static_cast<uint32_t>(__builtin_ctzll(miss)) : 64u;
        l = sh + i0 + run;
        if (run < 64) break;
      }
    }
    lcp = l;
    klen = sh + ns;
    if (klen == key_len && lcp == key_len) {
      uint64_t fo, fsz;
      if (!decode_handle(q + ns, q + ns + vl, &fo, &fsz, nullptr)) return;  // ReadFilter: ignored
      const Fit f = handle_fit(fo, fsz, tb.size);
      if (lane == 0) {
        h.fo = f == kFitOk ? fo : 0;
        h.fs = f == kFitOk ? fsz : 0;
        h.filter_status = f == kFitOk ? LVKV_BLOCK_OK : unfit_status(tb.img, f, fo);
        h.has_filter = 1;
      }
      return;
    }
    p = q + ns + vl;
  }
}

// Wave 0 of table t's workgroup: first = sum of the entry counts published by
// tables 0..t-1 (spin until each carries this call's generation). Table
// workgroups are dispatched in order, so every table waited on is resident or
// done. The last table also derives the launch's entry total: entries up to
// the first table that does not fit in `capacity`.
__device__ uint32_t place_table(lvkv_sst_report* reports, uint32_t t, uint32_t ntables,
                                uint32_t gen, uint32_t nb, uint32_t capacity, uint32_t lane,
                                uint32_t* total) {
  const uint64_t mine = (static_cast<uint64_t>(gen) << 32) | nb;
  if (lane == 0)
    __hip_atomic_store(&reports[t].link_, mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  uint64_t run = 0;  // inclusive prefix so far (u64: no wrap)
  uint64_t cut = ~uint64_t{0};
  const uint32_t upto = (t == ntables - 1) ? ntables : t;
  for (uint32_t b = 0; b < upto; b += 64) {
    const uint32_t j = b + lane;
    uint64_t v = 0;
    if (j < upto) {
      uint64_t x;
      // tag and count travel in one 64-bit atomic word: nothing else is read
      // on the strength of it, so no acquire is needed
      do {
        x = __hip_atomic_load(&reports[j].link_, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } while (static_cast<uint32_t>(x >> 32) != gen);
      v = x & 0xffffffffull;
    }
    // inclusive prefix over the 64 lanes
    const uint64_t inc = wave_scan_dpp<uint64_t>(v, lane);
    const uint64_t p = run + inc;
    // first table (in order) whose end passes the capacity: the total stops
    // at its start
    const uint64_t start = p - v;
    const bool over = j < upto && v != 0 && p > capacity;
    const uint64_t mask = __ballot(over);
    if (mask != 0 && cut == ~uint64_t{0}) {
      const uint32_t src = static_cast<uint32_t>(__builtin_ctzll(mask));
      cut = lane_u64(start, src);
    }
    run = lane_u64(p, 63);
  }
  if (t == ntables - 1) {
    *total = static_cast<uint32_t>(min<uint64_t>(run, min<uint64_t>(cut, capacity)));
    // `run` included this table: its own start is run - nb
    return static_cast<uint32_t>(min<uint64_t>(run - nb, capacity));
  }
  return static_cast<uint32_t>(min<uint64_t>(run, capacity));
}

struct Entry {
  uint64_t off, size;  // the handle (0/0 unless st is LVKV_BLOCK_OK)
  uint8_t st;          // LVKV_BLOCK_* of the parse
};

// The index entry at restart offset rs, ending at `end` (the next restart
// offset, or ro for the last): its data block handle and parse status. The
// entry bytes are read from `w` (a copy of index bytes [wlo, whi)) when they
// lie inside it, else from the index `idx` itself; `ro` is the restart
// array's offset.
__device__ __forceinline__ Entry decode_index_entry(const uint8_t* idx, uint64_t ro, uint32_t rs,
                                                    uint64_t end, const uint8_t* w, uint64_t wlo,
                                                    uint64_t whi, const Table& tb) {
  uint8_t st = LVKV_BLOCK_BAD_ENTRY;
  uint64_t off = 0, size = 0;
  if (rs < ro && end <= ro) {
    // DecodeEntry's limit is the restart array (block.cc:55-75, :181-195)
    // (pointers formed only inside their buffer: no out-of-range base)
    const bool in = rs >= wlo && end <= whi && rs <= end;
    const uint8_t* p = in ? w + (rs - wlo) : idx + rs;
    const uint8_t* pe = in ? w + (end - wlo) : idx + end;
    const uint8_t* limit = in ? w + (whi - wlo) : idx + ro;
    uint32_t sh, ns, vl;
    const uint8_t* q = decode_entry(p, limit, &sh, &ns, &vl);
    if (q != nullptr && sh == 0 && q + ns + vl == pe) {
      uint64_t ho, hs;
      if (!decode_handle(q + ns, q + ns + vl, &ho, &hs, nullptr)) {
        st = LVKV_BLOCK_BAD_HANDLE;
      } else {
        const Fit f = handle_fit(ho, hs, tb.size);
        if (f == kFitOk) {
          st = LVKV_BLOCK_OK;
          off = ho;
          size = hs;
        } else {
          st = unfit_status(tb.img, f, ho);
        }
      }
    }
  }
  if (st != LVKV_BLOCK_OK) off = size = 0;
  return Entry{off, size, st};
}

// Index entry i (restart point i, block_restart_interval = 1) -> its handle
// and status in the shared arrays at first + i.
__device__ __forceinline__ void emit_entry(const uint8_t* idx, uint64_t ro, uint64_t nr, uint32_t i,
                           const uint8_t* w, uint64_t wlo, uint64_t whi, const Table& tb,
                           uint32_t first, uint64_t* out_off, uint32_t* out_size,
                           uint8_t* out_status) {
  const uint32_t rs = ld_le32(idx + ro + 4ull * i);
  const uint64_t end = i + 1 < nr ? ld_le32(idx + ro + 4ull * (i + 1)) : ro;
  const Entry x = decode_index_entry(idx, ro, rs, end, w, wlo, whi, tb);
  const uint32_t e = first + i;
  out_off[e] = tb.base + x.off;  // into d_file
  out_size[e] = static_cast<uint32_t>(x.size);
  out_status[e] = x.st;
}

// What a table's workgroup keeps in LDS after the 64 KiB CRC image.
constexpr uint32_t kFilterKeyWords = (kMaxFilterKey + 4) / 4;

struct SstHeadLds {
  uint32_t acc[16];  // per-wave CRC shares
  uint32_t ftail, ftrail, ftype;  // the filter block's last bytes (speculative form)
  uint32_t fkey[kFilterKeyWords];  // the metaindex key sought, from the kernel argument
  uint8_t foot[kFooterLen];
  uint8_t mbuf[kMetaStage];
  Head h;
  uint64_t win_lo, win_hi;
};

// Probe build: phase timestamps (s_memrealtime, 100 MHz) of table t's head
// and of the first CRC workgroup, 16 u64 per table (tools/probe/sst_probe.py).
__device__ __forceinline__ void sst_stamp(uint64_t* stamps, uint32_t t, int slot) {
#ifdef LVKV_PROBE_BUILD
  if (stamps != nullptr && threadIdx.x == 0) stamps[t * 16u + slot] = __builtin_amdgcn_s_memrealtime();
#endif
}

// Index bytes prefetched into registers during the CRCs, per thread: an
// index of up to 64 W * kIndexPf dwords is staged from these, without a
// memory round trip after its checksum.
constexpr int kIndexPf = 6;

// Table t's head with W waves (Table::Open + ReadMeta + the index walk):
// footer; index and metaindex CRCs at once (index on waves [0, wi),
// metaindex on [wi, W), shifts as constant operators, group_crc_part), with
// every byte the verdicts need (type bytes, trailers, restart count, the
// 0-3 bytes after the last 4-byte boundary), the metaindex and a small index
// loaded before the walks; verdicts in ReadBlock's order; the filter key;
// the table's place; every entry's handle and status into the shared arrays.
// `lds`: the compact image followed by SstHeadLds.
template <int W>
__device__ __forceinline__ void sst_head(uint32_t* lds, const uint8_t* file, const uint64_t* toff,
                         const uint64_t* tsize, uint64_t single_size, uint32_t t,
                         uint32_t ntables, uint32_t capacity, uint32_t gen, const FilterKey& fk,
                         lvkv_sst_report* reports, uint64_t* out_off, uint32_t* out_size,
                         uint8_t* out_status, const uint32_t* zpow, const uint32_t* lane_cols,
                         uint64_t* stamps, bool wide, uint32_t* spec_crc = nullptr) {
  constexpr uint32_t kT = 64 * W;
  // spec_crc set: the speculative form (sst_spec_kernel). The data entries
  // are decoded and checksummed by the CRC workgroups; the head checksums the
  // filter block itself (beside the placement) and writes its whole entry.
  const bool spec = spec_crc != nullptr;
  SstHeadLds& L = *reinterpret_cast<SstHeadLds*>(lds + kCompactLdsBytes / 4);
  Head& h = L.h;
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = lane_id();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const Table tb = table_of(file, toff, tsize, single_size, t);
  lvkv_sst_report* r = reports + t;

  sst_stamp(stamps, t, 0);
  // 1. Footer bytes (48 lanes) while the workgroup builds its LDS image;
  //    the filter key into LDS (constant word indices: the kernel argument
  //    is read with scalar loads, never copied to scratch for a byte walk).
  if (tid < kFooterLen && tb.size >= kFooterLen) L.foot[tid] = tb.img[tb.size - kFooterLen + tid];
  {
    const uint32_t* kw = reinterpret_cast<const uint32_t*>(fk.key);
#pragma unroll
    for (uint32_t w = 0; w < kFilterKeyWords; ++w)
      if (tid == 64u + w) L.fkey[w] = kw[w];
  }
  // the table's last 32 KiB (where the index and metaindex usually sit)
  // pulled towards the CUs beside the footer: the CRC phase's loads then hit
  // the cache. The values are only "used" by an empty asm after the footer.
  uint32_t warm = 0;
  {
    const uint64_t span = min<uint64_t>(tb.size, uint64_t{32} * 1024) & ~uint64_t{63};
    const uint64_t at = tb.size - span;
    if (64u * tid < span) warm = *reinterpret_cast<const uint32_t*>(tb.img + ((at + 64u * tid) & ~uint64_t{3}));
  }
  build_compact_image<W>(lds, zpow, lane_cols, tid, wave, lane);  // ends with a barrier
  if (tid == 0) parse_footer(h, L.foot, tb.size);
  __syncthreads();
  asm volatile("" ::"v"(warm));
  const bool footer_ok = h.status == LVKV_SST_OK;  // workgroup-uniform from here on
  sst_stamp(stamps, t, 1);
  const bool ifit = footer_ok && h.ifit == kFitOk;
  const bool mfit = footer_ok && h.mfit == kFitOk;
  const uint64_t istart = reinterpret_cast<uint64_t>(tb.img) + h.io, iend = istart + h.is + 1;
  const uint64_t mstart = reinterpret_cast<uint64_t>(tb.img) + h.mo, mend = mstart + h.ms + 1;
  // A large index of a one-table call is left to sst_index_kernel (its CRC
  // cut over the grid, its entries decoded by every thread of it): here only
  // its type byte and restart array, provisionally.
  const bool defer = wide && ifit && h.is + 1 > kWideIndexMin && h.is + 1 <= kWideIndexMax;

  // 2. Loads whose values are used after the CRCs, issued before them.
  uint32_t itype = 0, itrail = 0, inr = 0xffffffffu, itail = 0, mtype = 0, mtrail = 0, mtail = 0;
  if (tid == 0) {
    if (ifit) {
      const uint8_t* e = tb.img + h.io + h.is;
      itype = e[0];
      itrail = ld_le32(e + 1);
      if (h.is >= 4) inr = ld_le32(e - 4);
      itail = group_crc_tail(istart, iend);
    }
    if (mfit) {
      const uint8_t* e = tb.img + h.mo + h.ms;
      mtype = e[0];
      mtrail = ld_le32(e + 1);
      mtail = group_crc_tail(mstart, mend);
    }
  }
  // a small index, as the aligned dwords holding it (the dword before it
  // only when that is inside the image)
  const uint64_t ia4 = istart & ~uint64_t{3};
  const uint32_t ind = static_cast<uint32_t>((istart + h.is + 3 - ia4) >> 2);
  const bool ipf = !spec && ifit && ind <= kT * kIndexPf && ia4 >= reinterpret_cast<uint64_t>(tb.img);
  uint32_t pf[kIndexPf];
  if (ipf) {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(ia4);
#pragma unroll
    for (int k = 0; k < kIndexPf; ++k) {
      const uint32_t i = tid + kT * static_cast<uint32_t>(k);
      pf[k] = i < ind ? src[i] : 0u;
    }
  }

  // 3. Index and metaindex CRCs (contents + type byte) side by side.
  const LaneKeys keys = lane_keys(lane);
  const uint32_t lane_base = compact_lane_base(lane);
  const uint32_t wi = defer ? 0u : h.ms + 1 > 4096 ? W / 2 : W - 1;  // waves on the index
  uint32_t part = 0;
  if (wave < wi) {
    if (ifit)
      part = group_crc_part(lds, istart, iend, 0u, wave, wi, group_log2seg(h.is + 1, wi), keys,
                            lane, lane_base, zpow);
  } else if (mfit) {
    part = group_crc_part(lds, mstart, mend, 0u, wave - wi, W - wi,
                          group_log2seg(h.ms + 1, W - wi), keys, lane, lane_base, zpow);
  }
  // ReadMeta's filter lookup (table.cc:76-102) on the last wave, beside the
  // index CRC: speculative, it counts only once the index and the metaindex
  // prove readable (step 4), and it no longer stands between the verdicts
  // and the placement. The wave stages the metaindex in LDS itself (its own
  // stores, then its loads: one wave's LDS accesses are in order).
  if (wave == W - 1 && mfit) {
    const bool staged = h.ms < kMetaStage;
    if (staged)
      for (uint32_t i = lane; i < h.ms; i += 64) L.mbuf[i] = tb.img[h.mo + i];
    find_filter(h, staged ? L.mbuf : tb.img + h.mo, h.ms, reinterpret_cast<const uint8_t*>(L.fkey),
                fk.len, tb, lane);
  }
  if (lane == 0) L.acc[wave] = part;
  __syncthreads();
  sst_stamp(stamps, t, 2);

  // 4. Verdicts (ReadBlock's order), restart array.
  if (tid == 0 && footer_ok) {
    uint32_t ip = 0, mp = 0;
#pragma unroll
    for (int w = 0; w < W; ++w) {
      if (static_cast<uint32_t>(w) < wi) ip ^= L.acc[w]; else mp ^= L.acc[w];
    }
    h.icrc = ifit && !defer ? group_crc_finish(ip, istart, iend, 0u, itail) : 0u;
    h.mcrc = mfit ? group_crc_finish(mp, mstart, mend, 0u, mtail) : 0u;
    if (!ifit) {
      h.index_status = unfit_status(tb.img, static_cast<Fit>(h.ifit), h.io);
    } else {
      h.itype = static_cast<uint8_t>(itype);
      h.index_status = read_status(defer || h.icrc == crc_unmask(itrail), h.itype);
    }
    if (!mfit) {
      h.meta_status = unfit_status(tb.img, static_cast<Fit>(h.mfit), h.mo);
    } else {
      h.mtype = static_cast<uint8_t>(mtype);
      h.meta_status = read_status(h.mcrc == crc_unmask(mtrail), h.mtype);
    }
    switch (h.index_status) {
      case LVKV_BLOCK_OK: break;
      case LVKV_BLOCK_TRUNCATED: h.status = LVKV_SST_INDEX_TRUNCATED; break;
      case LVKV_BLOCK_CHECKSUM: h.status = LVKV_SST_INDEX_CHECKSUM; break;
      default: h.status = LVKV_SST_INDEX_TYPE; break;  // compressed / bad type
    }
    h.nr = 0;
    if (h.status == LVKV_SST_OK) {
      if (h.is < 4 || inr > (h.is - 4) / 4)  // Block::Block (block.cc:28-37)
        h.status = LVKV_SST_INDEX_CORRUPT;
      else
        h.nr = inr;
    }
    // ReadMeta runs only when Table::Open read the index (table.cc:62-76),
    // and ReadFilter only on a readable metaindex
    if (h.index_status != LVKV_BLOCK_OK || h.meta_status != LVKV_BLOCK_OK) {
      h.has_filter = 0;
      h.fo = h.fs = 0;
      h.filter_status = LVKV_BLOCK_OK;
    }
  }
  __syncthreads();
  // Table::Open succeeded iff the index block was read (Block::Block's
  // restart test only makes the index iterator fail, table.cc:62-75); then
  // ReadMeta runs (:76).
  sst_stamp(stamps, t, 3);
  const bool index_usable = h.status == LVKV_SST_OK;
  const bool stage_index = !spec && index_usable && h.is <= kIndexStage;
  uint8_t* ibuf = reinterpret_cast<uint8_t*>(lds);  // the CRC image is spent
  if (stage_index) {
    if (ipf) {
#pragma unroll
      for (int k = 0; k < kIndexPf; ++k) {
        const uint32_t i = tid + kT * static_cast<uint32_t>(k);
        if (i < ind) lds[i] = pf[k];
      }
      ibuf += istart & 3u;
    } else {
      for (uint32_t i = tid; i < h.is; i += kT) ibuf[i] = tb.img[h.io + i];
    }
  }
  __syncthreads();
  sst_stamp(stamps, t, 4);
  // entries: the data blocks the index lists (none when its restart array is
  // unusable), then the filter block
  if (tid == 0) h.nb = (index_usable ? h.nr : 0u) + h.has_filter;
  __syncthreads();

  sst_stamp(stamps, t, 5);
  // 5. Place this table's entries in the shared arrays (wave 0); in the
  //    speculative form the other waves checksum the filter block meanwhile
  //    (the CRC image is intact: nothing was staged over it).
  const bool fcrc = spec && h.has_filter && h.filter_status == LVKV_BLOCK_OK;
  const uint64_t fstart = reinterpret_cast<uint64_t>(tb.img) + h.fo, fend = fstart + h.fs + 1;
  if (wave != 0) {
    if (fcrc && wave == 1 && lane == 0) {  // the verdict's bytes, loaded beside the walk
      const uint8_t* fe = tb.img + h.fo + h.fs;
      L.ftail = group_crc_tail(fstart, fend);
      L.ftype = fe[0];
      L.ftrail = ld_le32(fe + 1);
    }
    uint32_t fpart = 0;
    if (fcrc)
      fpart = group_crc_part(lds, fstart, fend, 0u, wave - 1u, W - 1u,
                             group_log2seg(h.fs + 1, W - 1u), keys, lane, lane_base, zpow);
    if (lane == 0) L.acc[wave] = fpart;
  }
  if (wave == 0) {
    uint32_t total = 0, first = 0;
    if (ntables == 1) {
      total = h.nb <= capacity ? h.nb : 0u;
    } else {
      first = place_table(reports, t, ntables, gen, h.nb, capacity, lane, &total);
    }
    if (lane == 0) {
      h.first = first;
      const bool over = static_cast<uint64_t>(first) + h.nb > capacity;
      if (over) h.status = LVKV_SST_CAPACITY;
      r->status = h.status;
      r->ndata = index_usable || over ? h.nr : 0u;
      r->has_filter = h.has_filter;
      r->nblocks = over ? 0u : h.nb;  // entries written to the shared arrays
      r->nbad = 0;
      r->first_bad = 0xffffffffu;
      r->index_crc = footer_ok ? h.icrc : 0u;
      r->meta_crc = footer_ok ? h.mcrc : 0u;
      r->index_status = h.index_status;
      r->meta_status = h.meta_status;
      r->first = first;
      r->index_offset = h.io;
      r->index_size = h.is;
      r->meta_offset = h.mo;
      r->meta_size = h.ms;
      // the speculative form's CRC workgroups need only the above: published
      // now, while the other waves finish the filter block (its entry and
      // its share of nbad / first_bad follow, atomically)
      if (spec) __hip_atomic_store(&r->done_, gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      if (t == ntables - 1) reports[0].total_ = total;
      if (wide) {
        // sst_index_kernel's tag (this call's generation when it has the
        // index to finish) and its accumulator / arrival words
        r->link_ = 0;
        r->done_ = defer ? gen : 0u;
      }
    }
  }
  __syncthreads();
  sst_stamp(stamps, t, 6);
  if (h.status == LVKV_SST_CAPACITY || h.nb == 0) return;

  // 6. Every entry: index entries 0..nr-1, then the filter block.
  const uint64_t nr = index_usable ? h.nr : 0u;
  if (tid == 0 && h.has_filter) {
    const uint32_t e = h.first + static_cast<uint32_t>(nr);
    uint8_t st = h.filter_status;
    out_off[e] = tb.base + (st == LVKV_BLOCK_OK ? h.fo : 0);
    out_size[e] = static_cast<uint32_t>(st == LVKV_BLOCK_OK ? h.fs : 0);
    if (spec) {
      // ReadBlock's verdict on the filter block (format.cc:92-158), as the
      // CRC store merges it for the data blocks
      uint32_t crc = 0;
      if (fcrc) {
        uint32_t fp = 0;
#pragma unroll
        for (int w = 1; w < W; ++w) fp ^= L.acc[w];
        crc = group_crc_finish(fp, fstart, fend, 0u, L.ftail);
        st = read_status(crc == crc_unmask(L.ftrail), static_cast<uint8_t>(L.ftype));
      }
      spec_crc[e] = crc;
      if (st != LVKV_BLOCK_OK) {
        atomicAdd(&r->nbad, 1u);
        atomicMin(&r->first_bad, static_cast<uint32_t>(nr));
      }
    }
    out_status[e] = st;
  }
  if (nr == 0 || defer || spec) return;
  const uint64_t ro = h.is - (1 + nr) * 4;
  if (stage_index) {
    for (uint32_t i = tid; i < nr; i += kT)
      emit_entry(ibuf, ro, nr, i, ibuf, 0, ro, tb, h.first, out_off, out_size, out_status);
    return;
  }
  // An index larger than LDS: windows of up to kT consecutive entries, the
  // window's bytes staged in LDS (one coalesced pass) and the entries decoded
  // from there; an entry that does not fit its window is decoded from the
  // image.
  const uint8_t* idx = tb.img + h.io;
  uint32_t* wnd = lds;
  for (uint64_t i0 = 0; i0 < nr; i0 += kT) {
    const uint64_t i1 = min<uint64_t>(nr, i0 + kT);
    if (tid == 0) {
      // restart offsets are ascending in a well-formed block; a window that
      // is not (or is too long) is decoded from the image
      const uint64_t lo = ld_le32(idx + ro + 4 * i0);
      const uint64_t hi = i1 < nr ? ld_le32(idx + ro + 4 * i1) : ro;
      const bool ok = lo <= hi && hi <= ro && hi - lo <= kIndexStage - 16;
      L.win_lo = ok ? (lo & ~uint64_t{3}) : 0;
      L.win_hi = ok ? hi : 0;
    }
    __syncthreads();
    const uint64_t lo = L.win_lo, hi = L.win_hi;
    const uint64_t ndw = (hi - lo + 3) / 4;
    for (uint64_t k = tid; k < ndw; k += kT) {
      const uint64_t b = lo + 4 * k;
      wnd[k] = (b + 4 <= ro) ? ld_le32(idx + b)
                             : (static_cast<uint32_t>(idx[b]) |
                                (b + 1 < ro ? static_cast<uint32_t>(idx[b + 1]) << 8 : 0u) |
                                (b + 2 < ro ? static_cast<uint32_t>(idx[b + 2]) << 16 : 0u));
    }
    __syncthreads();
    const uint64_t i = i0 + tid;
    if (i < i1)
      emit_entry(idx, ro, nr, static_cast<uint32_t>(i), reinterpret_cast<const uint8_t*>(wnd), lo,
                 hi, tb, h.first, out_off, out_size, out_status);
    __syncthreads();
  }
}

constexpr int kW = 16;  // waves per head of the two-launch form
constexpr int kFW = 8;  // waves per workgroup of the fused form

// Two-launch form, launch 1: table t = blockIdx.x, 16 waves (large indexes).
__global__ void __launch_bounds__(64 * kW, 1)
    sst_table_kernel(const uint8_t* file, const uint64_t* toff, const uint64_t* tsize,
                     uint64_t single_size, uint32_t ntables, uint32_t capacity, uint32_t gen,
                     FilterKey fk, lvkv_sst_report* reports, uint64_t* out_off,
                     uint32_t* out_size, uint8_t* out_status, const uint32_t* zpow,
                     const uint32_t* lane_cols, uint64_t* stamps, bool wide) {
  __shared__ __attribute__((aligned(16)))
  uint32_t lds[kCompactLdsBytes / 4 + (sizeof(SstHeadLds) + 3) / 4];
  sst_head<kW>(lds, file, toff, tsize, single_size, blockIdx.x, ntables, capacity, gen, fk,
               reports, out_off, out_size, out_status, zpow, lane_cols, stamps, wide);
  __syncthreads();
  sst_stamp(stamps, blockIdx.x, 7);
}

// Two-launch form of a one-table call, between the head and the CRC launch:
// the index the head deferred (report.done_ == this call's generation), on
// kWideGroups workgroups instead of one. Its bytes (contents + type) are cut
// into chunks of C = 2^c bytes back from e4 = floor4(end); workgroup g takes
// chunks g, g + G, ...: each chunk's register over its 8 waves
// (group_crc_part, zero state except the front chunk), shifted to e4 by
// Z_{k C} = Z_{16 k1 C} Z_{k0 C} (k = k0 + 16 k1, two zmul column sets, no
// dependent table chain), xored into the report's link_ word. Every entry
// (block_restart_interval = 1: restart i is entry i) is decoded by one
// thread of the grid. The last workgroup to arrive (link_'s high word)
// finishes the CRC with the 0-3 tail bytes and settles the index verdict in
// ReadBlock's order (checksum, type; then Block::Block's restart test, which
// the head applied): a bad index leaves the table no entries (total_ 0), as
// Table::Open's failure does (table/table.cc:62-75).
__global__ void __launch_bounds__(64 * kWideWaves, 1)
    sst_index_kernel(const uint8_t* file, uint64_t size, uint32_t gen, lvkv_sst_report* reports,
                     uint64_t* out_off, uint32_t* out_size, uint8_t* out_status,
                     const uint32_t* zpow, const uint32_t* lane_cols) {
  constexpr uint32_t W = kWideWaves, kT = 64 * W;
  __shared__ __attribute__((aligned(16))) uint32_t lds[kCompactLdsBytes / 4];
  __shared__ uint32_t acc[W];
  __shared__ uint32_t last_s;
  lvkv_sst_report* r = reports;
  if (__hip_atomic_load(&r->done_, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != gen) return;
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = lane_id();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint64_t io = r->index_offset, is = r->index_size;
  const uint8_t* idx = file + io;
  const uint64_t istart = reinterpret_cast<uint64_t>(idx), iend = istart + is + 1;
  const uint64_t e4 = iend & ~uint64_t{3};
  uint32_t lc = kWideChunkMinLog2;
  while (lc < kWideChunkMaxLog2 && (uint64_t{kWideGroups} << lc) < e4 - istart) ++lc;
  const uint64_t C = uint64_t{1} << lc;
  const uint32_t m = static_cast<uint32_t>((e4 - istart + C - 1) >> lc);  // <= 256
  build_compact_image<W>(lds, zpow, lane_cols, tid, wave, lane);  // ends with a barrier
  const LaneKeys keys = lane_keys(lane);
  const uint32_t lane_base = compact_lane_base(lane);
  uint32_t mine = 0;  // the xor of this workgroup's shifted chunk registers (wave-uniform)
  for (uint32_t k = blockIdx.x; k < m; k += gridDim.x) {
    const uint64_t ce = e4 - uint64_t{k} * C;
    const bool front = k == m - 1u;
    const uint64_t cs = front ? istart : ce - C;
    const uint32_t part = group_crc_part(lds, cs, ce, front ? 0u : 0xffffffffu, wave, W, lc - 3u,
                                         keys, lane, lane_base, zpow);
    if (lane == 0) acc[wave] = part;
    __syncthreads();
    uint32_t reg = 0;
#pragma unroll
    for (uint32_t w = 0; w < W; ++w) reg ^= acc[w];
    __syncthreads();
    // Z_{k C}: lanes [0, 32) hold Z_{k0 C}, lanes [32, 64) Z_{k1 16 C}
    const uint32_t k0 = k & 15u, k1 = k >> 4;
    const uint32_t colv = lane < 32u ? (k0 ? zmul_cols(zpow, lc, k0)[lane] : 0u)
                                     : (k1 ? zmul_cols(zpow, lc + 4u, k1)[lane - 32u] : 0u);
    if (k0) reg = apply_lane_cols(colv, reg, 0, lane);
    if (k1) reg = apply_lane_cols(colv, reg, 1, lane);
    mine ^= reg;
  }
  // every entry, from the image (decoded without a window)
  const uint64_t inr = is >= 4 ? ld_le32(idx + is - 4) : 0u;
  const bool restarts_ok = is >= 4 && inr <= (is - 4) / 4;
  const uint32_t first = r->first;
  const uint64_t nr = restarts_ok ? inr : 0u;
  const Table tb = table_of(file, nullptr, nullptr, size, 0);
  if (static_cast<int32_t>(r->status) == LVKV_SST_OK) {
    const uint64_t ro = is - (1 + nr) * 4;
    for (uint64_t i = uint64_t{blockIdx.x} * kT + tid; i < nr; i += uint64_t{gridDim.x} * kT)
      emit_entry(idx, ro, nr, static_cast<uint32_t>(i), idx, 0, 0, tb, first, out_off, out_size,
                 out_status);
  }
  // arrival: this workgroup's register and the count in one 64-bit add
  // (the registers are xored, so they go through a separate atomic)
  __syncthreads();
  if (tid == 0) {
    uint32_t* words = reinterpret_cast<uint32_t*>(&r->link_);
    if (mine) __hip_atomic_fetch_xor(&words[0], mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t old =
        __hip_atomic_fetch_add(&words[1], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    last_s = old + 1 == gridDim.x ? 1u : 0u;
  }
  __syncthreads();
  if (!last_s || tid != 0) return;
  uint32_t* words = reinterpret_cast<uint32_t*>(&r->link_);
  const uint32_t parts = __hip_atomic_load(&words[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t crc = group_crc_finish(parts, istart, iend, 0u, group_crc_tail(istart, iend));
  const uint8_t itype = idx[is];
  const uint8_t st = read_status(crc == crc_unmask(ld_le32(idx + is + 1)), itype);
  r->index_crc = crc;
  r->index_status = st;
  if (st != LVKV_BLOCK_OK) {
    r->status = st == LVKV_BLOCK_CHECKSUM ? LVKV_SST_INDEX_CHECKSUM : LVKV_SST_INDEX_TYPE;
    r->ndata = 0;
    r->has_filter = 0;
    r->nblocks = 0;
    r->total_ = 0;
  }
  r->link_ = 0;
  r->done_ = 0;
}

constexpr uint32_t kHeadLdsDwords =
    static_cast<uint32_t>(kCompactLdsBytes / 4 + (sizeof(SstHeadLds) + 3) / 4);
constexpr uint32_t kFusedLdsDwords =
    RagLds<kFW>::kDwords > kHeadLdsDwords ? RagLds<kFW>::kDwords : kHeadLdsDwords;

// Fused form, ONE launch: workgroups [0, ntables) are the table heads
// (sst_head<8>), each publishing its report's done_ word (this call's
// generation, release at agent scope) when its entries are written; the
// others build their CRC image, wait for every head (acquire) and run the
// ragged walk in kModeSstTable over all entries, reading the descriptors
// with vector loads (KernelArgs::fresh_desc). Heads never wait on a CRC
// workgroup, and have the lower workgroup ids, so they are dispatched first:
// every wait ends.
__global__ void __launch_bounds__(64 * kFW, 2)
    sst_fused_kernel(KernelArgs a, const uint8_t* file, const uint64_t* toff,
                     const uint64_t* tsize, uint64_t single_size, uint32_t ntables,
                     uint32_t capacity, uint32_t gen, FilterKey fk, lvkv_sst_report* reports,
                     const uint32_t* zpow, const uint32_t* lane_cols, uint64_t* stamps) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kFusedLdsDwords];
  const uint32_t tid = threadIdx.x;
  if (blockIdx.x < ntables) {
    sst_head<kFW>(lds, file, toff, tsize, single_size, blockIdx.x, ntables, capacity, gen, fk,
                  reports, const_cast<uint64_t*>(a.offsets), const_cast<uint32_t*>(a.lengths),
                  a.out_status, zpow, lane_cols, stamps, false);
    // every wave's stores are done at the barrier; one agent-scope release
    // (writes this XCD's L2 back) publishes them with the tag
    __syncthreads();
    if (tid == 0)
      __hip_atomic_store(&reports[blockIdx.x].done_, gen, __ATOMIC_RELEASE,
                         __HIP_MEMORY_SCOPE_AGENT);
    sst_stamp(stamps, blockIdx.x, 7);
    return;
  }
  const uint32_t lane = lane_id();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (tid == 0) lds[RagLds<kFW>::kFlag] = 0;
  build_compact_image<kFW>(lds, zpow, lane_cols, tid, wave, lane);  // ends with a barrier
  if (blockIdx.x == ntables) sst_stamp(stamps, 0, 10);
  // Wait for every head, then one agent-scope acquire (pairing with the
  // heads' release of done_). Everything the heads wrote is also read with
  // agent-scope atomic loads (desc_u64/_u32, the kModeSstTable store).
  if (wave == 0) {
    for (uint32_t j = lane; j < ntables; j += 64)
      while (__hip_atomic_load(&reports[j].done_, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != gen)
        __builtin_amdgcn_s_sleep(8);
    // pairs with the heads' release of done_ (one acquire once every wait
    // has ended, not one per spin)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
  const bool probe = blockIdx.x == ntables;  // the first CRC workgroup's stamps (table 0's row)
  if (probe) sst_stamp(stamps, 0, 8);
  const uint32_t total = min(
      capacity, __builtin_amdgcn_readfirstlane(__hip_atomic_load(
                    &reports[0].total_, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)));
  ragged_run<kFW, 2, 24>(a, zpow, lane_cols, lds, blockIdx.x - ntables, gridDim.x - ntables, total,
                         true);
  if (probe) sst_stamp(stamps, 0, 9);
}

// ---- Speculative form, ONE launch (sst_spec_kernel) ----------------------
// The heads' chain (footer, index and metaindex CRCs, verdicts, the filter
// lookup, the placement) no longer stands before the data CRCs: each CRC
// workgroup takes a share of one table's index entries, reads the footer and
// the index itself, decodes its entries (restart point i is entry i), walks
// their blocks, and only then waits for its table's head to publish the
// verdict and the table's place; the results are written there, or dropped
// when the head found the index unusable (Table::Open failed) or the arrays
// full. Decoding the same index bytes as the head would gives the same
// entries, so the outputs are the two-launch form's.
constexpr uint32_t kSpecPass = 256;    // entries decoded and walked per pass
constexpr uint32_t kSpecTail = 4096;   // index tail staged: restart arrays of <= 1023 entries
constexpr uint32_t kSpecWindow = 6144; // entry bytes staged per pass

struct SpecLds {
  uint64_t off[kSpecPass];       // handle offset in the table (0 unless parsed)
  uint32_t size[kSpecPass];      // contents bytes
  uint32_t rst[kSpecPass + 1];   // the pass's restart offsets, then its end
  uint8_t st[kSpecPass];         // parse status, then ReadBlock's verdict
  union {
    uint32_t tail[kSpecTail / 4 + 16];  // the table's / index's last bytes (aligned dwords)
    uint32_t win[kSpecWindow / 4 + 1];  // the pass's entry bytes (aligned dwords)
    uint32_t crc[kSpecPass];            // computed CRCs (after the decode)
  };
  uint64_t wsum[kFW];            // size scan: per-wave totals
  Head h;
  uint8_t foot[kFooterLen];
  uint64_t wlo, whi;
  uint32_t slot_t, slot_k, slot_c;
  uint32_t nr_raw;
  uint32_t first, nblocks, ndata;
  uint32_t nbad, minbad;
};

// A 64-bit value every lane holds alike, as scalars.
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
  return (static_cast<uint64_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v >> 32)))
          << 32) |
         __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v));
}

// The walk's blocks: the pass's decoded entries in LDS; its results go back
// there (CRC, ReadBlock's verdict merged as rag_store's kModeSstTable does).
struct SpecSrc {
  SpecLds* L;
  uint64_t img;  // the table image's address
  // the stored CRC after each block: loaded by the walk (RagRound::adopt)
  __device__ __forceinline__ bool trailer(const KernelArgs&) const { return true; }
  __device__ __forceinline__ RagBlock block(const KernelArgs& a, uint32_t b, bool live) const {
    RagBlock g;
    g.ptr_lo = g.ptr_hi = g.len = g.s0 = g.expected = 0;
    g.kind = kRagNone;
    if (!live) return g;
    if (__builtin_amdgcn_readfirstlane(L->st[b]) != LVKV_BLOCK_OK) return g;
    const uint64_t o = L->off[b];
    const uint64_t ptr = img + ((static_cast<uint64_t>(__builtin_amdgcn_readfirstlane(
                                     static_cast<uint32_t>(o >> 32))) << 32) |
                                __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(o)));
    const uint32_t len = __builtin_amdgcn_readfirstlane(L->size[b]) + 1u;  // + the type byte
    g.ptr_lo = static_cast<uint32_t>(ptr);
    g.ptr_hi = static_cast<uint32_t>(ptr >> 32);
    g.len = len;
    g.s0 = 0xffffffffu;  // init 0
    g.kind = len > a.long_split ? kRagSkip : len < 4 ? kRagTiny : kRagRows;
    return g;
  }
  __device__ __forceinline__ void store(const KernelArgs&, uint32_t b, const RagBlock& g,
                                        uint32_t crc) const {
    if (lane_id() != 0) return;
    const uint8_t type = *reinterpret_cast<const uint8_t*>(g.ptr() + g.len - 1);
    L->crc[b] = crc;
    L->st[b] = read_status(crc == g.expected, type);
  }
  __device__ __forceinline__ uint32_t covered(const KernelArgs&, uint32_t b) const {
    return L->st[b] == LVKV_BLOCK_OK ? L->size[b] + 1u : 0u;
  }
};

constexpr uint32_t kSpecLdsDwords =
    RagLds<kFW>::kDwords + static_cast<uint32_t>((sizeof(SpecLds) + 3) / 4);
constexpr uint32_t kSpecKernelLdsDwords =
    kSpecLdsDwords > kHeadLdsDwords ? kSpecLdsDwords : kHeadLdsDwords;

// CRC workgroup j of G (G > ntables): its table t and share k of c. Table t
// owns the workgroups [ceil(P_t G / P), ceil(P_{t+1} G / P)), P_t the prefix of
// (size + U) over the tables before t and U > T / (G - ntables) (T the
// tables' bytes), so every table has at least one and large tables more.
template <int W>
__device__ __forceinline__ void spec_crc_group(const KernelArgs& a, const uint8_t* file,
                                               const uint64_t* toff, const uint64_t* tsize,
                                               uint64_t single_size, uint32_t ntables,
                                               uint32_t gen, lvkv_sst_report* reports,
                                               const uint32_t* zpow, const uint32_t* lane_cols,
                                               uint32_t* lds, uint32_t j, uint32_t G,
                                               uint64_t* stamps) {
  constexpr uint32_t kT = 64 * W;
  SpecLds& L = *reinterpret_cast<SpecLds*>(lds + RagLds<W>::kDwords);
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = lane_id();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  // 1. The share, the sizes' load beside the CRC image.
  const uint64_t mysz = (ntables > 1 && tid < ntables) ? tsize[tid] : 0u;
  build_compact_image<W>(lds, zpow, lane_cols, tid, wave, lane);  // ends with a barrier
  if (ntables == 1) {
    if (tid == 0) {
      L.slot_t = 0;
      L.slot_k = j;
      L.slot_c = G;
    }
  } else {
    const uint64_t inc = wave_scan_dpp<uint64_t>(mysz, lane);  // inclusive prefix within the wave
    if (lane == 63) L.wsum[wave] = inc;
    __syncthreads();
    uint64_t before = 0, T = 0;
#pragma unroll
    for (uint32_t w = 0; w < W; ++w) {
      const uint64_t v = L.wsum[w];
      before += w < wave ? v : 0u;
      T += v;
    }
    if (tid < ntables) {
      const uint64_t U = T / (G - ntables) + 1u;
      const uint64_t P = T + uint64_t{ntables} * U;
      const uint64_t p0 = before + inc - mysz + uint64_t{tid} * U;
      const uint64_t p1 = before + inc + uint64_t{tid + 1} * U;
      const uint64_t lo = (p0 * G + P - 1) / P, hi = (p1 * G + P - 1) / P;
      if (lo <= j && j < hi) {
        L.slot_t = tid;
        L.slot_k = j - static_cast<uint32_t>(lo);
        L.slot_c = static_cast<uint32_t>(hi - lo);
      }
    }
  }
  __syncthreads();
  const uint32_t t = __builtin_amdgcn_readfirstlane(L.slot_t);
  const uint32_t k = __builtin_amdgcn_readfirstlane(L.slot_k);
  const uint32_t c = __builtin_amdgcn_readfirstlane(L.slot_c);
  const Table tb = table_of(file, toff, tsize, single_size, t);
  lvkv_sst_report* r = reports + t;
  // probe stamps of the table's first CRC workgroup: 8 share known, 9 entries
  // decoded, 10 walked, 11 head seen, 12 stored (first pass)
  uint64_t* st = k == 0 ? stamps : nullptr;
  sst_stamp(st, t, 8);

  // 2. The table's last bytes in one round trip: the footer (format.cc:43-67)
  //    and, where TableBuilder leaves the index (right before its 5-byte
  //    trailer and the footer), the index's last kSpecTail bytes with its
  //    restart array. A table whose index cannot be read or has no usable
  //    restart array has no data entries (its head reports why).
  uint8_t* tb8 = reinterpret_cast<uint8_t*>(L.tail);
  const uint64_t img = reinterpret_cast<uint64_t>(tb.img), tend = img + tb.size;
  const uint64_t s4 =
      (tend - min<uint64_t>(tb.size, kSpecTail + kFooterLen + kTrailer)) & ~uint64_t{3};
  const bool staged = s4 >= img && tb.size >= kFooterLen;
  if (staged) {
    const uint64_t e4 = tend & ~uint64_t{3};
    const uint32_t ndw = static_cast<uint32_t>((e4 - s4) >> 2);
    for (uint32_t i = tid; i < ndw; i += kT) L.tail[i] = *reinterpret_cast<const uint32_t*>(s4 + 4u * i);
    if (tid < (tend & 3u)) tb8[e4 - s4 + tid] = *reinterpret_cast<const uint8_t*>(e4 + tid);
  } else if (tid < kFooterLen && tb.size >= kFooterLen) {
    L.foot[tid] = tb.img[tb.size - kFooterLen + tid];
  }
  __syncthreads();
  if (tid == 0) parse_footer(L.h, staged ? tb8 + (tend - kFooterLen - s4) : L.foot, tb.size);
  __syncthreads();
  if (L.h.status != LVKV_SST_OK || L.h.ifit != kFitOk || L.h.is < 4) return;
  // (LDS values the whole workgroup shares: made scalar, so what derives from
  // them does not hold vector registers through the walk)
  const uint64_t io = uni64(L.h.io), is = uni64(L.h.is);
  const uint8_t* idx = tb.img + io;
  const uint64_t istart = reinterpret_cast<uint64_t>(idx), iend = istart + is;

  // 3. The index's last bytes (the restart array): already staged when the
  //    index ends where TableBuilder puts it, else staged now.
  const uint64_t tlo = iend - min<uint64_t>(is, kSpecTail);
  bool tail_ok = staged && tlo >= s4;
  uint64_t t4 = s4;
  if (!tail_ok) {
    t4 = tlo & ~uint64_t{3};
    tail_ok = t4 >= img;
    __syncthreads();  // the footer's bytes are read
    if (tail_ok) {
      const uint32_t ndw = static_cast<uint32_t>((iend - t4 + 3) >> 2);
      for (uint32_t i = tid; i < ndw; i += kT)
        L.tail[i] = *reinterpret_cast<const uint32_t*>(t4 + 4u * i);
    }
    __syncthreads();
  }
  auto le32_at = [&](uint64_t addr) -> uint32_t {  // index bytes, staged when possible
    if (tail_ok && addr >= tlo) {
      const uint8_t* q = tb8 + (addr - t4);
      return static_cast<uint32_t>(q[0]) | (static_cast<uint32_t>(q[1]) << 8) |
             (static_cast<uint32_t>(q[2]) << 16) | (static_cast<uint32_t>(q[3]) << 24);
    }
    return ld_le32(reinterpret_cast<const uint8_t*>(addr));
  };
  const uint32_t nr = __builtin_amdgcn_readfirstlane(le32_at(iend - 4));
  if (nr > (is - 4) / 4 || nr == 0) return;  // Block::Block (block.cc:28-37)
  const uint64_t ro = is - (1 + uint64_t{nr}) * 4;
  const uint32_t i0 = static_cast<uint32_t>(uint64_t{k} * nr / c);
  const uint32_t i1 = static_cast<uint32_t>(uint64_t{k + 1} * nr / c);
  const SpecSrc src{&L, reinterpret_cast<uint64_t>(tb.img)};

  bool waited = false;
  for (uint32_t p0 = i0; p0 < i1; p0 += kSpecPass) {
    const uint32_t n = min(kSpecPass, i1 - p0);
    // 4. The pass's restart offsets, then its entry bytes [rst[0], rst[n]).
    for (uint32_t i = tid; i <= n; i += kT) {
      const uint32_t q = p0 + i;
      L.rst[i] = q == nr ? static_cast<uint32_t>(ro) : le32_at(istart + ro + 4ull * q);
    }
    __syncthreads();
    if (tid == 0) {
      // restart offsets ascend in a well-formed index; a pass whose bytes do
      // not (or are too many) is decoded from the index itself
      const uint64_t lo = L.rst[0], hi = L.rst[n];
      const bool ok = lo <= hi && hi <= ro && hi - lo <= kSpecWindow - 8 &&
                      ((istart + lo) & ~uint64_t{3}) >= reinterpret_cast<uint64_t>(tb.img);
      L.wlo = ok ? lo : 0;
      L.whi = ok ? hi : 0;
    }
    __syncthreads();  // the tail is read: the window may overwrite it
    const uint64_t wlo = uni64(L.wlo), whi = uni64(L.whi);
    const uint64_t w4 = (istart + wlo) & ~uint64_t{3};
    const uint32_t wsh = static_cast<uint32_t>((istart + wlo) & 3u);
    if (whi > wlo) {
      const uint32_t ndw = static_cast<uint32_t>((whi - wlo + wsh + 3) >> 2);
      for (uint32_t i = tid; i < ndw; i += kT)
        L.win[i] = *reinterpret_cast<const uint32_t*>(w4 + 4u * i);
    }
    __syncthreads();
    Entry x{0, 0, LVKV_BLOCK_OK};
    if (tid < n)
      x = decode_index_entry(idx, ro, L.rst[tid], L.rst[tid + 1],
                             reinterpret_cast<const uint8_t*>(L.win) + wsh, wlo, whi, tb);
    __syncthreads();  // the window is read: the CRCs overlay it
    if (tid < n) {
      L.off[tid] = x.off;
      L.size[tid] = static_cast<uint32_t>(x.size);
      L.st[tid] = x.st;
      L.crc[tid] = 0;
    }
    if (tid == 0) lds[RagLds<W>::kFlag] = 0;
    __syncthreads();
    if (p0 == i0) sst_stamp(st, t, 9);
    // 5. The walk (ragged_run over the LDS list, long blocks by the group).
    ragged_run<W, 3, 17>(a, zpow, lane_cols, lds, 0, 1, n, true, src);
    __syncthreads();
    if (p0 == i0) sst_stamp(st, t, 10);
    // 6. The head's verdict and the table's place (agent-scope loads of what
    //    it released with done_), then this pass's entries.
    if (!waited) {
      if (tid == 0) {
        while (__hip_atomic_load(&r->done_, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != gen)
          __builtin_amdgcn_s_sleep(8);
        // pairs with the head's release of done_: the report's fields below
        // are read after it
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        L.first = __hip_atomic_load(&r->first, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        L.nblocks = __hip_atomic_load(&r->nblocks, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        L.ndata = __hip_atomic_load(&r->ndata, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __syncthreads();
      waited = true;
      sst_stamp(st, t, 11);
    }
    const uint32_t first = __builtin_amdgcn_readfirstlane(L.first);
    const uint32_t nblocks = __builtin_amdgcn_readfirstlane(L.nblocks);
    const uint32_t ndata = __builtin_amdgcn_readfirstlane(L.ndata);
    if (tid == 0) {
      L.nbad = 0;
      L.minbad = 0xffffffffu;
    }
    __syncthreads();
    if (tid < n && nblocks != 0 && p0 + tid < ndata) {
      const uint32_t e = first + p0 + tid;
      const uint8_t st = L.st[tid];
      const_cast<uint64_t*>(a.offsets)[e] = tb.base + L.off[tid];
      const_cast<uint32_t*>(a.lengths)[e] = L.size[tid];
      a.out_crc[e] = L.crc[tid];
      a.out_status[e] = st;
      if (st != LVKV_BLOCK_OK) {
        atomicAdd(&L.nbad, 1u);
        atomicMin(&L.minbad, p0 + tid);
      }
    }
    __syncthreads();
    if (tid == 0 && L.nbad) {
      atomicAdd(&r->nbad, L.nbad);
      atomicMin(&r->first_bad, L.minbad);
    }
    if (p0 == i0) sst_stamp(st, t, 12);
    // The staged tail shares its LDS with the window and the CRCs, which
    // this pass overwrote: later passes read their restart offsets from the
    // index in memory.
    tail_ok = false;
  }
}

// The speculative form: workgroups [0, ntables) are the heads (the filter
// block checksummed by the head, no data entries), each releasing its report
// with done_ = this call's generation; the others are CRC workgroups
// (spec_crc_group). Heads have the lower ids and never wait on a CRC
// workgroup, so every wait ends.
__global__ void __launch_bounds__(64 * kFW, 4)
    sst_spec_kernel(KernelArgs a, const uint8_t* file, const uint64_t* toff,
                    const uint64_t* tsize, uint64_t single_size, uint32_t ntables,
                    uint32_t capacity, uint32_t gen, FilterKey fk, lvkv_sst_report* reports,
                    const uint32_t* zpow, const uint32_t* lane_cols, uint64_t* stamps) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kSpecKernelLdsDwords];
  if (blockIdx.x < ntables) {
    sst_head<kFW>(lds, file, toff, tsize, single_size, blockIdx.x, ntables, capacity, gen, fk,
                  reports, const_cast<uint64_t*>(a.offsets), const_cast<uint32_t*>(a.lengths),
                  a.out_status, zpow, lane_cols, stamps, false, a.out_crc);
    __syncthreads();
    if (threadIdx.x == 0)
      __hip_atomic_store(&reports[blockIdx.x].done_, gen, __ATOMIC_RELEASE,
                         __HIP_MEMORY_SCOPE_AGENT);
    sst_stamp(stamps, blockIdx.x, 7);
    return;
  }
  spec_crc_group<kFW>(a, file, toff, tsize, single_size, ntables, gen, reports, zpow, lane_cols,
                      lds, blockIdx.x - ntables, gridDim.x - ntables, stamps);
}

}  // namespace

hipError_t launch_crc32c_general(const KernelArgs& a, int cus, hipStream_t stream);

#ifdef LVKV_PROBE_BUILD
uint64_t* g_sst_stamps = nullptr;  // lvkv_debug_sst_stamps
static uint64_t* sst_stamps() { return g_sst_stamps; }
#else
static uint64_t* sst_stamps() { return nullptr; }
#endif

// Whole-table verify of `ntables` images (toff/tsize device arrays, or
// nullptr and `single_size` for one image at d_file); `verify` carries the
// KernelArgs template (tables) the caller filled. `form`: kSstFormSpec one
// launch (sst_spec_kernel; ntables < groups), kSstFormFused one launch
// (sst_fused_kernel), kSstFormTwo the two-launch form (16-wave heads, then
// the ragged kernel).
hipError_t launch_sst_tables(const uint8_t* file, const uint64_t* toff, const uint64_t* tsize,
                             uint64_t single_size, uint32_t ntables, uint64_t* d_off,
                             uint32_t* d_size, uint32_t* d_actual, uint8_t* d_status,
                             uint32_t capacity, lvkv_sst_report* reports, const FilterKey& fk,
                             uint32_t gen, const KernelArgs& verify, const uint32_t* zpow,
                             const uint32_t* lane_cols, int groups, int form,
                             hipStream_t stream) {
  // every data and filter block of every table: CRC, then the merge into
  // LVKV_BLOCK_* and the per-table totals in the kernel's store
  KernelArgs a = verify;
  a.base = file;
  a.offsets = d_off;
  a.lengths = d_size;
  a.inits = nullptr;
  a.out_crc = d_actual;
  a.out_status = d_status;
  a.mode = kModeSstTable;
  a.nblocks = capacity;
  a.count = &reports[0].total_;
  a.long_split = kLongBytes;  // large data/filter blocks: one workgroup each
  a.sst_reports = reports;
  a.sst_ntables = ntables;
  if (form == kSstFormSpec && ntables < static_cast<uint32_t>(groups)) {
    a.run_base = nullptr;
    // two workgroups per CU resident: the heads, then 2 * groups - ntables
    // CRC workgroups (more than ntables)
    const uint32_t grid = 2u * static_cast<uint32_t>(groups);
    hipLaunchKernelGGL(sst_spec_kernel, dim3(grid), dim3(64 * kFW), 0, stream, a, file, toff,
                       tsize, single_size, ntables, capacity, gen, fk, reports, zpow, lane_cols,
                       sst_stamps());
    return hipGetLastError();
  }
  if (form == kSstFormFused) {
    a.fresh_desc = 1;
    // two workgroups per CU resident; the heads come first
    const uint32_t grid = max(2u * static_cast<uint32_t>(groups), ntables + static_cast<uint32_t>(groups));
    hipLaunchKernelGGL(sst_fused_kernel, dim3(grid), dim3(64 * kFW), 0, stream, a, file, toff,
                       tsize, single_size, ntables, capacity, gen, fk, reports, zpow, lane_cols,
                       sst_stamps());
    return hipGetLastError();
  }
  // one table: a large index goes to sst_index_kernel (a no-op launch when
  // the head kept it)
  const bool wide = ntables == 1 && toff == nullptr;
  hipLaunchKernelGGL(sst_table_kernel, dim3(ntables), dim3(64 * kW), 0, stream, file, toff,
                     tsize, single_size, ntables, capacity, gen, fk, reports, d_off, d_size,
                     d_status, zpow, lane_cols, sst_stamps(), wide);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (wide) {
    hipLaunchKernelGGL(sst_index_kernel, dim3(kWideGroups), dim3(64 * kWideWaves), 0, stream,
                       file, single_size, gen, reports, d_off, d_size, d_status, zpow, lane_cols);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  return launch_crc32c_general(a, groups, stream);
}

}  // namespace lvkv
