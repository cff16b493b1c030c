// Whole-SSTable verify on the device, for one table or
// many at once: the footer, index and metaindex walk of Table::Open /
// Table::ReadMeta (table/table.cc:38-105) and ReadBlock's checks
// (table/format.cc:69-160) for every block, as four launches on one stream
// whatever the number of tables, with no host round trip:
//
//   1. sst_open_kernel           two 1024-thread workgroups per table: the
//                                footer (format.cc:43-67: size, magic, the
//                                two BlockHandles, range checks), then the
//                                index resp. metaindex CRC, 16 KiB segments
//                                over the waves (workgroup_crc)
//   2. sst_head_kernel           one wave per table: index checksum verdict,
//                                type byte, restart array (block.cc:25-39),
//                                the "filter." handle in the metaindex
//                                (table.cc:95-104), entry count; the last
//                                wave packs the tables' entries into the
//                                shared arrays (first, capacity)
//   3. sst_entry_kernel          one lane per entry of every table: the index
//                                is written with block_restart_interval = 1
//                                (table_builder.cc:35, :90), so restart point
//                                i IS entry i and the entries decode in
//                                parallel (DecodeEntry, block.cc:55-75;
//                                BlockHandle varints, format.cc:24-30)
//   4. crc32c_ragged_kernel      SST-table mode over all entries (count read
//                                on the device): the CRC, then stored trailer
//                                vs computed CRC, type byte and parse status
//                                -> LVKV_BLOCK_*, per-table nbad / first_bad
//                                (format.cc:92-97, :104-158)
//
// Bounds: every byte the kernels touch is inside its table image: handles
// are range-checked before they reach the CRC kernels (a bad one becomes 0/0
// with a non-zero status), varints are decoded against explicit limits.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_compact_common.h"
#include "crc32c_device_common.h"
#include "lvkv_crc32c.h"
#include "lvkv_kernel_args.h"

namespace lvkv {
namespace {

constexpr uint64_t kTableMagic = 0xdb4775248b80fb57ull;  // table/format.h:76
constexpr uint64_t kFooterLen = 48;  // table/format.h:53 (2 * 20 + 8)
constexpr uint64_t kTrailer = 5;     // table/format.h:79
constexpr uint32_t kThreads = 256;

struct Table {  // one image of the batch
  const uint8_t* img;
  uint64_t base;  // offset of the image in d_file
  uint64_t size;
};

// Table t: from the descriptor arrays, or the single-table call's scalars.
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
__device__ uint32_t get_varint(const uint8_t* p, const uint8_t* limit, uint32_t max_shift,
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
__device__ bool decode_handle(const uint8_t* p, const uint8_t* limit, uint64_t* off,
                              uint64_t* size, const uint8_t** next) {
  const uint32_t n1 = get_varint(p, limit, 63, off);
  if (n1 == 0) return false;
  const uint32_t n2 = get_varint(p + n1, limit, 63, size);
  if (n2 == 0) return false;
  if (next) *next = p + n1 + n2;
  return true;
}

// ReadBlock's short-read test (format.cc:78-87) plus what the CRC kernels
// need: contents + type byte + 4-byte trailer inside the image, n + 1 < 4 GiB.
__device__ __forceinline__ bool handle_in_file(uint64_t off, uint64_t size, uint64_t file_size) {
  return off <= file_size && size + kTrailer <= file_size - off && size + 1 <= 0xffffffffull;
}

// DecodeEntry (table/block.cc:55-75): pointer to the key delta or nullptr.
__device__ const uint8_t* decode_entry(const uint8_t* p, const uint8_t* limit, uint32_t* shared,
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

// Footer (format.cc:43-67): the two BlockHandles and the magic, from the 48
// footer bytes `f` (nullptr: file shorter than a footer).
struct Footer {
  int32_t status;
  uint64_t mo, ms, io, is;
  bool index_ok, meta_ok;  // handle inside the file (handle_in_file)
};

__device__ Footer parse_footer(const uint8_t* f, uint64_t size) {
  Footer r;
  r.status = LVKV_SST_OK;
  r.mo = r.ms = r.io = r.is = 0;
  r.index_ok = r.meta_ok = false;
  if (size < kFooterLen) {  // table/table.cc:40-42
    r.status = LVKV_SST_TOO_SHORT;
    return r;
  }
  const uint64_t magic = static_cast<uint64_t>(ld_le32(f + 40)) |
                         (static_cast<uint64_t>(ld_le32(f + 44)) << 32);
  if (magic != kTableMagic) {  // format.cc:48-55
    r.status = LVKV_SST_BAD_MAGIC;
    return r;
  }
  const uint8_t* p = nullptr;
  if (!decode_handle(f, f + kFooterLen, &r.mo, &r.ms, &p) ||
      !decode_handle(p, f + kFooterLen, &r.io, &r.is, nullptr)) {  // format.cc:58-61
    r.status = LVKV_SST_BAD_HANDLE;
    return r;
  }
  r.index_ok = handle_in_file(r.io, r.is, size);
  r.meta_ok = handle_in_file(r.mo, r.ms, size);
  if (!r.index_ok) r.status = LVKV_SST_INDEX_TRUNCATED;
  return r;
}

// Launch 1, sst_open_kernel: workgroup 2t + w parses table t's footer (its
// 48 bytes staged in LDS by 48 lanes, then one lane) and checksums the index
// (w = 0) or the metaindex (w = 1), contents + type byte, against the stored
// trailer (format.cc:92-97): 16 KiB segments over the 16 waves
// (workgroup_crc). Workgroup 2t writes the report; 2t + 1 only its scratch
// fields.
__global__ void __launch_bounds__(1024, 1)
    sst_open_kernel(const uint8_t* file, const uint64_t* toff, const uint64_t* tsize,
                    uint64_t single_size, lvkv_sst_report* reports, const uint32_t* zpow,
                    const uint32_t* lane_cols) {
  constexpr int W = 16;
  __shared__ __attribute__((aligned(16))) uint32_t lds[kCompactLdsBytes / 4 + W];
  __shared__ uint8_t foot[kFooterLen];
  __shared__ Footer fs;
  const uint32_t t = blockIdx.x >> 1, which = blockIdx.x & 1u;
  const uint32_t tid = threadIdx.x;
  const Table tb = table_of(file, toff, tsize, single_size, t);
  if (tid < kFooterLen && tb.size >= kFooterLen) foot[tid] = tb.img[tb.size - kFooterLen + tid];
  __syncthreads();
  lvkv_sst_report* r = reports + t;
  if (tid == 0) {
    fs = parse_footer(foot, tb.size);
    r->scratch_crc_[which] = 0;
    r->scratch_status_[which] = 0;
    if (which == 0) {
      r->status = fs.status;
      r->nblocks = r->ndata = r->has_filter = r->nbad = 0;
      r->first_bad = 0xffffffffu;
      r->index_crc = r->meta_crc = 0;
      r->index_status = fs.status == LVKV_SST_INDEX_TRUNCATED ? LVKV_BLOCK_TRUNCATED : LVKV_BLOCK_OK;
      r->meta_status = fs.meta_ok ? LVKV_BLOCK_OK : LVKV_BLOCK_TRUNCATED;
      r->first = 0;
      r->index_offset = fs.io;
      r->index_size = fs.is;
      r->meta_offset = fs.mo;
      r->meta_size = fs.ms;
      r->filter_off_ = 0;
      r->filter_size_ = 0;
      r->filter_status_ = LVKV_BLOCK_OK;
      r->total_ = 0;
      r->reserved2_ = 0;  // tables[0]: sst_head_kernel's arrival counter
    }
  }
  __syncthreads();
  if (fs.status != LVKV_SST_OK || (which == 1 && !fs.meta_ok)) return;  // workgroup-uniform
  const uint32_t lane = lane_id();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  build_compact_image<W>(lds, zpow, lane_cols, tid, wave, lane);
  const uint64_t off = which ? fs.mo : fs.io;
  const uint64_t len = (which ? fs.ms : fs.is) + 1;
  const uint64_t start = reinterpret_cast<uint64_t>(tb.img) + off;
  const uint32_t crc = workgroup_crc<W>(lds, lds + kCompactLdsBytes / 4, start, start + len, 0u,
                                        lane_keys(lane), tid, wave, lane, compact_lane_base(lane),
                                        zpow);
  if (tid == 0) {
    r->scratch_crc_[which] = crc;
    r->scratch_status_[which] = crc != crc_unmask(ld_le32(tb.img + off + len)) ? 1 : 0;
  }
}

// Table::ReadMeta's lookup (table.cc:95-104) over the metaindex bytes m[0,
// msize] (contents + type byte): the first key with the "filter." prefix (the
// reference matches "filter." + the policy name, which this path does not
// know; a table carries one filter).
__device__ void find_filter(const uint8_t* m, uint64_t msize, uint64_t file_size,
                            lvkv_sst_report* r) {
  if (m[msize] != 0 || msize < 4) return;  // compressed or no restart array
  const uint32_t nr = ld_le32(m + msize - 4);
  if (nr > (msize - 4) / 4) return;
  const uint8_t* limit = m + (msize - (1 + static_cast<uint64_t>(nr)) * 4);
  // Only the first 7 bytes of each key matter for the test: they are kept in
  // one register (byte i of key7), not a key buffer (private arrays live in
  // scratch memory, one memory round trip per access).
  constexpr uint64_t kFilterPrefix = 0x2e7265746c6966ull;  // "filter." little-endian
  uint64_t key7 = 0;
  uint32_t klen = 0;
  const uint8_t* p = m;
  while (p < limit) {
    uint32_t sh, ns, vl;
    const uint8_t* q = decode_entry(p, limit, &sh, &ns, &vl);
    if (q == nullptr || sh > klen) return;
    // key = key[0, sh) + delta
    for (uint32_t i = sh; i < 7 && i < sh + ns; ++i)
      key7 = (key7 & ~(0xffull << (8 * i))) | (static_cast<uint64_t>(q[i - sh]) << (8 * i));
    klen = sh + ns;
    const bool is_filter = klen >= 7 && (key7 & 0xffffffffffffffull) == kFilterPrefix;
    if (is_filter) {
      uint64_t fo, fsz;
      if (!decode_handle(q + ns, q + ns + vl, &fo, &fsz, nullptr)) return;
      const bool ok = handle_in_file(fo, fsz, file_size);
      r->filter_off_ = ok ? fo : 0;
      r->filter_size_ = ok ? static_cast<uint32_t>(fsz) : 0;
      r->filter_status_ = ok ? LVKV_BLOCK_OK : LVKV_BLOCK_TRUNCATED;
      r->has_filter = 1;
      return;
    }
    p = q + ns + vl;
  }
}

// Index verdict, restart array (Block::Block, block.cc:25-39), the filter
// handle; `meta` = the metaindex bytes (an LDS copy or the image itself).
__device__ void table_head(const Table& tb, lvkv_sst_report* r, const uint8_t* meta) {
  r->index_crc = r->scratch_crc_[0];
  if (r->meta_status == LVKV_BLOCK_OK) {
    r->meta_crc = r->scratch_crc_[1];
    if (r->scratch_status_[1] != 0)
      r->meta_status = LVKV_BLOCK_CHECKSUM;
    else if (meta[r->meta_size] > 2)
      r->meta_status = LVKV_BLOCK_BAD_TYPE;
  }
  if (r->scratch_status_[0] != 0) {  // ReadBlock on the index (format.cc:92-97)
    r->index_status = LVKV_BLOCK_CHECKSUM;
    r->status = LVKV_SST_INDEX_CHECKSUM;
    return;
  }
  const uint8_t* idx = tb.img + r->index_offset;
  const uint64_t isize = r->index_size;
  const uint8_t itype = idx[isize];
  const uint32_t nr = isize >= 4 ? ld_le32(idx + isize - 4) : 0xffffffffu;
  if (itype != 0) {  // kNoCompression only: snappy/zstd are not on this path
    if (itype > 2) r->index_status = LVKV_BLOCK_BAD_TYPE;
    r->status = LVKV_SST_INDEX_TYPE;
    return;
  }
  if (isize < 4 || nr > (isize - 4) / 4) {
    r->status = LVKV_SST_INDEX_CORRUPT;
    return;
  }
  r->ndata = nr;
  if (r->meta_status == LVKV_BLOCK_OK) find_filter(meta, r->meta_size, tb.size, r);
  r->nblocks = nr + r->has_filter;
}

// Launch 2, sst_head_kernel: one wave per table. The metaindex (typically
// tens of bytes) is staged in LDS by the 64 lanes so that lane 0's serial
// parse reads LDS, not HBM. The last wave to finish (arrival counter in
// tables[0], agent-scope fences) then packs the tables' entries: first =
// exclusive prefix of nblocks over the tables still OK; a table that would
// end past `capacity` gets LVKV_SST_CAPACITY, and so does every later table.
constexpr uint32_t kMetaStage = 2048;

__global__ void __launch_bounds__(64)
    sst_head_kernel(const uint8_t* file, const uint64_t* toff, const uint64_t* tsize,
                    uint64_t single_size, uint32_t ntables, uint32_t capacity,
                    lvkv_sst_report* reports) {
  __shared__ uint8_t mbuf[kMetaStage];
  __shared__ uint32_t part[64];
  __shared__ uint32_t last, overflow_at;
  const uint32_t t = blockIdx.x, lane = threadIdx.x;
  lvkv_sst_report* r = reports + t;
  if (r->status == LVKV_SST_OK) {
    const Table tb = table_of(file, toff, tsize, single_size, t);
    const bool stage = r->meta_status == LVKV_BLOCK_OK && r->meta_size + 1 <= kMetaStage;
    if (stage) {
      const uint8_t* m = tb.img + r->meta_offset;
      for (uint32_t i = lane; i <= r->meta_size; i += 64) mbuf[i] = m[i];
    }
    __syncthreads();
    if (lane == 0) table_head(tb, r, stage ? mbuf : tb.img + r->meta_offset);
  }
  if (lane == 0) {
    __threadfence();
    last = atomicAdd(&reports[0].reserved2_, 1u) == ntables - 1 ? 1u : 0u;
    overflow_at = 0xffffffffu;
  }
  __syncthreads();
  if (!last) return;
  __threadfence();
  // the scan, 64 lanes over contiguous chunks of tables
  volatile lvkv_sst_report* vr = reports;
  const uint32_t per = (ntables + 63) / 64;
  const uint32_t lo = min(ntables, lane * per), hi = min(ntables, lo + per);
  uint32_t sum = 0;
  for (uint32_t i = lo; i < hi; ++i) sum += vr[i].status == LVKV_SST_OK ? vr[i].nblocks : 0u;
  part[lane] = sum;
  __syncthreads();
  for (uint32_t d = 1; d < 64; d <<= 1) {  // Hillis-Steele, inclusive
    const uint32_t v = lane >= d ? part[lane - d] : 0u;
    __syncthreads();
    part[lane] += v;
    __syncthreads();
  }
  uint64_t run = part[lane] - sum;
  for (uint32_t i = lo; i < hi; ++i) {
    const uint32_t nb = vr[i].status == LVKV_SST_OK ? vr[i].nblocks : 0u;
    vr[i].first = static_cast<uint32_t>(min<uint64_t>(run, capacity));
    if (run + nb > capacity) {
      if (nb) vr[i].status = LVKV_SST_CAPACITY;
      atomicMin(&overflow_at, static_cast<uint32_t>(min<uint64_t>(run, capacity)));
    }
    run += nb;
  }
  __syncthreads();
  if (lane == 63) {
    vr[0].total_ = min(part[63], overflow_at);
    vr[0].reserved2_ = 0;
  }
}

// Table of entry e: the last table whose first <= e (binary search; tables
// hold contiguous, increasing ranges).
__device__ __forceinline__ uint32_t table_of_entry(const lvkv_sst_report* reports,
                                                   uint32_t ntables, uint32_t e) {
  uint32_t lo = 0, hi = ntables;  // answer in [lo, hi)
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (reports[mid].first <= e) lo = mid; else hi = mid;
  }
  return lo;
}

// Launch 3, sst_entry_kernel: one lane per entry of every table. Entry i of
// the index starts at restart point i and, with interval 1, ends at the next
// one (or at the restart array).
__global__ void __launch_bounds__(kThreads)
    sst_entry_kernel(const uint8_t* file, const uint64_t* toff, const uint64_t* tsize,
                     uint64_t single_size, uint32_t ntables, const lvkv_sst_report* reports,
                     uint64_t* out_off, uint32_t* out_size, uint8_t* out_status) {
  const uint32_t e = blockIdx.x * kThreads + threadIdx.x;
  if (e >= reports[0].total_) return;
  const uint32_t t = table_of_entry(reports, ntables, e);
  const lvkv_sst_report* r = reports + t;
  const uint32_t i = e - r->first;
  const Table tb = table_of(file, toff, tsize, single_size, t);
  uint8_t st = LVKV_BLOCK_BAD_ENTRY;
  uint64_t off = 0, size = 0;
  // (entries below total_ all belong to OK tables, see the scan; the test
  // only keeps the CRC kernel on an empty range should that ever not hold)
  if (r->status != LVKV_SST_OK || i >= r->nblocks) {
  } else if (i == r->ndata) {  // the filter block
    st = r->filter_status_;
    off = r->filter_off_;
    size = r->filter_size_;
  } else {
    const uint8_t* idx = tb.img + r->index_offset;
    const uint64_t nr = r->ndata;
    const uint64_t ro = r->index_size - (1 + nr) * 4;
    const uint32_t rs = ld_le32(idx + ro + 4ull * i);
    const uint64_t end = i + 1 < nr ? ld_le32(idx + ro + 4ull * (i + 1)) : ro;
    if (rs < ro && end <= ro) {
      uint32_t sh, ns, vl;
      const uint8_t* q = decode_entry(idx + rs, idx + ro, &sh, &ns, &vl);
      if (q != nullptr && sh == 0 && q + ns + vl == idx + end) {
        uint64_t ho, hs;
        if (!decode_handle(q + ns, q + ns + vl, &ho, &hs, nullptr)) {
          st = LVKV_BLOCK_BAD_HANDLE;
        } else if (!handle_in_file(ho, hs, tb.size)) {
          st = LVKV_BLOCK_TRUNCATED;
        } else {
          st = LVKV_BLOCK_OK;
          off = ho;
          size = hs;
        }
      }
    }
  }
  if (st != LVKV_BLOCK_OK) off = size = 0;
  out_off[e] = tb.base + off;  // into d_file
  out_size[e] = static_cast<uint32_t>(size);
  out_status[e] = st;
}

}  // namespace

hipError_t launch_crc32c_general(const KernelArgs& a, int cus, hipStream_t stream);

// The four launches for `ntables` images (toff/tsize device arrays, or
// nullptr and `single_size` for one image at d_file); `verify` carries the
// KernelArgs template (tables) the caller filled.
hipError_t launch_sst_tables(const uint8_t* file, const uint64_t* toff, const uint64_t* tsize,
                             uint64_t single_size, uint32_t ntables, uint64_t* d_off,
                             uint32_t* d_size, uint32_t* d_actual, uint8_t* d_status,
                             uint32_t capacity, lvkv_sst_report* reports,
                             const KernelArgs& verify, const uint32_t* zpow,
                             const uint32_t* lane_cols, int groups, hipStream_t stream) {
  hipLaunchKernelGGL(sst_open_kernel, dim3(2 * ntables), dim3(1024), 0, stream, file, toff, tsize,
                     single_size, reports, zpow, lane_cols);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(sst_head_kernel, dim3(ntables), dim3(64), 0, stream, file, toff, tsize,
                     single_size, ntables, capacity, reports);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  const uint32_t egrid = (capacity + kThreads - 1) / kThreads;
  hipLaunchKernelGGL(sst_entry_kernel, dim3(egrid), dim3(kThreads), 0, stream, file, toff, tsize,
                     single_size, ntables, reports, d_off, d_size, d_status);
  if ((e = hipGetLastError()) != hipSuccess) return e;

  // 4. every data and filter block of every table: CRC, then the merge into
  //    LVKV_BLOCK_* and the per-table totals in the kernel's store
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
  return launch_crc32c_general(a, groups, stream);
}

}  // namespace lvkv
