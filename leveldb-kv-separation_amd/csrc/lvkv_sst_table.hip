// Whole-SSTable verify on the device: the footer, index
// and metaindex walk of Table::Open / Table::ReadMeta (table/table.cc:38-105)
// and ReadBlock's checks (table/format.cc:69-160) for every block, as five
// launches on one stream with no host round trip:
//
//   1. sst_footer_kernel      one lane: size check, magic, the two footer
//                             BlockHandles (format.cc:43-67); index and
//                             metaindex handles into the report's scratch
//   2. crc32c_batch_kernel    the index and metaindex cut into up to 64
//                             segments each, checksummed in parallel
//      sst_combine_kernel     one lane per segment: shift by the bytes after
//                             it (Z_n as a product of Z_{2^j} byte tables),
//                             wave xor -> the two block CRCs vs their trailers
//   3. sst_index_kernel       one lane per index entry: the index is written
//                             with block_restart_interval = 1
//                             (table_builder.cc:35, :90), so restart point i
//                             IS entry i and the entries decode in parallel
//                             (DecodeEntry, block.cc:55-75; BlockHandle
//                             varints, format.cc:24-30); lane 0 also walks
//                             the metaindex for the "filter." key
//   4. crc32c_batch_kernel    SST-verify mode over data + filter blocks,
//                             computed CRC only
//   5. sst_merge_kernel       stored trailer vs computed CRC, type byte,
//                             parse status -> LVKV_BLOCK_*, nbad, first_bad
//
// Bounds: every byte the kernels touch is inside [0, file_size): handles are
// range-checked before they reach the CRC kernel (a bad one becomes 0/0 with a
// non-zero status), varints are decoded against explicit limits.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc32c_device_common.h"
#include "lvkv_crc32c.h"
#include "lvkv_kernel_args.h"

namespace lvkv {
namespace {

constexpr uint64_t kTableMagic = 0xdb4775248b80fb57ull;  // table/format.h:76
constexpr uint64_t kFooterLen = 48;  // table/format.h:53 (2 * 20 + 8)
constexpr uint64_t kTrailer = 5;     // table/format.h:79
constexpr uint32_t kIndexThreads = 256;

constexpr uint64_t kSegMin = 16384;

// Z_n(v): the register advanced over n zero bytes, as the product of the
// Z_{2^j} for the set bits j of n (zpow: kZPowCount byte-table sets).
__device__ uint32_t zshift(const uint32_t* zpow, uint32_t v, uint64_t n) {
  while (n) {
    const uint32_t j = __builtin_ctzll(n);
    const uint32_t* t = zpow + j * 1024u;
    v = t[v & 255u] ^ t[256u + ((v >> 8) & 255u)] ^ t[512u + ((v >> 16) & 255u)] ^
        t[768u + (v >> 24)];
    n &= n - 1;
  }
  return v;
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

// ReadBlock's short-read test (format.cc:78-87) plus what the CRC kernel
// needs: contents + type byte + 4-byte trailer inside the file, n + 1 < 4 GiB.
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

__global__ void sst_footer_kernel(const uint8_t* file, uint64_t size, lvkv_sst_report* r) {
  if (threadIdx.x != 0) return;
  r->status = LVKV_SST_OK;
  r->nblocks = 0;
  r->ndata = 0;
  r->has_filter = 0;
  r->nbad = 0;
  r->first_bad = 0xffffffffu;
  r->index_crc = 0;
  r->meta_crc = 0;
  r->index_status = LVKV_BLOCK_OK;
  r->meta_status = LVKV_BLOCK_OK;
  r->index_offset = r->index_size = r->meta_offset = r->meta_size = 0;
  r->scratch_count_ = 0;
  r->scratch_nseg_[0] = r->scratch_nseg_[1] = 0;
  r->scratch_status_[0] = r->scratch_status_[1] = 0;
  if (size < kFooterLen) {  // table/table.cc:40-42
    r->status = LVKV_SST_TOO_SHORT;
    return;
  }
  const uint8_t* f = file + size - kFooterLen;
  const uint64_t magic = static_cast<uint64_t>(ld_le32(f + 40)) |
                         (static_cast<uint64_t>(ld_le32(f + 44)) << 32);
  if (magic != kTableMagic) {  // format.cc:48-55
    r->status = LVKV_SST_BAD_MAGIC;
    return;
  }
  uint64_t mo, ms, io, is;
  const uint8_t* p = nullptr;
  if (!decode_handle(f, f + kFooterLen, &mo, &ms, &p) ||
      !decode_handle(p, f + kFooterLen, &io, &is, nullptr)) {  // format.cc:58-61
    r->status = LVKV_SST_BAD_HANDLE;
    return;
  }
  r->meta_offset = mo;
  r->meta_size = ms;
  r->index_offset = io;
  r->index_size = is;
  if (!handle_in_file(io, is, size)) {
    r->index_status = LVKV_BLOCK_TRUNCATED;
    r->status = LVKV_SST_INDEX_TRUNCATED;
    return;
  }
  const bool meta_ok = handle_in_file(mo, ms, size);
  if (!meta_ok) r->meta_status = LVKV_BLOCK_TRUNCATED;
  // Covered ranges (contents + type byte) cut into m <= 64 segments of at
  // least kSegMin bytes; segment k > 0 starts from register 0 (init ~0).
  uint32_t n = 0;
  for (int blk = 0; blk < 2; ++blk) {
    const uint64_t off = blk == 0 ? io : mo;
    const uint64_t len = blk == 0 ? is + 1 : (meta_ok ? ms + 1 : 0);
    uint64_t m = len ? (len + kSegMin - 1) / kSegMin : 0;
    if (m > 64) m = 64;
    const uint64_t seg = m ? (len + m - 1) / m : 0;
    for (uint64_t k = 0; k < m; ++k) {
      const uint64_t a = k * seg;
      r->seg_off_[n] = off + a;
      r->seg_len_[n] = static_cast<uint32_t>(min(seg, len - a));
      r->seg_init_[n] = k ? 0xffffffffu : 0u;
      ++n;
    }
    r->scratch_nseg_[blk] = static_cast<uint32_t>(m);
  }
  r->scratch_count_ = n;
}

// Wave 0: the index block, wave 1: the metaindex. Lane k owns segment k:
// its register (CRC ^ ~0) advanced over the bytes after the segment, then
// xored over the wave: the block's register, so CRC = reg ^ ~0.
__global__ void __launch_bounds__(128)
    sst_combine_kernel(const uint8_t* file, lvkv_sst_report* r, const uint32_t* zpow) {
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  if (r->status != LVKV_SST_OK || r->scratch_count_ == 0) return;
  const uint32_t m = r->scratch_nseg_[w];
  if (m == 0) return;
  const uint32_t first = w ? r->scratch_nseg_[0] : 0u;
  uint32_t v = 0;
  if (lane < m) {
    const uint32_t i = first + lane;
    const uint64_t end = (w ? r->meta_offset + r->meta_size : r->index_offset + r->index_size) + 1;
    v = zshift(zpow, r->seg_crc_[i] ^ 0xffffffffu, end - (r->seg_off_[i] + r->seg_len_[i]));
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v ^= __shfl_xor(v, d, 64);
  if (lane == 0) {
    const uint32_t crc = v ^ 0xffffffffu;
    const uint8_t* t = file + (w ? r->meta_offset + r->meta_size : r->index_offset + r->index_size);
    r->scratch_crc_[w] = crc;
    r->scratch_status_[w] = crc != crc_unmask(ld_le32(t + 1)) ? 1 : 0;
  }
}

// Lane 0: Table::ReadMeta's lookup (table.cc:95-104) — the first key with
// the "filter." prefix (the reference matches "filter." + the policy name,
// which this path does not know; a table carries one filter).
__device__ void find_filter(const uint8_t* file, uint64_t file_size, lvkv_sst_report* r,
                            uint64_t* out_off, uint32_t* out_size, uint8_t* out_status,
                            uint32_t slot) {
  if (r->meta_status != LVKV_BLOCK_OK || r->scratch_status_[1] != 0) return;
  const uint8_t* m = file + r->meta_offset;
  const uint64_t msize = r->meta_size;
  if (m[msize] != 0 || msize < 4) return;  // compressed or no restart array
  const uint32_t nr = ld_le32(m + msize - 4);
  if (nr > (msize - 4) / 4) return;
  const uint8_t* limit = m + (msize - (1 + static_cast<uint64_t>(nr)) * 4);
  constexpr uint32_t kKeyCap = 64;
  uint8_t key[kKeyCap];
  uint32_t klen = 0;
  const uint8_t* p = m;
  while (p < limit) {
    uint32_t sh, ns, vl;
    const uint8_t* q = decode_entry(p, limit, &sh, &ns, &vl);
    if (q == nullptr || sh > klen) return;
    // key = key[0, sh) + delta; only the first 7 bytes matter for the test
    for (uint32_t i = 0; i < ns && sh + i < kKeyCap; ++i) key[sh + i] = q[i];
    klen = sh + ns;
    const bool is_filter = klen >= 7 && key[0] == 'f' && key[1] == 'i' && key[2] == 'l' &&
                           key[3] == 't' && key[4] == 'e' && key[5] == 'r' && key[6] == '.';
    if (is_filter) {
      uint64_t fo, fs;
      if (!decode_handle(q + ns, q + ns + vl, &fo, &fs, nullptr)) return;
      const bool ok = handle_in_file(fo, fs, file_size);
      out_off[slot] = ok ? fo : 0;
      out_size[slot] = ok ? static_cast<uint32_t>(fs) : 0;
      out_status[slot] = ok ? LVKV_BLOCK_OK : LVKV_BLOCK_TRUNCATED;
      r->has_filter = 1;
      return;
    }
    p = q + ns + vl;
  }
}

__global__ void __launch_bounds__(kIndexThreads)
    sst_index_kernel(const uint8_t* file, uint64_t file_size, lvkv_sst_report* r,
                     uint64_t* out_off, uint32_t* out_size, uint8_t* out_status,
                     uint32_t capacity) {
  const uint32_t gid = blockIdx.x * kIndexThreads + threadIdx.x;
  if (r->status != LVKV_SST_OK) return;
  const bool lead = gid == 0;
  if (r->scratch_status_[0] != 0) {  // ReadBlock on the index (format.cc:92-97)
    if (lead) {
      r->index_status = LVKV_BLOCK_CHECKSUM;
      r->status = LVKV_SST_INDEX_CHECKSUM;
    }
    return;
  }
  const uint8_t* idx = file + r->index_offset;
  const uint64_t isize = r->index_size;
  if (idx[isize] != 0) {  // kNoCompression only: snappy/zstd are not on this path
    if (lead) {
      if (idx[isize] > 2) r->index_status = LVKV_BLOCK_BAD_TYPE;
      r->status = LVKV_SST_INDEX_TYPE;
    }
    return;
  }
  // Block::Block (block.cc:25-39)
  const uint32_t nr = isize >= 4 ? ld_le32(idx + isize - 4) : 0xffffffffu;
  if (isize < 4 || nr > (isize - 4) / 4) {
    if (lead) r->status = LVKV_SST_INDEX_CORRUPT;
    return;
  }
  const uint64_t ro = isize - (1 + static_cast<uint64_t>(nr)) * 4;
  if (static_cast<uint64_t>(nr) + 1 > capacity) {
    if (lead) {
      r->ndata = nr;
      r->status = LVKV_SST_CAPACITY;
    }
    return;
  }
  if (gid < nr) {
    // Entry gid starts at restart point gid and, with interval 1, ends at the
    // next restart point (or at the restart array).
    const uint32_t rs = ld_le32(idx + ro + 4ull * gid);
    const uint64_t end = gid + 1 < nr ? ld_le32(idx + ro + 4ull * (gid + 1)) : ro;
    uint8_t st = LVKV_BLOCK_BAD_ENTRY;
    uint64_t off = 0, size = 0;
    if (rs < ro && end <= ro) {
      uint32_t sh, ns, vl;
      const uint8_t* q = decode_entry(idx + rs, idx + ro, &sh, &ns, &vl);
      if (q != nullptr && sh == 0 && q + ns + vl == idx + end) {
        uint64_t ho, hs;
        if (!decode_handle(q + ns, q + ns + vl, &ho, &hs, nullptr)) {
          st = LVKV_BLOCK_BAD_HANDLE;
        } else if (!handle_in_file(ho, hs, file_size)) {
          st = LVKV_BLOCK_TRUNCATED;
        } else {
          st = LVKV_BLOCK_OK;
          off = ho;
          size = hs;
        }
      }
    }
    out_off[gid] = off;
    out_size[gid] = static_cast<uint32_t>(size);
    out_status[gid] = st;
  }
  if (lead) {
    r->ndata = nr;
    find_filter(file, file_size, r, out_off, out_size, out_status, nr);
    r->nblocks = nr + r->has_filter;
  }
}

__global__ void __launch_bounds__(kIndexThreads)
    sst_merge_kernel(const uint8_t* file, lvkv_sst_report* r, const uint64_t* off,
                     const uint32_t* size, const uint32_t* actual, uint8_t* status) {
  const uint32_t gid = blockIdx.x * kIndexThreads + threadIdx.x;
  if (gid == 0 && r->scratch_count_ > 0) {
    r->index_crc = r->scratch_crc_[0];
    if (r->meta_status == LVKV_BLOCK_OK) {
      r->meta_crc = r->scratch_crc_[1];
      if (r->scratch_status_[1] != 0)
        r->meta_status = LVKV_BLOCK_CHECKSUM;
      else if (file[r->meta_offset + r->meta_size] > 2)
        r->meta_status = LVKV_BLOCK_BAD_TYPE;
    }
  }
  if (r->status != LVKV_SST_OK || gid >= r->nblocks) return;
  uint8_t st = status[gid];
  if (st == LVKV_BLOCK_OK) {
    // ReadBlock (format.cc:92-97, :104-158): checksum first, then the type
    const uint8_t* t = file + off[gid] + size[gid];
    if (actual[gid] != crc_unmask(ld_le32(t + 1)))
      st = LVKV_BLOCK_CHECKSUM;
    else if (t[0] > 2)
      st = LVKV_BLOCK_BAD_TYPE;
    status[gid] = st;
  }
  if (st != LVKV_BLOCK_OK) {
    atomicAdd(&r->nbad, 1u);
    atomicMin(&r->first_bad, gid);
  }
}

}  // namespace

hipError_t launch_crc32c_batch(const KernelArgs& args, bool uniform_aligned, int num_groups,
                               hipStream_t stream);
hipError_t launch_crc32c_long(const KernelArgs& args, const uint32_t* zpow,
                              const uint32_t* lane_cols, int num_groups, hipStream_t stream);

// The five launches; `verify` is the SST-verify KernelArgs template (tables,
// mode) the caller filled.
hipError_t launch_sst_table(const uint8_t* file, uint64_t file_size, uint64_t* d_off,
                            uint32_t* d_size, uint32_t* d_actual, uint8_t* d_status,
                            uint32_t capacity, lvkv_sst_report* r, const KernelArgs& verify,
                            const uint32_t* zpow, const uint32_t* lane_cols, int groups,
                            hipStream_t stream) {
  hipLaunchKernelGGL(sst_footer_kernel, dim3(1), dim3(64), 0, stream, file, file_size, r);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;

  KernelArgs a = verify;
  a.base = file;
  a.mode = kModeCompute;
  a.offsets = r->seg_off_;
  a.lengths = r->seg_len_;
  a.inits = r->seg_init_;
  a.out_crc = r->seg_crc_;
  a.out_status = nullptr;
  a.nblocks = 128;
  a.count = &r->scratch_count_;
  e = launch_crc32c_batch(a, false, 8, stream);  // 8 x 16 waves: one segment each
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(sst_combine_kernel, dim3(1), dim3(128), 0, stream, file, r, zpow);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  a.mode = verify.mode;
  a.inits = nullptr;

  const uint32_t grid = (capacity + kIndexThreads - 1) / kIndexThreads;
  hipLaunchKernelGGL(sst_index_kernel, dim3(grid), dim3(kIndexThreads), 0, stream, file,
                     file_size, r, d_off, d_size, d_status, capacity);
  if ((e = hipGetLastError()) != hipSuccess) return e;

  a.offsets = d_off;
  a.lengths = d_size;
  a.out_crc = d_actual;
  a.out_status = nullptr;  // merged below with the parse status
  a.nblocks = capacity;
  a.count = &r->nblocks;
  a.long_split = 1;  // large data/filter blocks: one workgroup each
  e = launch_crc32c_batch(a, false, groups, stream);
  if (e != hipSuccess) return e;
  if ((e = launch_crc32c_long(a, zpow, lane_cols, groups, stream)) != hipSuccess) return e;

  hipLaunchKernelGGL(sst_merge_kernel, dim3(grid), dim3(kIndexThreads), 0, stream, file, r,
                     d_off, d_size, d_actual, d_status);
  return hipGetLastError();
}

}  // namespace lvkv
