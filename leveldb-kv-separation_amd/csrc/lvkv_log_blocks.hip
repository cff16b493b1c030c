// WAL / MANIFEST verify on the device: every physical
// record of a log image, with log::Reader::ReadPhysicalRecord's reporting
// (db/log_reader.cc:189-271, checksum = true, initial_offset = 0).
//
// Headers never straddle a 32 KiB block (the writer pads the tail of a block
// with zeros, db/log_writer.cc:44-55) and the reader drops the REST OF THE
// BLOCK on every error, so each block's verdict depends on that block only:
// one lane walks one block's headers. Five launches, no host round trip:
//
//   1. log_count_kernel   per block: walk the headers (length, type) to the
//                         first stop (bad length, zero record, end); count
//                         the candidate records, keep the walk verdict
//   2. log_scan_kernel    one workgroup: exclusive scan of the counts -> the
//                         block's first record slot; total vs capacity
//   3. log_emit_kernel    per block: walk again, write the header offsets
//   4. crc32c_ragged_kernel log-verify mode over all candidates (count read
//                         on the device)
//   5. log_merge_kernel   per block: the first checksum mismatch drops the
//                         rest of the block; per-block status and reported
//                         drop bytes (Reporter::Corruption), report totals
//
// Measured and rejected: copying each block into LDS (coalesced) before the
// walk. The three walks then read the whole image three times; walking the
// headers straight from HBM/MALL reads a few bytes per record and was faster
// (142 vs 178 us for a 66 MB log).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lvkv_crc32c.h"
#include "lvkv_kernel_args.h"

namespace lvkv {
namespace {

constexpr uint64_t kLogBlock = 32768;  // db/log_format.h kBlockSize
constexpr uint64_t kLogHeader = 7;     // db/log_format.h kHeaderSize
constexpr uint32_t kWalkThreads = 256;
constexpr uint32_t kScanThreads = 1024;

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

// Walks one block's headers, calling f(hdr_offset, k) for candidate record k.
// Returns the walk verdict (LVKV_LOGBLK_OK / BAD_LENGTH / ZERO / EOF) and the
// stop position (where a bad length was found).
template <typename F>
__device__ uint8_t walk_block(const uint8_t* file, const BlockSpan& s, uint64_t* stop, F&& f) {
  uint64_t pos = s.start;
  uint32_t k = 0;
  while (s.end - pos >= kLogHeader) {
    const uint8_t* h = file + pos;
    const uint64_t length = static_cast<uint64_t>(h[4]) | (static_cast<uint64_t>(h[5]) << 8);
    const uint8_t type = h[6];
    if (kLogHeader + length > s.end - pos) {  // :221-232
      *stop = pos;
      return s.eof ? LVKV_LOGBLK_EOF : LVKV_LOGBLK_BAD_LENGTH;
    }
    if (type == 0 && length == 0) {  // :234-240 (preallocated region)
      *stop = pos;
      return LVKV_LOGBLK_ZERO;
    }
    f(pos, k++);
    pos += kLogHeader + length;
  }
  *stop = pos;
  // A short tail: a trailer inside the file (skipped), or a truncated header
  // at the end of the file (kEof, not an error; :206-213).
  return (s.eof && pos < s.end) ? LVKV_LOGBLK_EOF : LVKV_LOGBLK_OK;
}

__global__ void __launch_bounds__(kWalkThreads)
    log_count_kernel(const uint8_t* file, uint64_t size, uint32_t nblocks, uint32_t* counts,
                     uint8_t* block_status, lvkv_log_report* r) {
  const uint32_t b = blockIdx.x * kWalkThreads + threadIdx.x;
  if (b == 0) {
    r->status = LVKV_OK;
    r->nblocks = nblocks;
    r->nrecords = 0;
    r->ngood = 0;
    r->ncorrupt = 0;
    r->first_bad_block = 0xffffffffu;
    r->dropped_bytes = 0;
    r->count_ = 0;
  }
  if (b >= nblocks) return;
  uint64_t stop;
  uint32_t n = 0;
  block_status[b] = walk_block(file, block_span(b, size), &stop, [&](uint64_t, uint32_t) { ++n; });
  counts[b] = n;
}

// Exclusive scan of counts[0, n) in place by one workgroup: each thread sums a
// contiguous chunk, the chunk sums are scanned in LDS, then each thread
// rewrites its chunk.
__global__ void __launch_bounds__(kScanThreads)
    log_scan_kernel(uint32_t* counts, uint32_t n, uint32_t capacity, lvkv_log_report* r) {
  __shared__ uint32_t part[kScanThreads];
  const uint32_t t = threadIdx.x;
  const uint32_t per = (n + kScanThreads - 1) / kScanThreads;
  const uint32_t lo = min(n, t * per), hi = min(n, lo + per);
  uint32_t sum = 0;
  for (uint32_t i = lo; i < hi; ++i) sum += counts[i];
  part[t] = sum;
  __syncthreads();
  for (uint32_t d = 1; d < kScanThreads; d <<= 1) {  // Hillis-Steele, inclusive
    const uint32_t v = t >= d ? part[t - d] : 0u;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint32_t run = part[t] - sum;
  for (uint32_t i = lo; i < hi; ++i) {
    const uint32_t c = counts[i];
    counts[i] = run;
    run += c;
  }
  if (t == kScanThreads - 1) {
    const uint32_t total = part[t];
    r->nrecords = total;
    if (total > capacity) {
      r->status = LVKV_LOG_CAPACITY;
      r->count_ = 0;
    } else {
      r->count_ = total;
    }
  }
}

__global__ void __launch_bounds__(kWalkThreads)
    log_emit_kernel(const uint8_t* file, uint64_t size, uint32_t nblocks, const uint32_t* base,
                    uint64_t* hdr_off, const lvkv_log_report* r) {
  const uint32_t b = blockIdx.x * kWalkThreads + threadIdx.x;
  if (b >= nblocks || r->status != LVKV_OK) return;
  const uint32_t first = base[b];
  uint64_t stop;
  walk_block(file, block_span(b, size), &stop,
             [&](uint64_t pos, uint32_t k) { hdr_off[first + k] = pos; });
}

__global__ void __launch_bounds__(kWalkThreads)
    log_merge_kernel(const uint8_t* file, uint64_t size, uint32_t nblocks, uint32_t* base_drop,
                     uint8_t* block_status, uint8_t* rec_status, lvkv_log_report* r) {
  const uint32_t b = blockIdx.x * kWalkThreads + threadIdx.x;
  if (b >= nblocks || r->status != LVKV_OK) return;
  const uint32_t first = base_drop[b];
  const BlockSpan s = block_span(b, size);
  bool mismatch = false;
  uint64_t drop = 0;
  uint32_t good = 0;
  uint64_t stop;
  const uint8_t walked = walk_block(file, s, &stop, [&](uint64_t pos, uint32_t k) {
    uint8_t* st = rec_status + first + k;
    if (mismatch) {
      *st = LVKV_REC_DROPPED;  // the reader cleared the buffer (:248-255)
    } else if (*st != LVKV_REC_OK) {
      mismatch = true;
      drop = s.end - pos;  // ReportCorruption(buffer_.size(), "checksum mismatch")
    } else {
      ++good;
    }
  });
  uint8_t status = walked;
  if (mismatch) {
    status = LVKV_LOGBLK_CHECKSUM;
  } else if (walked == LVKV_LOGBLK_BAD_LENGTH) {
    drop = s.end - stop;  // ReportCorruption(drop_size, "bad record length")
  }
  block_status[b] = status;
  base_drop[b] = static_cast<uint32_t>(drop);
  if (good) atomicAdd(&r->ngood, good);
  if (status == LVKV_LOGBLK_CHECKSUM || status == LVKV_LOGBLK_BAD_LENGTH) {
    atomicAdd(&r->ncorrupt, 1u);
    atomicAdd(reinterpret_cast<unsigned long long*>(&r->dropped_bytes),
              static_cast<unsigned long long>(drop));
    atomicMin(&r->first_bad_block, b);
  }
}

}  // namespace

hipError_t launch_crc32c_general(const KernelArgs& a, int cus, hipStream_t stream);

hipError_t launch_log_blocks(const uint8_t* file, uint64_t size, uint64_t* hdr_off,
                             uint32_t* actual, uint8_t* rec_status, uint32_t capacity,
                             uint8_t* block_status, uint32_t* block_drop, lvkv_log_report* r,
                             const KernelArgs& verify, int groups, hipStream_t stream) {
  const uint32_t nblocks = static_cast<uint32_t>((size + kLogBlock - 1) / kLogBlock);
  const uint32_t grid = max(1u, (nblocks + kWalkThreads - 1) / kWalkThreads);
  hipLaunchKernelGGL(log_count_kernel, dim3(grid), dim3(kWalkThreads), 0, stream, file, size,
                     nblocks, block_drop, block_status, r);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(log_scan_kernel, dim3(1), dim3(kScanThreads), 0, stream, block_drop,
                     nblocks, capacity, r);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(log_emit_kernel, dim3(grid), dim3(kWalkThreads), 0, stream, file, size,
                     nblocks, block_drop, hdr_off, r);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  KernelArgs a = verify;
  a.base = file;
  a.offsets = hdr_off;
  a.out_crc = actual;
  a.out_status = rec_status;
  a.nblocks = capacity;
  a.count = &r->count_;
  if ((e = launch_crc32c_general(a, groups, stream)) != hipSuccess) return e;
  hipLaunchKernelGGL(log_merge_kernel, dim3(grid), dim3(kWalkThreads), 0, stream, file, size,
                     nblocks, block_drop, block_status, rec_status, r);
  return hipGetLastError();
}

}  // namespace lvkv
