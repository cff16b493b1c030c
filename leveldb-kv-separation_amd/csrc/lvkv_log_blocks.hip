// WAL / MANIFEST verify on the device: every physical
// record of a log image, with log::Reader::ReadPhysicalRecord's reporting
// (db/log_reader.cc:189-271, checksum = true, initial_offset = 0).
//
// Headers never straddle a 32 KiB block (the writer pads the tail of a block
// with zeros, db/log_writer.cc:44-55) and the reader drops the REST OF THE
// BLOCK on every error, so each block's verdict depends on that block only.
// Five launches, no host round trip:
//
//   1. log_count_kernel   one workgroup per block: the block is staged in LDS
//                         (coalesced 16-byte loads), then one lane walks its
//                         headers (length, type) from LDS to the first stop
//                         (bad length, zero record, end): record count and
//                         walk verdict
//   2. log_scan_kernel    one workgroup: exclusive scan of the counts -> the
//                         block's first record slot; total vs capacity
//   3. log_emit_kernel    per block: staged again, walked again, header
//                         offsets written
//   4. crc32c_ragged_kernel log-verify mode over all records (count read on
//                         the device)
//   5. log_merge_kernel   one wave per block, no walk: the block's records
//                         are a contiguous run of the header array; the
//                         first checksum mismatch (a wave min) drops the
//                         rest of the block; per-block status and reported
//                         drop bytes (Reporter::Corruption), report totals
//
// A walk reads a few bytes per record, each dependent on the last. From HBM
// that is one memory round trip per record (the walks were 3/4 of the
// pipeline's time); from LDS it is a few cycles. Staging reads every block
// twice more in full, at streaming bandwidth. The merge takes its record
// positions from the header array instead of a third walk.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lvkv_crc32c.h"
#include "lvkv_kernel_args.h"

namespace lvkv {
namespace {

constexpr uint64_t kLogBlock = 32768;  // db/log_format.h kBlockSize
constexpr uint32_t kLogHeader = 7;     // db/log_format.h kHeaderSize
constexpr uint32_t kStageThreads = 256;
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

// Block bytes [0, n) into LDS by the whole workgroup, then a barrier. A full
// block: all eight 16-byte loads of a thread in flight before the first LDS
// store (a load-store loop waits out one memory round trip per iteration).
__device__ __forceinline__ void stage_block(uint8_t* buf, const uint8_t* src, uint32_t n) {
  const bool vec = (reinterpret_cast<uintptr_t>(src) & 15u) == 0;
  constexpr uint32_t kPer = static_cast<uint32_t>(kLogBlock) / (kStageThreads * 16u);
  if (vec && n == kLogBlock) {
    uint4 v[kPer];
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k)
      v[k] = reinterpret_cast<const uint4*>(src)[threadIdx.x + kStageThreads * k];
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k)
      reinterpret_cast<uint4*>(buf)[threadIdx.x + kStageThreads * k] = v[k];
    __syncthreads();
    return;
  }
  for (uint32_t i = threadIdx.x * 16u; i < n; i += kStageThreads * 16u) {
    if (vec && i + 16u <= n) {
      *reinterpret_cast<uint4*>(buf + i) = *reinterpret_cast<const uint4*>(src + i);
    } else {
      for (uint32_t j = i; j < min(n, i + 16u); ++j) buf[j] = src[j];
    }
  }
  __syncthreads();
}

// Walks one block's headers in blk[0, n) (LDS), calling f(pos, k) for
// candidate record k at block offset pos. Returns the walk verdict
// (LVKV_LOGBLK_OK / BAD_LENGTH / ZERO / EOF).
template <typename F>
__device__ uint8_t walk_block(const uint8_t* blk, uint32_t n, bool eof, F&& f) {
  uint32_t pos = 0, k = 0;
  while (n - pos >= kLogHeader) {
    const uint8_t* h = blk + pos;
    const uint32_t length = static_cast<uint32_t>(h[4]) | (static_cast<uint32_t>(h[5]) << 8);
    const uint8_t type = h[6];
    if (kLogHeader + length > n - pos)  // :221-232
      return eof ? LVKV_LOGBLK_EOF : LVKV_LOGBLK_BAD_LENGTH;
    if (type == 0 && length == 0) return LVKV_LOGBLK_ZERO;  // :234-240 (preallocated)
    f(pos, k++);
    pos += kLogHeader + length;
  }
  // A short tail: a trailer inside the file (skipped), or a truncated header
  // at the end of the file (kEof, not an error; :206-213).
  return (eof && pos < n) ? LVKV_LOGBLK_EOF : LVKV_LOGBLK_OK;
}

__global__ void __launch_bounds__(kStageThreads)
    log_count_kernel(const uint8_t* file, uint64_t size, uint32_t nblocks, uint32_t* counts,
                     uint8_t* block_status, lvkv_log_report* r) {
  __shared__ __attribute__((aligned(16))) uint8_t buf[kLogBlock];
  const uint32_t b = blockIdx.x;
  const BlockSpan s = block_span(b, size);
  if (b == 0 && threadIdx.x == 0) {
    r->status = LVKV_OK;
    r->nblocks = nblocks;
    r->nrecords = 0;
    r->ngood = 0;
    r->ncorrupt = 0;
    r->first_bad_block = 0xffffffffu;
    r->dropped_bytes = 0;
    r->count_ = 0;
  }
  if (b >= nblocks) return;  // an empty log: one workgroup writes the report
  const uint32_t n = static_cast<uint32_t>(s.end - s.start);
  stage_block(buf, file + s.start, n);
  if (threadIdx.x == 0) {
    uint32_t c = 0;
    block_status[b] = walk_block(buf, n, s.eof, [&](uint32_t, uint32_t) { ++c; });
    counts[b] = c;
  }
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
    r->ngood = total;  // log_merge_kernel subtracts the records it drops
    if (total > capacity) {
      r->status = LVKV_LOG_CAPACITY;
      r->count_ = 0;
    } else {
      r->count_ = total;
    }
  }
}

__global__ void __launch_bounds__(kStageThreads)
    log_emit_kernel(const uint8_t* file, uint64_t size, const uint32_t* base, uint64_t* hdr_off,
                    const lvkv_log_report* r) {
  __shared__ __attribute__((aligned(16))) uint8_t buf[kLogBlock];
  const uint32_t b = blockIdx.x;
  if (r->status != LVKV_OK) return;  // workgroup-uniform
  const BlockSpan s = block_span(b, size);
  const uint32_t n = static_cast<uint32_t>(s.end - s.start);
  stage_block(buf, file + s.start, n);
  if (threadIdx.x == 0) {
    uint64_t* out = hdr_off + base[b];
    walk_block(buf, n, s.eof, [&](uint32_t pos, uint32_t k) { out[k] = s.start + pos; });
  }
}

__global__ void __launch_bounds__(64)
    log_merge_kernel(const uint8_t* file, uint64_t size, uint32_t nblocks, uint32_t* base_drop,
                     uint8_t* block_status, const uint64_t* hdr_off, uint8_t* rec_status,
                     lvkv_log_report* r) {
  const uint32_t b = blockIdx.x, lane = threadIdx.x;
  if (r->status != LVKV_OK) return;
  const BlockSpan s = block_span(b, size);
  const uint32_t total = r->nrecords;
  const uint32_t first = base_drop[b];
  // The block's records: the run of header offsets from `first` that lie
  // inside the block (a prefix, hdr_off ascending). Lanes test 64 at a time.
  uint32_t cnt = 0, bad = 0xffffffffu;
  for (uint32_t j = 0;; j += 64) {
    const uint32_t k = j + lane;
    const bool in = first + k < total && hdr_off[first + k] < s.end;
    const uint64_t in_mask = __ballot(in);
    cnt += static_cast<uint32_t>(__builtin_popcountll(in_mask));
    const bool mis = in && rec_status[first + k] != LVKV_REC_OK;
    const uint64_t mis_mask = __ballot(mis);
    if (mis_mask != 0 && bad == 0xffffffffu) bad = j + static_cast<uint32_t>(__builtin_ctzll(mis_mask));
    if (in_mask != ~0ull) break;
  }
  // records after the first mismatch: the reader cleared the buffer (:248-255)
  if (bad != 0xffffffffu)
    for (uint32_t k = bad + 1 + lane; k < cnt; k += 64) rec_status[first + k] = LVKV_REC_DROPPED;
  if (lane != 0) return;
  const uint8_t walked = block_status[b];
  uint8_t status = walked;
  uint64_t drop = 0;
  if (bad != 0xffffffffu) {
    status = LVKV_LOGBLK_CHECKSUM;
    drop = s.end - hdr_off[first + bad];  // ReportCorruption(buffer_.size(), "checksum mismatch")
  } else if (walked == LVKV_LOGBLK_BAD_LENGTH) {
    // the walk stopped at the header after the block's last record
    uint64_t stop = s.start;
    if (cnt) {
      const uint64_t h = hdr_off[first + cnt - 1];
      stop = h + kLogHeader + (static_cast<uint32_t>(file[h + 4]) |
                               (static_cast<uint32_t>(file[h + 5]) << 8));
    }
    drop = s.end - stop;  // ReportCorruption(drop_size, "bad record length")
  }
  block_status[b] = status;
  base_drop[b] = static_cast<uint32_t>(drop);
  // ngood starts at the total: one atomic per damaged block, not per block
  if (bad != 0xffffffffu) atomicSub(&r->ngood, cnt - bad);
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
  hipLaunchKernelGGL(log_count_kernel, dim3(max(1u, nblocks)), dim3(kStageThreads), 0, stream,
                     file, size, nblocks, block_drop, block_status, r);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(log_scan_kernel, dim3(1), dim3(kScanThreads), 0, stream, block_drop,
                     nblocks, capacity, r);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if (nblocks == 0) return hipSuccess;
  hipLaunchKernelGGL(log_emit_kernel, dim3(nblocks), dim3(kStageThreads), 0, stream, file, size,
                     block_drop, hdr_off, r);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  KernelArgs a = verify;
  a.base = file;
  a.offsets = hdr_off;
  a.out_crc = actual;
  a.out_status = rec_status;
  a.nblocks = capacity;
  a.count = &r->count_;
  a.long_split = kLogLongBytes;  // 32 KiB fragments: one workgroup each
  a.run_base = block_drop;       // each workgroup: whole 32 KiB blocks
  a.run_units = nblocks;
  if ((e = launch_crc32c_general(a, groups, stream)) != hipSuccess) return e;
  hipLaunchKernelGGL(log_merge_kernel, dim3(nblocks), dim3(64), 0, stream, file, size, nblocks,
                     block_drop, block_status, hdr_off, rec_status, r);
  return hipGetLastError();
}

}  // namespace lvkv
