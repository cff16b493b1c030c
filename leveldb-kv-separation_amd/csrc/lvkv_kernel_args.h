// Shared host/device definitions for the batched CRC32C engine.
//
// LDS image of one workgroup (gfx950: 160 KiB per CU, all of it used):
//
//   [0, 128 KiB)    row operator Z_256 ("advance the CRC register over 256
//                   zero bytes") as four byte tables A_t[i] = Z_256(i << 8t),
//                   each replicated 32x so that lane l always reads bank l%32:
//                   byte address (t, i, copy c) =
//                       (t >> 1) * 64 KiB + i * 256 + (t & 1) * 128 + c * 4
//   [128, 160 KiB)  per-lane end shift Z_{256-4s} as eight nibble tables,
//                   private to lane s:  byte address (k, nib, s) =
//                       128 KiB + ((k * 16 + nib) * 64 + s) * 4
//
// The tables are generated on the host (lvkv_tables.cpp) and copied once per
// device; each workgroup of the persistent grid replicates them into LDS.
#ifndef LVKV_KERNEL_ARGS_H_
#define LVKV_KERNEL_ARGS_H_

#include <stdint.h>

#include "lvkv_crc32c.h"

namespace lvkv {

constexpr int kWaveLanes = 64;
constexpr int kWavesPerGroup = 16;
constexpr int kGroupThreads = kWaveLanes * kWavesPerGroup;  // 1024
constexpr int kRowBytes = 256;      // one wave-wide row: 64 lanes x 4 B
constexpr int kRowsPerChunk = 16;   // one pipeline stage = 4 KiB per wave
constexpr uint32_t kRowTabDwords = 4 * 256;
constexpr uint32_t kLaneTabDwords = 8 * 16 * 64;
constexpr uint32_t kLaneColDwords = 8 * 64 * 4;  // lane_cols (lvkv_tables.h)
// Blocks longer than this are split over a whole workgroup
// (crc32c_long_kernel) instead of one wave walking them alone.
constexpr uint32_t kLongBytes = 64 * 1024;
// The same for WAL records (<= 32 KiB, most far smaller): a 32 KiB fragment
// walked by one wave would hold up its workgroup.
constexpr uint32_t kLogLongBytes = 8 * 1024;
constexpr uint32_t kZPowCount = 48;               // Z_{2^j}, j < 48 (256 TiB)
constexpr uint32_t kZPowDwords = kZPowCount * 1024;
constexpr uint32_t kZPowOffset = 1024 + 8 * 16 * 64 + 8 * 64 * 4;  // in d_tables
// Columns of Z_{c * 2^j}, j in [kZMulLog0, kZMulLog0 + kZMulLogs), c in
// [1, kZMulMaxC] (lvkv_tables.h), right after zpow in d_tables.
constexpr uint32_t kZMulLog0 = 8, kZMulLogs = 16, kZMulMaxC = 16;
constexpr uint32_t kZMulDwords = kZMulLogs * kZMulMaxC * 32;
constexpr uint32_t kTableDwords = kZPowOffset + kZPowDwords + kZMulDwords;
constexpr uint32_t kLdsRowRegionBytes = 64 * 1024;
constexpr uint32_t kLdsLaneTabBase = 128 * 1024;
constexpr uint32_t kLdsBytes = 160 * 1024;

constexpr uint32_t kCastagnoliReflected = 0x82f63b78u;
constexpr uint32_t kMaskDelta = 0xa282ead8u;  // util/crc32c.h:22

// Kernel modes (KernelArgs::mode).
enum : uint32_t {
  kModeCompute = 0,    // out_crc[i] = Extend(init_i, base + off_i, len_i)
  kModeSstVerify = 1,  // table/format.cc:92-99: covers n+1, trailer after it
  kModeLogVerify = 2,  // db/log_reader.cc:243-257: header at off, len parsed
  kModeSstFill = 3,    // table_builder.cc:199-203: covers n+1, writes the
                       // masked CRC into trailer bytes 1..4
  kModeLogFill = 4,    // log_writer.cc:94-96: header at off, writes the
                       // masked CRC into header bytes 0..3
  kModeSstTable = 5,   // kModeSstVerify whose store also merges the index
                       // parse status (out_status in), the type byte and
                       // the per-table totals (sst_reports)
  kModeLogStaged = 6,  // kModeLogVerify over the WAL walk's staged headers
                       // (lvkv_log_blocks.hip): out_crc, out_status (1 =
                       // mismatch), and on a mismatch the lowest staged
                       // index per 32 KiB block into log_first_bad[hdr >> 15]
};

struct KernelArgs {
  const uint8_t* base;        // device bytes all offsets are relative to
  const uint64_t* offsets;    // per-block offsets; nullptr = uniform stride
  const uint32_t* lengths;    // per-block lengths (ignored in uniform mode)
  const uint32_t* inits;      // per-block init CRCs; nullptr = `init`
  uint64_t stride;            // uniform mode: block i at base + i*stride
  uint32_t length;            // uniform mode length
  uint32_t init;              // init CRC when inits == nullptr
  uint32_t* out_crc;          // nblocks u32 (masked if `mask`)
  uint8_t* out_status;        // verify modes: 0 = match, 1 = mismatch
  const uint32_t* row_tab;    // kRowTabDwords
  const uint32_t* lane_tab;   // kLaneTabDwords, already in LDS order
  uint32_t nblocks;
  uint32_t mode;
  uint32_t mask;              // 1: store Mask(crc) (util/crc32c.h:29-32)
  uint32_t long_split;        // non-zero: blocks whose covered length
                              // exceeds it (bytes) are walked by a whole
                              // workgroup (crc32c_ragged.hip) or left to
                              // crc32c_long_kernel (crc32c_kernel.hip, which
                              // takes kLongBytes whatever the value)
  uint64_t* stamps;           // probe builds only: per-wave timestamps
  const uint32_t* count;      // optional device-side block count: the launch
                              // covers min(nblocks, *count) blocks (a count
                              // produced by an earlier kernel, e.g. an index
                              // parse); nullptr = nblocks
  void* sst_reports;          // kModeSstTable: lvkv_sst_report[sst_ntables]
  uint32_t sst_ntables;
  uint32_t run_units;         // with run_base: workgroup g of G walks blocks
  const uint32_t* run_base;   //   [run_base[gU/G], run_base[(g+1)U/G]) (the
                              //   last one to the count): runs balanced in
                              //   bytes when a unit is a fixed-size region
                              //   (the WAL's 32 KiB blocks); nullptr = equal
                              //   block counts per workgroup
  uint32_t fresh_desc;        // 1: offsets/lengths were written by this same
                              //   launch (vector loads after an acquire)
  uint32_t* log_first_bad;    // kModeLogStaged: per 32 KiB block (atomicMin)
  int32_t general_cfg;        // host side: kernel of general-layout batches
  int32_t log_cfg;            //   and of WAL records (launch_crc32c_general);
                              //   the device context's choice, never read
                              //   by a kernel
};

// Whole-SSTable verify forms (launch_sst_tables, lvkv_sst_table.hip).
enum : int { kSstFormTwo = 0, kSstFormFused = 1, kSstFormSpec = 2 };

// "filter." + FilterPolicy::Name() (table/table.cc:100-101), the metaindex
// key the whole-SSTable verify looks for; len 0: no filter policy.
constexpr uint32_t kMaxFilterKey = 7 + LVKV_SST_MAX_POLICY_NAME;
struct FilterKey {
  uint32_t len;
  uint8_t key[kMaxFilterKey + 1];
};

// Arguments of the uniform-layout kernel (crc32c_uniform.hip): nblocks
// blocks of `length` bytes at base + i*stride, every block END 4-byte aligned.
struct UniformArgs {
  const uint8_t* base;
  uint64_t stride;
  uint32_t* out;              // nblocks u32 (masked if `mask`)
  const uint32_t* lane_tab;   // kLaneTabDwords, LDS order (loaded per launch)
  const uint32_t* lane_cols;  // kLaneColDwords (compact kernel generates the
                              // lane tables from these)
  uint64_t* stamps;           // probe builds only
  const uint32_t* zpow;       // kZPowDwords (Z_{2^j} byte tables)
  uint32_t length;            // >= 4
  uint32_t init;
  uint32_t nblocks;
  uint32_t mask;
  uint32_t ngroups;           // workgroups of the launch (engine dispatches)
  uint32_t zcol[32];          // zcol[k] = Z_256(1 << k): the row tables are
                              // generated in-kernel from these columns
};

// Arguments of the engine's general-layout kernels (lvkv_ek_ragged*,
// lvkv_engine_kernels.hip): the HIP path's KernelArgs plus what
// launch_crc32c_ragged passes beside it, and the grid size (the engine's
// dispatches read no hidden kernel arguments).
struct EngineRaggedArgs {
  KernelArgs k;
  const uint32_t* zpow;
  const uint32_t* lane_cols;
  uint32_t ngroups;
  uint32_t pad_;
};

}  // namespace lvkv

#endif  // LVKV_KERNEL_ARGS_H_
