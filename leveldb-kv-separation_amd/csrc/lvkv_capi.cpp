// C-ABI of the batched CRC32C engine (declarations: include/lvkv_crc32c.h).
//
// Device state per HIP device (tables, CU count, staging for the host API) is
// created once, lazily, under std::call_once; the per-call paths take no lock
// and allocate nothing, so device-resident calls can be captured in a graph.
// Errors are return codes: this library backs a -fno-exceptions caller
// (reference CMakeLists.txt:71-77) and never throws or aborts.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <unordered_map>
#include <mutex>
#include <thread>
#include <vector>

#include "lvkv_crc32c.h"
#include "lvkv_kernel_args.h"
#include "lvkv_snappy.h"
#include "lvkv_tables.h"

namespace lvkv {

hipError_t launch_crc32c_batch(const KernelArgs& args, bool uniform_aligned,
                               int num_groups, hipStream_t stream);
hipError_t launch_crc32c_general(const KernelArgs& a, int cus, hipStream_t stream);
#ifdef LVKV_PROBE_BUILD
extern uint64_t* g_log_stamps;
extern uint64_t* g_asm_stamps;
extern uint64_t* g_sst_stamps;
extern uint32_t g_log_knobs;
extern uint64_t* g_zstd_stamps;
extern uint64_t* g_zstdc_stamps;
hipError_t launch_crc32c_probe(const KernelArgs& args, int variant,
                               int num_groups, hipStream_t stream);
hipError_t launch_read_bw(const void* p, uint64_t bytes, uint32_t* out,
                          int num_groups, hipStream_t stream);
#endif
hipError_t launch_crc32c_uniform(const UniformArgs& args, int variant,
                                 int num_groups, hipStream_t stream);
// Lane tables loaded first and written with the row tables (no end barrier),
// chain A's loads issued before the row-table fill: the fastest schedule
// measured (tools/probe.py v780; profiles/).
constexpr int kSmallProductionVariant = 4 | 8;
hipError_t launch_crc32c_uniform_small(const UniformArgs& args, int variant,
                                       int num_groups, hipStream_t stream);
hipError_t launch_crc32c_compact(const UniformArgs& args, int cfg, int num_groups,
                                 hipStream_t stream);
size_t log_gather_scratch_bytes(size_t capacity);
hipError_t launch_log_gather(const uint8_t* file, const uint64_t* hdr_off, size_t capacity,
                             const lvkv_log_report* phys, const lvkv_log_record* recs,
                             uint32_t rec_cap, const lvkv_log_read_report* read, uint8_t* out,
                             uint64_t out_cap, uint64_t* rec_pos, void* look, uint32_t tag,
                             int cus, hipStream_t stream);
hipError_t launch_sst_tables(const uint8_t* file, const uint64_t* toff, const uint64_t* tsize,
                             uint64_t single_size, uint32_t ntables, uint64_t* d_off,
                             uint32_t* d_size, uint32_t* d_actual, uint8_t* d_status,
                             uint32_t capacity, lvkv_sst_report* reports, const FilterKey& fk,
                             uint32_t gen, const KernelArgs& verify, const uint32_t* zpow,
                             const uint32_t* lane_cols, int groups, int form,
                             hipStream_t stream);
hipError_t launch_log_blocks(const uint8_t* file, uint64_t size, uint64_t* hdr_off,
                             uint32_t* actual, uint8_t* rec_status, uint32_t capacity,
                             uint8_t* block_status, uint32_t* block_drop, lvkv_log_report* r,
                             const uint32_t* zpow, const uint32_t* lane_cols, int cus,
                             void* scratch, uint32_t* events, uint64_t* item_off,
                             hipStream_t stream);
size_t log_scratch_bytes(uint64_t size, uint32_t capacity, int cus);
hipError_t launch_log_assemble(const uint32_t* events, const uint64_t* item_off,
                               const uint64_t* hdr_off, const lvkv_log_report* phys,
                               uint64_t size, uint32_t capacity, uint64_t initial_offset,
                               lvkv_log_record* recs, uint32_t rec_cap,
                               lvkv_log_corruption* reps, uint32_t rep_cap,
                               lvkv_log_read_report* out, void* scratch, hipStream_t stream);
size_t log_asm_scratch_bytes(size_t max_items);
hipError_t launch_crc32c_long(const KernelArgs& args, const uint32_t* zpow,
                              const uint32_t* lane_cols, int num_groups, hipStream_t stream);
hipError_t launch_snappy_compress(const uint8_t* src, const uint64_t* src_off,
                                  const uint32_t* src_len, uint8_t* dst, const uint64_t* dst_off,
                                  uint32_t* dst_len, uint8_t* status, uint32_t nblocks,
                                  uint32_t max_len, hipStream_t stream);
hipError_t launch_snappy_uncompress(const uint8_t* src, const uint64_t* src_off,
                                    const uint32_t* src_len, uint8_t* dst, const uint64_t* dst_off,
                                    const uint32_t* dst_cap, uint32_t* out_len, uint8_t* status,
                                    uint32_t nblocks, uint32_t max_ulen, hipStream_t stream);
uint64_t snappy_write_stride(uint32_t max_len);
hipError_t launch_sst_write_blocks(const uint8_t* raw, const uint64_t* raw_off,
                                   const uint32_t* raw_len, uint32_t nblocks, int compression,
                                   uint32_t max_len, uint8_t* scratch, uint8_t* file,
                                   uint64_t file_offset, uint64_t* hoff, uint32_t* hsize,
                                   uint8_t* type, uint64_t* end, int zstd_level,
                                   hipStream_t stream);
hipError_t launch_zstd_compress(const uint8_t* src, const uint64_t* src_off, const uint32_t* src_len,
                                uint8_t* dst, const uint64_t* dst_off, uint32_t* dst_len,
                                uint8_t* status, uint32_t nblocks, uint32_t max_len, int level,
                                uint64_t dst_stride, hipStream_t stream);
hipError_t launch_sst_read_blocks(const uint8_t* file, const uint64_t* hoff, const uint32_t* hsize,
                                  uint32_t nblocks, uint8_t* out, const uint64_t* out_off,
                                  const uint32_t* out_cap, uint32_t* out_len, uint8_t* status,
                                  const uint8_t* vstatus, uint32_t max_ulen, hipStream_t stream);
hipError_t launch_zstd_uncompress(const uint8_t* src, const uint64_t* src_off,
                                  const uint32_t* src_len, uint8_t* dst, const uint64_t* dst_off,
                                  const uint32_t* dst_cap, uint32_t* out_len, uint8_t* status,
                                  uint32_t* detail, uint32_t nblocks, uint32_t max_ulen,
                                  uint32_t block_mode, const uint8_t* vstatus, hipStream_t stream);
int compact_capacity(int cfg);
int compact_occupancy(int cfg);
// 8 waves x 3 chains, two workgroups per CU, generated lane tables
constexpr int kCompactProductionCfg = 9;
uint32_t cpu_crc32c_extend(uint32_t crc, const uint8_t* data, size_t n);
const char* cpu_crc32c_impl_name();

namespace {

constexpr int kMaxDevices = 64;
// Blocks per launch: the kernel indexes blocks with u32.
constexpr size_t kMaxBlocksPerLaunch = size_t{1} << 30;

// Host-API staging (double-buffered chunks).
constexpr size_t kStageBytes = size_t{64} << 20;
constexpr size_t kStageBlocks = 1u << 16;

struct Stage {
  uint8_t* h_data = nullptr;  // pinned
  uint8_t* d_data = nullptr;
  size_t cap = 0;
  uint64_t* h_off = nullptr;  // pinned descriptors
  uint32_t* h_len = nullptr;
  uint32_t* h_init = nullptr;
  uint32_t* h_out = nullptr;
  uint64_t* d_off = nullptr;
  uint32_t* d_len = nullptr;
  uint32_t* d_init = nullptr;
  uint32_t* d_out = nullptr;
  hipStream_t stream = nullptr;
  hipEvent_t done = nullptr;
  size_t first = 0, count = 0;  // blocks of the batch held by this stage
  bool busy = false;
};

struct DeviceCtx {
  std::once_flag once;
  int status = LVKV_ERR_NO_DEVICE;
  int groups = 0;  // one workgroup per CU
  uint32_t* d_tables = nullptr;
  uint32_t zcol[32];  // columns of Z_256 (uniform kernel's row tables)
  // kernels of general-layout batches and of WAL records
  // (launch_crc32c_general; lvkv_debug_set_general_kernel/_log_kernel)
  std::atomic<int> general_cfg{0};  // ragged cfg 0: 8 waves x 2 chains x 24 rows
  std::atomic<int> log_cfg{8};      // one workgroup per round of 32 small records
  // whole-SSTable verify form: 0 by size, 1 fused, 2 two launches,
  // 3 speculative (lvkv_debug_set_sst_form)
  std::atomic<int> sst_form{0};
  std::mutex host_mu;  // serialises lvkv_crc32c_batch_host per device
  // WAL verify scratch: a pool of buffers, each lent to one call at a time
  // (busy from acquire to the event recorded after the call's launches,
  // free once that event completes), on any stream
  std::mutex scratch_mu;
  struct Scratch {
    void* p = nullptr;
    size_t bytes = 0;
    hipEvent_t ev = nullptr;
    hipStream_t stream = nullptr;  // of its last call
    bool lent = false;
  };
  std::vector<Scratch> log_pool;
  bool stages_ready = false;
  Stage stage[2];
};

DeviceCtx g_dev[kMaxDevices];
thread_local int t_last_hip_error = 0;

int hip_fail(hipError_t e) {
  t_last_hip_error = static_cast<int>(e);
  return LVKV_ERR_HIP;
}

void init_ctx(DeviceCtx& c, int dev) {
  int ncu = 0;
  hipError_t e =
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  if (e != hipSuccess || ncu <= 0) {
    c.status = hip_fail(e);
    return;
  }
  static_assert(kZPowOffset == kRowTabDwords + kLaneTabDwords + kLaneColDwords, "layout");
  std::vector<uint32_t> tab(kTableDwords);
  build_row_table(tab.data());
  build_lane_table(tab.data() + kRowTabDwords);
  build_lane_columns(tab.data() + kRowTabDwords + kLaneTabDwords);
  build_zpow_tables(tab.data() + kZPowOffset);
  build_zmul_columns(tab.data() + kZPowOffset + kZPowDwords);
  void* p = nullptr;
  e = hipMalloc(&p, tab.size() * sizeof(uint32_t));
  if (e != hipSuccess) {
    c.status = hip_fail(e);
    return;
  }
  e = hipMemcpy(p, tab.data(), tab.size() * sizeof(uint32_t),
                hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    (void)hipFree(p);
    c.status = hip_fail(e);
    return;
  }
  c.d_tables = static_cast<uint32_t*>(p);
  const Gf2Op z256 = gf2_zero_advance(kRowBytes);
  for (int b = 0; b < 32; ++b) c.zcol[b] = z256.col[b];
  c.groups = ncu;
  c.status = LVKV_OK;
}

DeviceCtx* current_ctx(int* rc) {
  int count = 0;
  hipError_t e = hipGetDeviceCount(&count);
  if (e != hipSuccess || count <= 0) {
    t_last_hip_error = static_cast<int>(e);
    *rc = LVKV_ERR_NO_DEVICE;
    return nullptr;
  }
  int dev = -1;
  e = hipGetDevice(&dev);
  if (e != hipSuccess) {
    *rc = hip_fail(e);
    return nullptr;
  }
  if (dev < 0 || dev >= kMaxDevices) {
    *rc = LVKV_ERR_INVALID;
    return nullptr;
  }
  DeviceCtx& c = g_dev[dev];
  std::call_once(c.once, [&] { init_ctx(c, dev); });
  *rc = c.status;
  return c.status == LVKV_OK ? &c : nullptr;
}

}  // namespace

// The current device's tables (lvkv_engine.cpp shares them).
uint32_t* device_tables(int* rc) {
  DeviceCtx* c = current_ctx(rc);
  return c != nullptr ? c->d_tables : nullptr;
}

namespace {

UniformArgs uniform_args(const DeviceCtx& c, const KernelArgs& b) {
  UniformArgs u;
  memset(&u, 0, sizeof(u));
  u.base = b.base;
  u.stride = b.stride;
  u.out = b.out_crc;
  u.lane_tab = c.d_tables + kRowTabDwords;
  u.lane_cols = c.d_tables + kRowTabDwords + kLaneTabDwords;
  u.stamps = b.stamps;
  u.zpow = c.d_tables + kZPowOffset;
  u.length = b.length;
  u.init = b.init;
  u.nblocks = b.nblocks;
  u.mask = b.mask;
  memcpy(u.zcol, c.zcol, sizeof(u.zcol));
  return u;
}

int run_batch(KernelArgs a, size_t nblocks, hipStream_t stream) {
  if (nblocks == 0) return LVKV_OK;
  int rc = LVKV_OK;
  DeviceCtx* c = current_ctx(&rc);
  if (c == nullptr) return rc;
  a.row_tab = c->d_tables;
  a.lane_tab = c->d_tables + kRowTabDwords;
  a.general_cfg = c->general_cfg.load(std::memory_order_relaxed);
  a.log_cfg = c->log_cfg.load(std::memory_order_relaxed);
  for (size_t done = 0; done < nblocks;) {
    const size_t n = std::min(nblocks - done, kMaxBlocksPerLaunch);
    KernelArgs b = a;
    b.nblocks = static_cast<uint32_t>(n);
    if (a.offsets != nullptr) {
      b.offsets = a.offsets + done;
      if (a.lengths != nullptr) b.lengths = a.lengths + done;
    } else {
      b.base = a.base + done * a.stride;
    }
    if (a.inits != nullptr) b.inits = a.inits + done;
    if (a.out_crc != nullptr) b.out_crc = a.out_crc + done;
    if (a.out_status != nullptr) b.out_status = a.out_status + done;
    const size_t want = (n + kWavesPerGroup - 1) / kWavesPerGroup;
    const int groups = static_cast<int>(
        std::min<size_t>(static_cast<size_t>(c->groups), want));
    // Uniform layout whose every block END is 4-byte aligned: the dedicated
    // uniform kernel (crc32c_uniform.hip).
    const bool uni_aligned =
        a.offsets == nullptr && a.mode == kModeCompute && a.length >= 4 &&
        (a.stride % 4) == 0 &&
        ((reinterpret_cast<uintptr_t>(b.base) + a.length) % 4) == 0;
    hipError_t e;
    if (uni_aligned) {
      // Blocks of <= 16 rows (4 KiB + 252 B) that fit one round of the
      // compact-LDS kernel (two 512-thread workgroups per CU, 24 blocks
      // each): crc32c_compact.hip. At least 3 blocks per workgroup.
      const int cgroups = static_cast<int>(std::min<size_t>(
          static_cast<size_t>(c->groups) * compact_occupancy(kCompactProductionCfg),
          (n + 2) / 3));
      const size_t waves = static_cast<size_t>(groups) * kWavesPerGroup;
      if (a.length <= kRowsPerChunk * kRowBytes &&
          n <= static_cast<size_t>(cgroups) * compact_capacity(kCompactProductionCfg))
        e = launch_crc32c_compact(uniform_args(*c, b), kCompactProductionCfg, cgroups, stream);
      // One round per wave when every wave owns <= 3 single-chunk blocks.
      else if (a.length <= kRowsPerChunk * kRowBytes && n <= 3 * waves)
        e = launch_crc32c_uniform_small(uniform_args(*c, b), kSmallProductionVariant,
                                        groups, stream);
      else
        e = launch_crc32c_uniform(uniform_args(*c, b), 0, groups, stream);
    } else if (b.offsets != nullptr && b.mode != kModeLogVerify && b.mode != kModeLogFill) {
      // Blocks longer than kLongBytes go to one workgroup each (segments in
      // parallel) instead of one wave; the main kernel leaves them alone.
      b.long_split = kLongBytes;
      e = launch_crc32c_general(b, c->groups, stream);
    } else if (b.offsets != nullptr) {  // log headers
      b.long_split = kLogLongBytes;
      e = launch_crc32c_general(b, c->groups, stream);
    } else {  // uniform layout, block ends not 4-byte aligned
      e = launch_crc32c_batch(b, false, groups, stream);
    }
    if (e != hipSuccess) return hip_fail(e);
    done += n;
  }
  return LVKV_OK;
}

// "filter." + policy name (table.cc:100-101); false if the name is too long.
bool filter_key(const char* policy, FilterKey* fk) {
  memset(fk, 0, sizeof(*fk));
  if (policy == nullptr) return true;  // no filter policy: no filter block
  const size_t n = strlen(policy);
  if (n > LVKV_SST_MAX_POLICY_NAME) return false;
  memcpy(fk->key, "filter.", 7);
  memcpy(fk->key + 7, policy, n);
  fk->len = static_cast<uint32_t>(7 + n);
  return true;
}

// The one-launch SST verify forms for one table up to this size (larger
// indexes are faster on the two-launch form's 16-wave heads and its wide
// index launch). Multi-table calls take the speculative form (each CRC
// workgroup decodes its own share of one table's index) up to half as many
// tables as CUs, the two launches beyond.
constexpr uint64_t kFusedTableBytes = uint64_t{32} << 20;
constexpr size_t kFusedMaxTables = 256;

// kSstForm* for a call: lvkv_debug_set_sst_form's 1 (fused), 2 (two
// launches), 3 (speculative), or by size (0). The speculative form needs
// fewer tables than half its grid.
int sst_form(const DeviceCtx& c, bool by_size, size_t ntables = 1) {
  const int mode = c.sst_form.load(std::memory_order_relaxed);
  const bool spec_ok = ntables * 2 <= static_cast<size_t>(c.groups);
  switch (mode) {
    case 1: return ntables <= kFusedMaxTables ? kSstFormFused : kSstFormTwo;
    case 2: return kSstFormTwo;
    case 3: return spec_ok ? kSstFormSpec : kSstFormTwo;
  }
  return by_size && spec_ok ? kSstFormSpec : kSstFormTwo;
}

// Per-call tag of the multi-table placement words (never 0: fresh report
// memory is often zeroed).
uint32_t next_sst_generation() {
  static std::atomic<uint32_t> g{0};
  uint32_t v;
  do {
    v = g.fetch_add(1, std::memory_order_relaxed) + 1;
  } while (v == 0);
  return v;
}

KernelArgs blank_args() {
  KernelArgs a;
  memset(&a, 0, sizeof(a));
  return a;
}

// Zeroed arguments with the device context's tables and kernel choices.
KernelArgs ctx_args(const DeviceCtx& c) {
  KernelArgs a = blank_args();
  a.row_tab = c.d_tables;
  a.lane_tab = c.d_tables + kRowTabDwords;
  a.general_cfg = c.general_cfg.load(std::memory_order_relaxed);
  a.log_cfg = c.log_cfg.load(std::memory_order_relaxed);
  return a;
}

// A WAL verify scratch buffer of at least `bytes` for one call on `stream`.
// A buffer whose last call has finished (its event completed; never
// recorded counts as completed) is taken as is; else one last used on this
// same stream, or, with four buffers in the pool, any big enough idle one, is
// taken behind its event (hipStreamWaitEvent: the new call starts after the
// old one ends, a no-op on the same stream). When none is big enough, an idle
// buffer is regrown in place (after its last call has ended: its event is
// synchronised before the free) or, below four buffers, one is added; the
// pool exceeds four only while every buffer is lent to a call in progress on
// another thread. A new buffer's counters (bytes [0, 32)) are zeroed on
// `stream`; every call leaves them at 0. Not capturable: a graph would replay
// the counters unzeroed. The buffers live as long as the process (the HIP
// runtime may be gone by the time static destructors run).
hipError_t log_scratch_acquire(DeviceCtx& c, hipStream_t stream, size_t bytes, void** out,
                               size_t* slot) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  hipError_t e = hipStreamIsCapturing(stream, &cs);
  if (e != hipSuccess) return e;
  if (cs != hipStreamCaptureStatusNone) return hipErrorStreamCaptureUnsupported;
  std::unique_lock<std::mutex> lk(c.scratch_mu);
  constexpr size_t kPoolMax = 4;
  size_t same = SIZE_MAX, any = SIZE_MAX, idle_small = SIZE_MAX, busy_small = SIZE_MAX;
  for (size_t i = 0; i < c.log_pool.size(); ++i) {
    auto& b = c.log_pool[i];
    if (b.lent) continue;
    const bool finished = hipEventQuery(b.ev) == hipSuccess;
    if (b.bytes < bytes) {
      if (finished)
        idle_small = i;
      else
        busy_small = i;
      continue;
    }
    if (finished) {
      b.lent = true;
      b.stream = stream;
      *out = b.p;
      *slot = i;
      return hipSuccess;
    }
    if (b.stream == stream) same = i;
    any = i;
  }
  const bool full = c.log_pool.size() >= kPoolMax;
  size_t pick = same != SIZE_MAX ? same : (full ? any : SIZE_MAX);
  if (pick != SIZE_MAX) {
    auto& b = c.log_pool[pick];
    if ((e = hipStreamWaitEvent(stream, b.ev, 0)) != hipSuccess) return e;
    b.lent = true;
    b.stream = stream;
    *out = b.p;
    *slot = pick;
    return hipSuccess;
  }
  // nothing big enough: regrow an idle buffer (a busy one once its call has
  // ended) when the pool is full, else add one
  if (idle_small == SIZE_MAX && full) idle_small = busy_small;
  if (idle_small == SIZE_MAX) {
    DeviceCtx::Scratch n;
    if ((e = hipEventCreateWithFlags(&n.ev, hipEventDisableTiming)) != hipSuccess) return e;
    c.log_pool.push_back(n);
    idle_small = c.log_pool.size() - 1;
  }
  // Take the slot out of the pool, then wait for its last call and
  // reallocate without the lock: other streams' acquires and releases on
  // this device go on meanwhile (the slot is addressed by index, since the
  // pool may grow).
  const size_t k = idle_small;
  void* old = c.log_pool[k].p;
  const hipEvent_t ev = c.log_pool[k].ev;
  c.log_pool[k].lent = true;
  c.log_pool[k].p = nullptr;
  c.log_pool[k].bytes = 0;
  lk.unlock();
  const size_t cap = std::max<size_t>(bytes, size_t{1} << 16);
  void* p = nullptr;
  if (old != nullptr) {
    e = hipEventSynchronize(ev);
    if (e == hipSuccess) e = hipFree(old);
  }
  if (e == hipSuccess) e = hipMalloc(&p, cap);
  if (e == hipSuccess) e = hipMemsetAsync(p, 0, 32, stream);
  lk.lock();
  auto& b = c.log_pool[k];
  if (e != hipSuccess) {
    if (p != nullptr) (void)hipFree(p);
    b.lent = false;  // empty: the next acquire allocates it afresh
    return e;
  }
  b.p = p;
  b.bytes = cap;
  b.stream = stream;
  *out = p;
  *slot = k;
  return hipSuccess;
}

// Hands the buffer back: busy until the work just launched on `stream` ends.
hipError_t log_scratch_release(DeviceCtx& c, size_t slot, hipStream_t stream) {
  std::lock_guard<std::mutex> lk(c.scratch_mu);
  auto& b = c.log_pool[slot];
  const hipError_t e = hipEventRecord(b.ev, stream);
  b.lent = false;
  return e;
}

// ---- host-resident pipeline ------------------------------------------

void free_stage(Stage& s) {
  if (s.h_data) (void)hipHostFree(s.h_data);
  if (s.d_data) (void)hipFree(s.d_data);
  s.h_data = s.d_data = nullptr;
  s.cap = 0;
}

int alloc_stage_data(Stage& s, size_t cap) {
  free_stage(s);
  hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&s.h_data), cap,
                               hipHostMallocDefault);
  if (e != hipSuccess) return hip_fail(e);
  e = hipMalloc(reinterpret_cast<void**>(&s.d_data), cap);
  if (e != hipSuccess) return hip_fail(e);
  s.cap = cap;
  return LVKV_OK;
}

int ensure_stages(DeviceCtx& c, size_t need_bytes) {
  const size_t cap = std::max(kStageBytes, (need_bytes + 4095) & ~size_t{4095});
  for (Stage& s : c.stage) {
    if (!c.stages_ready) {
      hipError_t e;
      if ((e = hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking)) !=
          hipSuccess)
        return hip_fail(e);
      if ((e = hipEventCreateWithFlags(&s.done, hipEventDisableTiming)) !=
          hipSuccess)
        return hip_fail(e);
      const size_t nb = kStageBlocks;
      if ((e = hipHostMalloc(reinterpret_cast<void**>(&s.h_off), nb * 8,
                             hipHostMallocDefault)) != hipSuccess ||
          (e = hipHostMalloc(reinterpret_cast<void**>(&s.h_len), nb * 4,
                             hipHostMallocDefault)) != hipSuccess ||
          (e = hipHostMalloc(reinterpret_cast<void**>(&s.h_init), nb * 4,
                             hipHostMallocDefault)) != hipSuccess ||
          (e = hipHostMalloc(reinterpret_cast<void**>(&s.h_out), nb * 4,
                             hipHostMallocDefault)) != hipSuccess ||
          (e = hipMalloc(reinterpret_cast<void**>(&s.d_off), nb * 8)) !=
              hipSuccess ||
          (e = hipMalloc(reinterpret_cast<void**>(&s.d_len), nb * 4)) !=
              hipSuccess ||
          (e = hipMalloc(reinterpret_cast<void**>(&s.d_init), nb * 4)) !=
              hipSuccess ||
          (e = hipMalloc(reinterpret_cast<void**>(&s.d_out), nb * 4)) !=
              hipSuccess)
        return hip_fail(e);
    }
    if (s.cap < cap) {
      int rc = alloc_stage_data(s, cap);
      if (rc != LVKV_OK) return rc;
    }
  }
  c.stages_ready = true;
  return LVKV_OK;
}

// Copy blocks into the pinned buffer; big chunks are split over threads.
void pack_parallel(uint8_t* dst, const uint8_t* src, const uint64_t* src_off,
                   const uint32_t* len, const uint64_t* dst_off, size_t n,
                   size_t bytes) {
  const size_t kPerThread = size_t{8} << 20;
  unsigned hw = std::thread::hardware_concurrency();
  size_t nt = std::min<size_t>(hw ? hw : 1, 16);
  nt = std::min(nt, std::max<size_t>(1, bytes / kPerThread));
  auto work = [&](size_t t) {
    for (size_t i = t; i < n; i += nt)
      memcpy(dst + dst_off[i], src + src_off[i], len[i]);
  };
  if (nt <= 1) {
    work(0);
    return;
  }
  std::vector<std::thread> th;
  for (size_t t = 1; t < nt; ++t) th.emplace_back(work, t);
  work(0);
  for (auto& x : th) x.join();
}

int drain_stage(Stage& s, uint32_t* h_out) {
  if (!s.busy) return LVKV_OK;
  hipError_t e = hipEventSynchronize(s.done);
  s.busy = false;
  if (e != hipSuccess) return hip_fail(e);
  memcpy(h_out + s.first, s.h_out, s.count * sizeof(uint32_t));
  return LVKV_OK;
}

}  // namespace
}  // namespace lvkv

using namespace lvkv;

extern "C" {

uint32_t lvkv_crc32c_extend(uint32_t init_crc, const char* data, size_t n) {
  return cpu_crc32c_extend(init_crc, reinterpret_cast<const uint8_t*>(data), n);
}

uint32_t lvkv_crc32c_value(const char* data, size_t n) {
  return cpu_crc32c_extend(0, reinterpret_cast<const uint8_t*>(data), n);
}

uint32_t lvkv_crc32c_mask(uint32_t crc) {
  return ((crc >> 15) | (crc << 17)) + kMaskDelta;
}

uint32_t lvkv_crc32c_unmask(uint32_t masked_crc) {
  const uint32_t r = masked_crc - kMaskDelta;
  return (r >> 17) | (r << 15);
}

int lvkv_crc32c_batch_device(const void* d_base, const uint64_t* d_offsets,
                             const uint32_t* d_lengths, const uint32_t* d_init,
                             uint32_t init, uint32_t* d_out, size_t nblocks,
                             uint32_t flags, void* stream) {
  if (nblocks == 0) return LVKV_OK;
  if (!d_base || !d_offsets || !d_lengths || !d_out) return LVKV_ERR_INVALID;
  KernelArgs a = blank_args();
  a.base = static_cast<const uint8_t*>(d_base);
  a.offsets = d_offsets;
  a.lengths = d_lengths;
  a.inits = d_init;
  a.init = init;
  a.out_crc = d_out;
  a.mode = kModeCompute;
  a.mask = (flags & LVKV_FLAG_MASK) ? 1u : 0u;
  return run_batch(a, nblocks, static_cast<hipStream_t>(stream));
}

int lvkv_crc32c_uniform_device(const void* d_base, uint64_t stride,
                               uint32_t length, uint32_t init, uint32_t* d_out,
                               size_t nblocks, uint32_t flags, void* stream) {
  if (nblocks == 0) return LVKV_OK;
  if (!d_base || !d_out) return LVKV_ERR_INVALID;
  KernelArgs a = blank_args();
  a.base = static_cast<const uint8_t*>(d_base);
  a.stride = stride;
  a.length = length;
  a.init = init;
  a.out_crc = d_out;
  a.mode = kModeCompute;
  a.mask = (flags & LVKV_FLAG_MASK) ? 1u : 0u;
  return run_batch(a, nblocks, static_cast<hipStream_t>(stream));
}

int lvkv_sst_verify_device(const void* d_file, const uint64_t* d_offsets,
                           const uint32_t* d_sizes, uint32_t* d_actual,
                           uint8_t* d_status, size_t nblocks, void* stream) {
  if (nblocks == 0) return LVKV_OK;
  if (!d_file || !d_offsets || !d_sizes || !d_actual || !d_status)
    return LVKV_ERR_INVALID;
  KernelArgs a = blank_args();
  a.base = static_cast<const uint8_t*>(d_file);
  a.offsets = d_offsets;
  a.lengths = d_sizes;
  a.out_crc = d_actual;
  a.out_status = d_status;
  a.mode = kModeSstVerify;
  return run_batch(a, nblocks, static_cast<hipStream_t>(stream));
}

int lvkv_sst_verify_table_device(const void* d_file, uint64_t file_size,
                                 uint64_t* d_offsets, uint32_t* d_sizes,
                                 uint32_t* d_actual, uint8_t* d_status, size_t capacity,
                                 const char* filter_policy, lvkv_sst_report* d_report,
                                 void* stream) {
  FilterKey fk;
  if (!d_file || !d_offsets || !d_sizes || !d_actual || !d_status || !d_report ||
      capacity == 0 || capacity > kMaxBlocksPerLaunch || !filter_key(filter_policy, &fk))
    return LVKV_ERR_INVALID;
  int rc = LVKV_OK;
  DeviceCtx* c = current_ctx(&rc);
  if (c == nullptr) return rc;
  KernelArgs a = ctx_args(*c);
  a.mode = kModeSstVerify;
  const hipError_t e = launch_sst_tables(
      static_cast<const uint8_t*>(d_file), nullptr, nullptr, file_size, 1, d_offsets, d_sizes,
      d_actual, d_status, static_cast<uint32_t>(capacity), d_report, fk, next_sst_generation(), a,
      c->d_tables + kZPowOffset, c->d_tables + kRowTabDwords + kLaneTabDwords, c->groups,
      sst_form(*c, file_size <= kFusedTableBytes), static_cast<hipStream_t>(stream));
  return e == hipSuccess ? LVKV_OK : hip_fail(e);
}

int lvkv_sst_verify_tables_device(const void* d_file, const uint64_t* d_table_off,
                                  const uint64_t* d_table_size, size_t ntables,
                                  uint64_t* d_offsets, uint32_t* d_sizes, uint32_t* d_actual,
                                  uint8_t* d_status, size_t capacity, const char* filter_policy,
                                  lvkv_sst_report* d_reports, void* stream) {
  if (ntables == 0) return LVKV_OK;
  FilterKey fk;
  if (!d_file || !d_table_off || !d_table_size || !d_offsets || !d_sizes || !d_actual ||
      !d_status || !d_reports || capacity == 0 || capacity > kMaxBlocksPerLaunch ||
      ntables > (size_t{1} << 20) || !filter_key(filter_policy, &fk))
    return LVKV_ERR_INVALID;
  int rc = LVKV_OK;
  DeviceCtx* c = current_ctx(&rc);
  if (c == nullptr) return rc;
  KernelArgs a = ctx_args(*c);
  a.mode = kModeSstVerify;
  const hipError_t e = launch_sst_tables(
      static_cast<const uint8_t*>(d_file), d_table_off, d_table_size, 0,
      static_cast<uint32_t>(ntables), d_offsets, d_sizes, d_actual, d_status,
      static_cast<uint32_t>(capacity), d_reports, fk, next_sst_generation(), a,
      c->d_tables + kZPowOffset,
      c->d_tables + kRowTabDwords + kLaneTabDwords, c->groups,
      sst_form(*c, true, ntables), static_cast<hipStream_t>(stream));
  return e == hipSuccess ? LVKV_OK : hip_fail(e);
}

int lvkv_log_verify_blocks_device(const void* d_file, uint64_t file_size,
                                  uint64_t* d_hdr_offsets, uint32_t* d_actual,
                                  uint8_t* d_rec_status, size_t capacity,
                                  uint8_t* d_block_status, uint32_t* d_block_drop,
                                  lvkv_log_report* d_report, void* stream) {
  if ((!d_file && file_size) || !d_hdr_offsets || !d_actual || !d_rec_status || !d_block_status ||
      !d_block_drop || !d_report || capacity == 0 || capacity > kMaxBlocksPerLaunch ||
      file_size > (uint64_t{1} << 46))
    return LVKV_ERR_INVALID;
  int rc = LVKV_OK;
  DeviceCtx* c = current_ctx(&rc);
  if (c == nullptr) return rc;
  const hipStream_t hs = static_cast<hipStream_t>(stream);
  void* scratch = nullptr;
  size_t slot = 0;
  hipError_t e = log_scratch_acquire(*c, hs, log_scratch_bytes(file_size, static_cast<uint32_t>(capacity), c->groups), &scratch, &slot);
  if (e == hipErrorStreamCaptureUnsupported) return LVKV_ERR_INVALID;
  if (e != hipSuccess) return hip_fail(e);
  e = launch_log_blocks(static_cast<const uint8_t*>(d_file), file_size, d_hdr_offsets, d_actual,
                        d_rec_status, static_cast<uint32_t>(capacity), d_block_status,
                        d_block_drop, d_report, c->d_tables + kZPowOffset,
                        c->d_tables + kRowTabDwords + kLaneTabDwords, c->groups, scratch, nullptr,
                        nullptr, hs);
  const hipError_t e2 = log_scratch_release(*c, slot, hs);
  if (e == hipSuccess) e = e2;
  return e == hipSuccess ? LVKV_OK : hip_fail(e);
}

int lvkv_log_read_device(const void* d_file, uint64_t file_size, uint64_t* d_hdr_offsets,
                         uint32_t* d_actual, uint8_t* d_rec_status, size_t capacity,
                         uint8_t* d_block_status, uint32_t* d_block_drop,
                         lvkv_log_report* d_report, lvkv_log_record* d_records,
                         size_t record_capacity, lvkv_log_corruption* d_reports,
                         size_t report_capacity, uint64_t initial_offset,
                         lvkv_log_read_report* d_read, void* stream) {
  if ((!d_file && file_size) || !d_hdr_offsets || !d_actual || !d_rec_status || !d_block_status ||
      !d_block_drop || !d_report || !d_read || (!d_records && record_capacity) ||
      (!d_reports && report_capacity) || capacity == 0 || capacity > kMaxBlocksPerLaunch ||
      record_capacity > kMaxBlocksPerLaunch || report_capacity > kMaxBlocksPerLaunch ||
      file_size > (uint64_t{1} << 46))
    return LVKV_ERR_INVALID;
  int rc = LVKV_OK;
  DeviceCtx* c = current_ctx(&rc);
  if (c == nullptr) return rc;
  const hipStream_t hs = static_cast<hipStream_t>(stream);
  // scratch: the verify's counters, the event stream (one u32 per candidate
  // record and per block) and the items' header offsets (u64 each), then the
  // logical layer's per-workgroup state
  const size_t nblocks = static_cast<size_t>((file_size + 32767) / 32768);
  const size_t ev_at =
      (log_scratch_bytes(file_size, static_cast<uint32_t>(capacity), c->groups) + 15) & ~size_t{15};
  const size_t off_at = (ev_at + (capacity + nblocks) * 4 + 15) & ~size_t{15};
  const size_t asm_at = (off_at + (capacity + nblocks) * 8 + 15) & ~size_t{15};
  void* scratch = nullptr;
  size_t slot = 0;
  hipError_t e = log_scratch_acquire(*c, hs, asm_at + log_asm_scratch_bytes(capacity + nblocks),
                                     &scratch, &slot);
  if (e == hipErrorStreamCaptureUnsupported) return LVKV_ERR_INVALID;
  if (e != hipSuccess) return hip_fail(e);
  uint8_t* sb = static_cast<uint8_t*>(scratch);
  uint32_t* events = reinterpret_cast<uint32_t*>(sb + ev_at);
  uint64_t* item_off = reinterpret_cast<uint64_t*>(sb + off_at);
  if (e == hipSuccess)
    e = launch_log_blocks(static_cast<const uint8_t*>(d_file), file_size, d_hdr_offsets,
                          d_actual, d_rec_status, static_cast<uint32_t>(capacity),
                          d_block_status, d_block_drop, d_report, c->d_tables + kZPowOffset,
                          c->d_tables + kRowTabDwords + kLaneTabDwords, c->groups, scratch,
                          events, item_off, hs);
  if (e == hipSuccess)
    e = launch_log_assemble(events, item_off, d_hdr_offsets, d_report, file_size,
                            static_cast<uint32_t>(capacity), initial_offset, d_records,
                            static_cast<uint32_t>(record_capacity), d_reports,
                            static_cast<uint32_t>(report_capacity), d_read, sb + asm_at, hs);
  const hipError_t e2 = log_scratch_release(*c, slot, hs);
  if (e == hipSuccess) e = e2;
  return e == hipSuccess ? LVKV_OK : hip_fail(e);
}

int lvkv_log_gather_device(const void* d_file, const uint64_t* d_hdr_offsets, size_t capacity,
                           const lvkv_log_report* d_report, const lvkv_log_record* d_records,
                           size_t record_capacity, const lvkv_log_read_report* d_read,
                           void* d_payload, uint64_t payload_capacity, uint64_t* d_record_pos,
                           void* stream) {
  if (!d_file || !d_hdr_offsets || !d_report || !d_read || (!d_records && record_capacity) ||
      (!d_payload && payload_capacity) || capacity == 0 || capacity > kMaxBlocksPerLaunch ||
      record_capacity > kMaxBlocksPerLaunch)
    return LVKV_ERR_INVALID;
  if (record_capacity == 0) return LVKV_OK;
  int rc = LVKV_OK;
  DeviceCtx* c = current_ctx(&rc);
  if (c == nullptr) return rc;
  const hipStream_t hs = static_cast<hipStream_t>(stream);
  void* scratch = nullptr;
  size_t slot = 0;
  // (the pool's buffers keep the verify's counters in bytes [0, 24), which
  // every call leaves at 0: the look-back slots go after them)
  hipError_t e =
      log_scratch_acquire(*c, hs, 32 + log_gather_scratch_bytes(capacity), &scratch, &slot);
  if (e == hipErrorStreamCaptureUnsupported) return LVKV_ERR_INVALID;
  if (e != hipSuccess) return hip_fail(e);
  // the look-back slots' tag: per call, 30 bits, never 0
  static std::atomic<uint32_t> tags{0};
  uint32_t tag;
  do {
    tag = (tags.fetch_add(1, std::memory_order_relaxed) + 1) & 0x3fffffffu;
  } while (tag == 0);
  e = launch_log_gather(static_cast<const uint8_t*>(d_file), d_hdr_offsets, capacity, d_report,
                        d_records, static_cast<uint32_t>(record_capacity), d_read,
                        static_cast<uint8_t*>(d_payload), payload_capacity, d_record_pos,
                        static_cast<uint8_t*>(scratch) + 32, tag, c->groups, hs);
  const hipError_t e2 = log_scratch_release(*c, slot, hs);
  if (e == hipSuccess) e = e2;
  return e == hipSuccess ? LVKV_OK : hip_fail(e);
}

int lvkv_sst_fill_trailers_device(void* d_file, const uint64_t* d_offsets,
                                  const uint32_t* d_sizes, uint32_t* d_crc, size_t nblocks,
                                  void* stream) {
  if (nblocks == 0) return LVKV_OK;
  if (!d_file || !d_offsets || !d_sizes) return LVKV_ERR_INVALID;
  KernelArgs a = blank_args();
  a.base = static_cast<const uint8_t*>(d_file);
  a.offsets = d_offsets;
  a.lengths = d_sizes;
  a.out_crc = d_crc;
  a.mode = kModeSstFill;
  return run_batch(a, nblocks, static_cast<hipStream_t>(stream));
}

int lvkv_log_fill_headers_device(void* d_file, const uint64_t* d_hdr_offsets, uint32_t* d_crc,
                                 size_t nrecords, void* stream) {
  if (nrecords == 0) return LVKV_OK;
  if (!d_file || !d_hdr_offsets) return LVKV_ERR_INVALID;
  KernelArgs a = blank_args();
  a.base = static_cast<const uint8_t*>(d_file);
  a.offsets = d_hdr_offsets;
  a.out_crc = d_crc;
  a.mode = kModeLogFill;
  return run_batch(a, nrecords, static_cast<hipStream_t>(stream));
}

int lvkv_log_verify_device(const void* d_file, const uint64_t* d_hdr_offsets,
                           uint32_t* d_actual, uint8_t* d_status,
                           size_t nrecords, void* stream) {
  if (nrecords == 0) return LVKV_OK;
  if (!d_file || !d_hdr_offsets || !d_actual || !d_status)
    return LVKV_ERR_INVALID;
  KernelArgs a = blank_args();
  a.base = static_cast<const uint8_t*>(d_file);
  a.offsets = d_hdr_offsets;
  a.out_crc = d_actual;
  a.out_status = d_status;
  a.mode = kModeLogVerify;
  return run_batch(a, nrecords, static_cast<hipStream_t>(stream));
}

size_t lvkv_snappy_max_compressed_length(size_t n) { return 32 + n + n / 6; }

int lvkv_snappy_compress_device(const void* d_src, const uint64_t* d_src_off,
                                const uint32_t* d_src_len, void* d_dst,
                                const uint64_t* d_dst_off, uint32_t* d_dst_len,
                                uint8_t* d_status, size_t nblocks, uint32_t max_len,
                                void* stream) {
  if (nblocks == 0) return LVKV_OK;
  if (!d_src || !d_src_off || !d_src_len || !d_dst || !d_dst_off || !d_dst_len || !d_status ||
      nblocks > kMaxBlocksPerLaunch)
    return LVKV_ERR_INVALID;
  int rc = LVKV_OK;
  if (current_ctx(&rc) == nullptr) return rc;
  const hipError_t e = launch_snappy_compress(
      static_cast<const uint8_t*>(d_src), d_src_off, d_src_len, static_cast<uint8_t*>(d_dst),
      d_dst_off, d_dst_len, d_status, static_cast<uint32_t>(nblocks), max_len,
      static_cast<hipStream_t>(stream));
  return e == hipSuccess ? LVKV_OK : hip_fail(e);
}

int lvkv_snappy_uncompressed_length_device(const void* d_src, const uint64_t* d_src_off,
                                           const uint32_t* d_src_len, uint32_t* d_ulen,
                                           uint8_t* d_status, size_t nblocks, void* stream) {
  if (nblocks == 0) return LVKV_OK;
  if (!d_src || !d_src_off || !d_src_len || !d_ulen || !d_status ||
      nblocks > kMaxBlocksPerLaunch)
    return LVKV_ERR_INVALID;
  int rc = LVKV_OK;
  if (current_ctx(&rc) == nullptr) return rc;
  const hipError_t e = launch_snappy_uncompress(
      static_cast<const uint8_t*>(d_src), d_src_off, d_src_len, nullptr, nullptr, nullptr,
      d_ulen, d_status, static_cast<uint32_t>(nblocks), 0, static_cast<hipStream_t>(stream));
  return e == hipSuccess ? LVKV_OK : hip_fail(e);
}

int lvkv_snappy_uncompress_device(const void* d_src, const uint64_t* d_src_off,
                                  const uint32_t* d_src_len, void* d_dst,
                                  const uint64_t* d_dst_off, const uint32_t* d_dst_cap,
                                  uint32_t* d_out_len, uint8_t* d_status, size_t nblocks,
                                  uint32_t max_ulen, void* stream) {
  if (nblocks == 0) return LVKV_OK;
  if (!d_src || !d_src_off || !d_src_len || !d_dst || !d_dst_off || !d_dst_cap || !d_out_len ||
      !d_status || nblocks > kMaxBlocksPerLaunch || max_ulen > LVKV_SNAPPY_MAX_BLOCK)
    return LVKV_ERR_INVALID;
  int rc = LVKV_OK;
  if (current_ctx(&rc) == nullptr) return rc;
  const hipError_t e = launch_snappy_uncompress(
      static_cast<const uint8_t*>(d_src), d_src_off, d_src_len, static_cast<uint8_t*>(d_dst),
      d_dst_off, d_dst_cap, d_out_len, d_status, static_cast<uint32_t>(nblocks), max_ulen,
      static_cast<hipStream_t>(stream));
  return e == hipSuccess ? LVKV_OK : hip_fail(e);
}

size_t lvkv_sst_write_scratch_bytes(size_t nblocks, uint32_t max_len) {
  return nblocks * (snappy_write_stride(max_len) + 5);
}

size_t lvkv_zstd_compress_bound(size_t n) {
  return n + (n >> 8) + (n < (size_t{128} << 10) ? ((size_t{128} << 10) - n) >> 11 : 0);
}

int lvkv_zstd_compress_device(const void* d_src, const uint64_t* d_src_off,
                              const uint32_t* d_src_len, void* d_dst, const uint64_t* d_dst_off,
                              uint32_t* d_dst_len, uint8_t* d_status, size_t nblocks,
                              uint32_t max_len, int level, void* stream) {
  if (nblocks == 0) return LVKV_OK;
  if (!d_src || !d_src_off || !d_src_len || !d_dst || !d_dst_off || !d_dst_len || !d_status ||
      nblocks > kMaxBlocksPerLaunch || max_len > LVKV_ZSTD_COMPRESS_MAX_BLOCK)
    return LVKV_ERR_INVALID;
  int rc = LVKV_OK;
  if (current_ctx(&rc) == nullptr) return rc;
  const hipError_t e = launch_zstd_compress(
      static_cast<const uint8_t*>(d_src), d_src_off, d_src_len, static_cast<uint8_t*>(d_dst),
      d_dst_off, d_dst_len, d_status, static_cast<uint32_t>(nblocks), max_len, level, 0,
      static_cast<hipStream_t>(stream));
  return e == hipSuccess ? LVKV_OK : hip_fail(e);
}

int lvkv_sst_write_blocks_device(const void* d_raw, const uint64_t* d_raw_off,
                                 const uint32_t* d_raw_len, size_t nblocks, int compression,
                                 uint32_t max_len, void* d_scratch, void* d_file,
                                 uint64_t file_offset, uint64_t* d_handle_off,
                                 uint32_t* d_handle_size, uint8_t* d_type, uint64_t* d_end,
                                 void* stream) {
  return lvkv_sst_write_blocks_level_device(d_raw, d_raw_off, d_raw_len, nblocks, compression, 1,
                                            max_len, d_scratch, d_file, file_offset, d_handle_off,
                                            d_handle_size, d_type, d_end, stream);
}

int lvkv_sst_write_blocks_level_device(const void* d_raw, const uint64_t* d_raw_off,
                                       const uint32_t* d_raw_len, size_t nblocks, int compression,
                                       int zstd_level, uint32_t max_len, void* d_scratch,
                                       void* d_file, uint64_t file_offset, uint64_t* d_handle_off,
                                       uint32_t* d_handle_size, uint8_t* d_type, uint64_t* d_end,
                                       void* stream) {
  if (!d_end || compression < 0 || compression > 2) return LVKV_ERR_INVALID;
  // kZstdCompression on the device: the ZSTD_fast levels (<= 2; 0 means 3)
  // and blocks the compressor's LDS plan holds
  if (compression == 2 &&
      (zstd_level == 0 || zstd_level > 2 || max_len > LVKV_ZSTD_COMPRESS_MAX_BLOCK))
    return LVKV_ERR_INVALID;
  if (nblocks == 0) {  // d_end = file_offset, by the layout kernel (no host pointer kept)
    int rc = LVKV_OK;
    if (current_ctx(&rc) == nullptr) return rc;
    const hipError_t e = launch_sst_write_blocks(nullptr, nullptr, nullptr, 0, compression, 0,
                                                 nullptr, nullptr, file_offset, nullptr, nullptr,
                                                 nullptr, d_end, zstd_level,
                                                 static_cast<hipStream_t>(stream));
    return e == hipSuccess ? LVKV_OK : hip_fail(e);
  }
  if (!d_raw || !d_raw_off || !d_raw_len || !d_file || !d_handle_off || !d_handle_size ||
      !d_type || (compression != 0 && !d_scratch) || nblocks > kMaxBlocksPerLaunch)
    return LVKV_ERR_INVALID;
  int rc = LVKV_OK;
  if (current_ctx(&rc) == nullptr) return rc;
  const hipStream_t hs = static_cast<hipStream_t>(stream);
  hipError_t e = launch_sst_write_blocks(
      static_cast<const uint8_t*>(d_raw), d_raw_off, d_raw_len, static_cast<uint32_t>(nblocks),
      compression, max_len, static_cast<uint8_t*>(d_scratch), static_cast<uint8_t*>(d_file),
      file_offset, d_handle_off, d_handle_size, d_type, d_end, zstd_level, hs);
  if (e != hipSuccess) return hip_fail(e);
  // the trailers: Mask(CRC32C(contents + type)) by the batch CRC kernel
  return lvkv_sst_fill_trailers_device(d_file, d_handle_off, d_handle_size, nullptr, nblocks,
                                       stream);
}

int lvkv_sst_read_blocks_device(const void* d_file, const uint64_t* d_handle_off,
                                const uint32_t* d_handle_size, size_t nblocks, int verify,
                                void* d_out, const uint64_t* d_out_off, const uint32_t* d_out_cap,
                                uint32_t* d_out_len, uint8_t* d_status, uint32_t max_ulen,
                                void* stream) {
  if (nblocks == 0) return LVKV_OK;
  if (!d_file || !d_handle_off || !d_handle_size || !d_out || !d_out_off || !d_out_cap ||
      !d_out_len || !d_status || nblocks > kMaxBlocksPerLaunch ||
      max_ulen > LVKV_SNAPPY_MAX_BLOCK)
    return LVKV_ERR_INVALID;
  int rc = LVKV_OK;
  if (current_ctx(&rc) == nullptr) return rc;
  if (verify) {  // the verdicts land in d_status (the CRCs in d_out_len) first
    rc = lvkv_sst_verify_device(d_file, d_handle_off, d_handle_size, d_out_len, d_status,
                                nblocks, stream);
    if (rc != LVKV_OK) return rc;
  }
  const hipStream_t hs = static_cast<hipStream_t>(stream);
  // raw and snappy blocks (zstd ones are left for the next launch)
  hipError_t e = launch_sst_read_blocks(
      static_cast<const uint8_t*>(d_file), d_handle_off, d_handle_size,
      static_cast<uint32_t>(nblocks), static_cast<uint8_t*>(d_out), d_out_off, d_out_cap,
      d_out_len, d_status, verify ? d_status : nullptr, max_ulen, hs);
  if (e != hipSuccess) return hip_fail(e);
  // kZstdCompression blocks whose checksum held (table/format.cc:138-155)
  e = launch_zstd_uncompress(static_cast<const uint8_t*>(d_file), d_handle_off, d_handle_size,
                             static_cast<uint8_t*>(d_out), d_out_off, d_out_cap, d_out_len,
                             d_status, nullptr, static_cast<uint32_t>(nblocks), max_ulen, 1,
                             verify ? d_status : nullptr, hs);
  return e == hipSuccess ? LVKV_OK : hip_fail(e);
}

int lvkv_zstd_uncompressed_length_device(const void* d_src, const uint64_t* d_src_off,
                                         const uint32_t* d_src_len, uint32_t* d_ulen,
                                         uint8_t* d_status, size_t nblocks, void* stream) {
  if (nblocks == 0) return LVKV_OK;
  if (!d_src || !d_src_off || !d_src_len || !d_ulen || !d_status ||
      nblocks > kMaxBlocksPerLaunch)
    return LVKV_ERR_INVALID;
  int rc = LVKV_OK;
  if (current_ctx(&rc) == nullptr) return rc;
  const hipError_t e = launch_zstd_uncompress(
      static_cast<const uint8_t*>(d_src), d_src_off, d_src_len, nullptr, nullptr, nullptr,
      d_ulen, d_status, nullptr, static_cast<uint32_t>(nblocks), 0, 0, nullptr,
      static_cast<hipStream_t>(stream));
  return e == hipSuccess ? LVKV_OK : hip_fail(e);
}

static int zstd_uncompress(const void* d_src, const uint64_t* d_src_off, const uint32_t* d_src_len,
                    void* d_dst, const uint64_t* d_dst_off, const uint32_t* d_dst_cap,
                    uint32_t* d_out_len, uint8_t* d_status, uint32_t* d_detail, size_t nblocks,
                    uint32_t max_ulen, void* stream) {
  if (nblocks == 0) return LVKV_OK;
  if (!d_src || !d_src_off || !d_src_len || !d_dst || !d_dst_off || !d_dst_cap || !d_out_len ||
      !d_status || nblocks > kMaxBlocksPerLaunch || max_ulen > LVKV_SNAPPY_MAX_BLOCK)
    return LVKV_ERR_INVALID;
  int rc = LVKV_OK;
  if (current_ctx(&rc) == nullptr) return rc;
  const hipError_t e = launch_zstd_uncompress(
      static_cast<const uint8_t*>(d_src), d_src_off, d_src_len, static_cast<uint8_t*>(d_dst),
      d_dst_off, d_dst_cap, d_out_len, d_status, d_detail, static_cast<uint32_t>(nblocks),
      max_ulen, 0, nullptr, static_cast<hipStream_t>(stream));
  return e == hipSuccess ? LVKV_OK : hip_fail(e);
}

int lvkv_zstd_uncompress_device(const void* d_src, const uint64_t* d_src_off,
                                const uint32_t* d_src_len, void* d_dst, const uint64_t* d_dst_off,
                                const uint32_t* d_dst_cap, uint32_t* d_out_len, uint8_t* d_status,
                                size_t nblocks, uint32_t max_ulen, void* stream) {
  return zstd_uncompress(d_src, d_src_off, d_src_len, d_dst, d_dst_off, d_dst_cap, d_out_len,
                         d_status, nullptr, nblocks, max_ulen, stream);
}

int lvkv_debug_zstd_uncompress_device(const void* d_src, const uint64_t* d_src_off,
                                      const uint32_t* d_src_len, void* d_dst,
                                      const uint64_t* d_dst_off, const uint32_t* d_dst_cap,
                                      uint32_t* d_out_len, uint8_t* d_status, uint32_t* d_detail,
                                      size_t nblocks, uint32_t max_ulen, void* stream) {
  return zstd_uncompress(d_src, d_src_off, d_src_len, d_dst, d_dst_off, d_dst_cap, d_out_len,
                         d_status, d_detail, nblocks, max_ulen, stream);
}

int lvkv_crc32c_batch_host(const void* h_base, const uint64_t* offsets,
                           const uint32_t* lengths, const uint32_t* init_arr,
                           uint32_t init, uint32_t* h_out, size_t nblocks,
                           uint32_t flags) {
  if (nblocks == 0) return LVKV_OK;
  if (!h_base || !offsets || !lengths || !h_out) return LVKV_ERR_INVALID;
  int rc = LVKV_OK;
  DeviceCtx* c = current_ctx(&rc);
  if (c == nullptr) return rc;
  std::lock_guard<std::mutex> lock(c->host_mu);
  size_t biggest = 0;
  for (size_t i = 0; i < nblocks; ++i)
    biggest = std::max<size_t>(biggest, lengths[i]);
  rc = ensure_stages(*c, biggest + 8);
  if (rc != LVKV_OK) return rc;
  // Every return leaves both stages idle: on an error the stage still in
  // flight is waited for and dropped, so no later call copies its results.
  struct StageGuard {
    DeviceCtx* c;
    ~StageGuard() {
      for (Stage& s : c->stage) {
        if (s.busy) (void)hipStreamSynchronize(s.stream);
        s.busy = false;
      }
    }
  } guard{c};
  const uint8_t* src = static_cast<const uint8_t*>(h_base);

  size_t next = 0;
  int k = 0;
  std::vector<uint64_t> src_off;
  while (next < nblocks) {
    Stage& s = c->stage[k];
    rc = drain_stage(s, h_out);
    if (rc != LVKV_OK) return rc;
    // Pack blocks so each one ENDS on a 4-byte boundary (the kernel's
    // aligned fast path), as many as fit.
    size_t n = 0, cursor = 0;
    src_off.clear();
    while (next + n < nblocks && n < kStageBlocks) {
      const size_t len = lengths[next + n];
      const size_t end = (cursor + len + 3) & ~size_t{3};
      if (end > s.cap) break;
      s.h_off[n] = end - len;
      s.h_len[n] = static_cast<uint32_t>(len);
      s.h_init[n] = init_arr ? init_arr[next + n] : init;
      src_off.push_back(offsets[next + n]);
      cursor = end;
      ++n;
    }
    pack_parallel(s.h_data, src, src_off.data(), s.h_len, s.h_off, n, cursor);
    hipError_t e;
    if ((e = hipMemcpyAsync(s.d_data, s.h_data, cursor, hipMemcpyHostToDevice,
                            s.stream)) != hipSuccess ||
        (e = hipMemcpyAsync(s.d_off, s.h_off, n * 8, hipMemcpyHostToDevice,
                            s.stream)) != hipSuccess ||
        (e = hipMemcpyAsync(s.d_len, s.h_len, n * 4, hipMemcpyHostToDevice,
                            s.stream)) != hipSuccess ||
        (e = hipMemcpyAsync(s.d_init, s.h_init, n * 4, hipMemcpyHostToDevice,
                            s.stream)) != hipSuccess)
      return hip_fail(e);
    rc = lvkv_crc32c_batch_device(s.d_data, s.d_off, s.d_len, s.d_init, 0,
                                  s.d_out, n, flags, s.stream);
    if (rc != LVKV_OK) return rc;
    if ((e = hipMemcpyAsync(s.h_out, s.d_out, n * 4, hipMemcpyDeviceToHost,
                            s.stream)) != hipSuccess ||
        (e = hipEventRecord(s.done, s.stream)) != hipSuccess)
      return hip_fail(e);
    s.first = next;
    s.count = n;
    s.busy = true;
    next += n;
    k ^= 1;
  }
  for (Stage& s : c->stage) {
    rc = drain_stage(s, h_out);
    if (rc != LVKV_OK) return rc;
  }
  return LVKV_OK;
}

const char* lvkv_strerror(int code) {
  switch (code) {
    case LVKV_OK:
      return "ok";
    case LVKV_ERR_INVALID:
      return "invalid argument";
    case LVKV_ERR_NO_DEVICE:
      return "no HIP device available (the batch API has no CPU fallback)";
    case LVKV_ERR_HIP:
      return "HIP runtime error";
    case LVKV_ERR_RANGE:
      return "block too large";
    default:
      return "unknown error";
  }
}

int lvkv_last_hip_error(void) { return t_last_hip_error; }

const char* lvkv_cpu_impl(void) { return cpu_crc32c_impl_name(); }

#ifdef LVKV_PROBE_BUILD
// Probe entry points (tools/probe/liblvkv_probe.so only).
void lvkv_debug_log_stamps(uint64_t* d_stamps) { g_log_stamps = d_stamps; }
void lvkv_debug_asm_stamps(uint64_t* d_stamps) { g_asm_stamps = d_stamps; }
void lvkv_debug_sst_stamps(uint64_t* d_stamps) { g_sst_stamps = d_stamps; }
void lvkv_debug_log_knobs(uint32_t knobs) { g_log_knobs = knobs; }
void lvkv_debug_zstd_stamps(uint64_t* d_stamps) { g_zstd_stamps = d_stamps; }
void lvkv_debug_zstdc_stamps(uint64_t* d_stamps) { g_zstdc_stamps = d_stamps; }
static uint64_t* g_debug_stamps = nullptr;

void lvkv_debug_set_stamps(uint64_t* d_stamps) { g_debug_stamps = d_stamps; }

int lvkv_debug_uniform_variant(int variant, int groups, const void* d_base,
                               uint64_t stride, uint32_t length,
                               uint32_t* d_out, size_t nblocks, void* stream) {
  if (nblocks == 0) return LVKV_OK;
  if (!d_base || !d_out || nblocks > kMaxBlocksPerLaunch) return LVKV_ERR_INVALID;
  int rc = LVKV_OK;
  DeviceCtx* c = current_ctx(&rc);
  if (c == nullptr) return rc;
  KernelArgs a = blank_args();
  a.base = static_cast<const uint8_t*>(d_base);
  a.stride = stride;
  a.length = length;
  a.out_crc = d_out;
  a.nblocks = static_cast<uint32_t>(nblocks);
  a.row_tab = c->d_tables;
  a.lane_tab = c->d_tables + kRowTabDwords;
  a.stamps = g_debug_stamps;
  if ((variant & 64) && g_debug_stamps == nullptr) return LVKV_ERR_INVALID;
  const int g = groups > 0 ? groups : c->groups;
  hipError_t e;
  if (variant & 256) {
    if (length < 4 || (stride % 4) != 0 ||
        ((reinterpret_cast<uintptr_t>(d_base) + length) % 4) != 0)
      return LVKV_ERR_INVALID;
    if (variant & 2048) {
      // compact-LDS kernel (crc32c_compact.hip), cfg in bits 16..22
      const int cfg = (variant >> 16) & 0x7f;
      const int gg = groups > 0 ? groups : c->groups * compact_occupancy(cfg);
      if (length > kRowsPerChunk * kRowBytes ||
          nblocks > static_cast<size_t>(gg) * compact_capacity(cfg))
        return LVKV_ERR_INVALID;
      e = launch_crc32c_compact(uniform_args(*c, a), cfg, gg, static_cast<hipStream_t>(stream));
    } else if (variant & 512) {
      if (length > kRowsPerChunk * kRowBytes ||
          nblocks > 3 * static_cast<size_t>(g) * kWavesPerGroup)
        return LVKV_ERR_INVALID;
      // debug bit 1024 -> kernel bit 256 (kSmallHalfA), 16384 -> 4096 (memory-only probe)
      // variant >= 1 << 16: kernel bits given directly in bits 16..30
      const int sv = variant >= (1 << 16)
                         ? (variant >> 16) | (variant & 64)
                         : (variant & 255) | ((variant & 1024) >> 2) | ((variant & 16384) >> 2);
      e = launch_crc32c_uniform_small(uniform_args(*c, a), sv, g,
                                      static_cast<hipStream_t>(stream));
    } else {
      e = launch_crc32c_uniform(uniform_args(*c, a), variant & 255, g,
                                static_cast<hipStream_t>(stream));
    }
  } else {
    e = launch_crc32c_probe(a, variant, g, static_cast<hipStream_t>(stream));
  }
  return e == hipSuccess ? LVKV_OK : hip_fail(e);
}

int lvkv_debug_read_bw(const void* d_data, uint64_t bytes, uint32_t* d_scratch,
                       int groups, void* stream) {
  if (!d_data || !d_scratch || (bytes & 15u)) return LVKV_ERR_INVALID;
  int rc = LVKV_OK;
  DeviceCtx* c = current_ctx(&rc);
  if (c == nullptr) return rc;
  const int g = groups != 0 ? groups : 8 * c->groups;
  hipError_t e = launch_read_bw(d_data, bytes, d_scratch, g,
                                static_cast<hipStream_t>(stream));
  return e == hipSuccess ? LVKV_OK : hip_fail(e);
}

#endif  // LVKV_PROBE_BUILD

// -1: crc32c_kernel.hip's persistent kernel for general-layout batches;
// 0..31: crc32c_ragged.hip cfgs (launch_crc32c_ragged). Timing only.
int lvkv_debug_set_general_kernel(int k) {
  if (k < -1 || k > 31) return LVKV_ERR_INVALID;
  int rc = LVKV_OK;
  DeviceCtx* c = current_ctx(&rc);
  if (c == nullptr) return rc;
  c->general_cfg.store(k, std::memory_order_relaxed);
  return LVKV_OK;
}

// The ragged cfg used for WAL records (8, 16, 24: small-record shapes).
int lvkv_debug_set_log_kernel(int k) {
  if (k < 0 || k > 31) return LVKV_ERR_INVALID;
  int rc = LVKV_OK;
  DeviceCtx* c = current_ctx(&rc);
  if (c == nullptr) return rc;
  c->log_cfg.store(k, std::memory_order_relaxed);
  return LVKV_OK;
}

// Whole-SSTable verify form: 0 by size (default), 1 always the fused launch,
// 2 always the two launches, 3 the speculative launch where it applies.
// Timing and tests.
int lvkv_debug_set_sst_form(int form) {
  if (form < 0 || form > 3) return LVKV_ERR_INVALID;
  int rc = LVKV_OK;
  DeviceCtx* c = current_ctx(&rc);
  if (c == nullptr) return rc;
  c->sst_form.store(form, std::memory_order_relaxed);
  return LVKV_OK;
}

int lvkv_device_groups(void) {
  int rc = LVKV_OK;
  DeviceCtx* c = current_ctx(&rc);
  return c ? c->groups : rc;
}

}  // extern "C"
