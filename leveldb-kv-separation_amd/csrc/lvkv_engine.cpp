// The AQL engine: batches dispatched straight into per-device hardware queues
// (include/lvkv_crc32c.h, lvkv_engine_*).
//
// Why (measured, tools/probe):
//   * a hipLaunchKernel costs 2.7-7 us of host time on this stack, as long as
//     the 10k x 4 KiB kernel itself (~7-9 us), so one-batch-per-call through
//     HIP is paced by the host; a submit here writes one 64-byte AQL packet
//     and its kernarg slot: ~1 us from Python;
//   * one AQL queue runs its dispatches one after another even without the
//     barrier bit (the next starts when the previous ends, timestamps in
//     profiles/), so the engine rotates dispatches over several hardware
//     queues: dispatch i goes to queue i % nq, and consecutive batches run
//     side by side;
//   * the production kernel takes one workgroup per CU (8 waves x 5 chains,
//     64 KiB LDS, half of a CU's waves), so the next dispatch's workgroups
//     are resident beside the running ones instead of waiting for them.
//
// The kernels come from a gfx950 code object embedded in this library
// (lvkv_engine_kernels.hip, assembled in by lvkv_engine_co.S) and loaded with
// the HSA loader. They read no hidden kernel arguments, so the kernarg
// segment is exactly UniformArgs.
//
// Memory model (gfx950: one L2 per XCD, not coherent with each other):
//   * kernargs live in VRAM, written through the PCIe BAR, then an HDP flush
//     (the path HIP's device kernargs take); a ring of kSlots slots, and a
//     slot is reused only after a fence covering its previous dispatch;
//   * every dispatch acquires at agent scope (inputs other agents wrote and
//     released are seen; LVKV_FLAG_SYSTEM_ACQUIRE: system scope, for input a
//     copy engine wrote into a reused buffer), each on its own queue, since a
//     submit's dispatches rotate over queues and run side by side; no
//     dispatch releases;
//   * lvkv_engine_wait (and the slot-reuse fence) puts a barrier-AND packet on
//     every queue with dispatches since the last fence, release at system
//     scope (none on a queue whose last dispatch was LVKV_FLAG_FINAL: that
//     one released at system scope itself): results are visible to the host,
//     to HIP streams and to copy engines after it.
// Engine dispatches are not ordered with HIP streams: synchronise the stream
// that produced the input before submitting.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <mutex>

#include "lvkv_crc32c.h"
#include "lvkv_kernel_args.h"
#include "lvkv_tables.h"

extern "C" const unsigned char lvkv_engine_co[];
extern "C" const unsigned char lvkv_engine_co_end[];

namespace lvkv {

uint32_t* device_tables(int* rc);  // lvkv_capi.cpp: per-device tables (d_tables)

namespace {

constexpr uint32_t kSlots = 1024;       // kernarg slots (dispatches between fences)
constexpr uint32_t kSlotBytes = 256;
// Kernel-argument cache (VRAM kernargs only): a dispatch whose arguments
// equal an earlier one's (a service cycling over a fixed set of buffers)
// points its packet at that earlier copy instead of writing the BAR and
// flushing the HDP again. kCacheSets sets of kCacheWays slots after the ring.
constexpr uint32_t kCacheSets = 256, kCacheWays = 4;
constexpr uint32_t kCacheSlots = kCacheSets * kCacheWays;
constexpr uint32_t kQueuePackets = 1024;
constexpr int kQueues = 4;              // hardware queues per engine
constexpr int kDefaultQueues = 3;       // in use by default (measured best)
constexpr uint32_t kProfSlots = 64;     // completion signals while profiling
constexpr uint32_t kProfLog = 4096;     // dispatch durations kept

struct EngineKernel {
  uint64_t object = 0;
  uint32_t kernarg_size = 0, group_size = 0, private_size = 0;
  uint32_t waves = 8, chains = 5, per_cu = 1;  // shape; per_cu = workgroups per CU
};

// Kernel-argument layouts of the engine's kernels.
enum ArgKind : uint32_t { kArgsUniform = 0, kArgsRagged = 1 };

// The engine's kernels (lvkv_engine_kernels.hip): symbol, timestamp build
// (nullptr: none), shape, argument layout. [0] is the production schedule of
// overlapped uniform batches, [1] of ordered ones; [2] and [3] walk
// general-layout batches.
struct KernelSpec {
  const char* name;
  const char* stamps;
  uint32_t waves, chains, per_cu;
  ArgKind kind;
};
constexpr KernelSpec kSpecs[] = {
    {"lvkv_ek_uniform.kd", "lvkv_ek_uniform_stamps.kd", 8, 5, 1, kArgsUniform},
    {"lvkv_ek_uniform_pair.kd", "lvkv_ek_uniform_pair_stamps.kd", 8, 3, 2, kArgsUniform},
    {"lvkv_ek_ragged.kd", nullptr, 8, 2, 2, kArgsRagged},
    {"lvkv_ek_ragged_small.kd", nullptr, 8, 4, 2, kArgsRagged},
    {"lvkv_ek_ragged_burst.kd", nullptr, 8, 4, 1, kArgsRagged},
    {"lvkv_ek_ragged_burst_small.kd", nullptr, 8, 6, 1, kArgsRagged},
};
constexpr int kNumSpecs = static_cast<int>(sizeof(kSpecs) / sizeof(kSpecs[0]));
constexpr int kNumUniformSpecs = 2;  // lvkv_engine_set_variant's choices
// general-layout kernels: persistent runs (two workgroups per CU, rounds of
// 16 / 32 blocks), and one round per dispatch (one workgroup per CU)
constexpr int kRaggedSpec = 2, kRaggedSmallSpec = 3, kBurstSpec = 4, kBurstSmallSpec = 5;
constexpr uint32_t kBurstRows = 17, kBurstSmallRows = 8;  // chunk rows of the SST / small shapes
static_assert(sizeof(EngineRaggedArgs) <= 256 && sizeof(UniformArgs) <= 256, "kernarg slot");

constexpr size_t args_size(ArgKind k) {
  return k == kArgsUniform ? sizeof(UniformArgs) : sizeof(EngineRaggedArgs);
}

struct AgentMatch {
  uint32_t domain, bdfid;
  hsa_agent_t agent;
  bool found;
};

hsa_status_t match_agent(hsa_agent_t agent, void* data) {
  AgentMatch* m = static_cast<AgentMatch*>(data);
  hsa_device_type_t type;
  if (hsa_agent_get_info(agent, HSA_AGENT_INFO_DEVICE, &type) != HSA_STATUS_SUCCESS ||
      type != HSA_DEVICE_TYPE_GPU)
    return HSA_STATUS_SUCCESS;
  uint32_t bdf = 0, dom = 0;
  if (hsa_agent_get_info(agent, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_BDFID), &bdf) !=
          HSA_STATUS_SUCCESS ||
      hsa_agent_get_info(agent, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_DOMAIN), &dom) !=
          HSA_STATUS_SUCCESS)
    return HSA_STATUS_SUCCESS;
  if (bdf == m->bdfid && dom == m->domain) {
    m->agent = agent;
    m->found = true;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

struct PoolFind {
  hsa_amd_memory_pool_t pool;
  bool found;
};

// The device's coarse-grained VRAM pool.
hsa_status_t find_vram_pool(hsa_amd_memory_pool_t pool, void* data) {
  hsa_amd_segment_t seg;
  uint32_t flags = 0;
  bool alloc = false;
  if (hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg) !=
          HSA_STATUS_SUCCESS ||
      seg != HSA_AMD_SEGMENT_GLOBAL)
    return HSA_STATUS_SUCCESS;
  if (hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags) !=
          HSA_STATUS_SUCCESS ||
      !(flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED))
    return HSA_STATUS_SUCCESS;
  if (hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_RUNTIME_ALLOC_ALLOWED,
                                   &alloc) != HSA_STATUS_SUCCESS ||
      !alloc)
    return HSA_STATUS_SUCCESS;
  PoolFind* f = static_cast<PoolFind*>(data);
  f->pool = pool;
  f->found = true;
  return HSA_STATUS_INFO_BREAK;
}

hsa_status_t find_cpu(hsa_agent_t agent, void* data) {
  hsa_device_type_t type;
  if (hsa_agent_get_info(agent, HSA_AGENT_INFO_DEVICE, &type) == HSA_STATUS_SUCCESS &&
      type == HSA_DEVICE_TYPE_CPU) {
    *static_cast<hsa_agent_t*>(data) = agent;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

// Fallback kernarg memory (system memory) when the BAR path is unavailable.
hsa_status_t find_kernarg_region(hsa_region_t region, void* data) {
  hsa_region_segment_t seg;
  if (hsa_region_get_info(region, HSA_REGION_INFO_SEGMENT, &seg) != HSA_STATUS_SUCCESS ||
      seg != HSA_REGION_SEGMENT_GLOBAL)
    return HSA_STATUS_SUCCESS;
  uint32_t flags = 0;
  if (hsa_region_get_info(region, HSA_REGION_INFO_GLOBAL_FLAGS, &flags) != HSA_STATUS_SUCCESS)
    return HSA_STATUS_SUCCESS;
  if (flags & HSA_REGION_GLOBAL_FLAG_KERNARG) {
    *static_cast<hsa_region_t*>(data) = region;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

std::once_flag g_hsa_once;
hsa_status_t g_hsa_status = HSA_STATUS_ERROR_NOT_INITIALIZED;

}  // namespace

struct Engine {
  int device = -1;
  int cus = 0;
  hsa_agent_t agent{};
  hsa_queue_t* queues[kQueues] = {};
  int nq = kDefaultQueues;
  int cur = 0;  // queue of the packet being written
  hsa_executable_t exe{};
  hsa_code_object_reader_t reader{};
  bool exe_ok = false, reader_ok = false;
  EngineKernel kern[kNumSpecs], kern_stamps[kNumSpecs];
  // a probe kernel loaded from a separate code object (tools/probe only)
  hsa_executable_t probe_exe{};
  hsa_code_object_reader_t probe_reader{};
  bool probe_exe_ok = false, probe_reader_ok = false, probe_on = false;
  bool probe_overlapped = false;  // the probe replaces overlapped (else ordered) dispatches' kernel
  EngineKernel probe;
  // fence scopes: a submission's first dispatch acquires at `dispatch_acq`;
  // the wait's barrier packets acquire/release at fence_acq/fence_rel
  // (LVKV_FLAG_SYSTEM_ACQUIRE raises it to system scope for one submission)
  int dispatch_acq = HSA_FENCE_SCOPE_AGENT;
  // (the fence acquires nothing: every later submission does its own
  // acquire; measured 2 us sooner than a system-scope acquire)
  int fence_acq = HSA_FENCE_SCOPE_NONE, fence_rel = HSA_FENCE_SCOPE_SYSTEM;
  int variant = 0;          // kernel of overlapped dispatches
  int ordered_variant = 1;  // kernel of ordered dispatches (the whole chip)
  int final_variant = -1;   // of LVKV_FLAG_FINAL dispatches (-1: as overlapped)
  uint8_t* kernarg = nullptr;     // (kSlots + kCacheSlots) x kSlotBytes
  bool kernarg_vram = false;      // BAR-written VRAM (else system memory)
  struct CachedArgs {             // host copy of a cached kernarg slot
    uint64_t hash = 0;
    uint64_t last = 0;            // 1 + index of the last dispatch that used it (0: empty)
    uint32_t size = 0;
    uint8_t bytes[kSlotBytes];
  };
  CachedArgs* ka_cache = nullptr;  // kCacheSlots
  uint64_t ka_hits = 0, ka_misses = 0;
  uint32_t* hdp_flush = nullptr;  // HDP_MEM_FLUSH_CNTL
  hsa_signal_t fence_sig{};       // barrier-AND fences, one decrement per queue
  bool fence_ok = false;
  // LVKV_FLAG_FINAL dispatches: each carries this completion signal (one
  // decrement) with a system-scope release, and the next fence needs no
  // barrier packet on a queue whose last dispatch is one of them
  hsa_signal_t fin_sig{};
  bool fin_ok = false;
  uint64_t q_last[kQueues] = {};   // 1 + index of the queue's last dispatch since the fence
  uint64_t q_final[kQueues] = {};  // 1 + index of its last FINAL dispatch

  uint64_t next = 0;    // dispatches submitted
  uint64_t fenced = 0;  // every dispatch before this index is known complete
  // probes
  uint64_t* stamps = nullptr;  // 8 u64 per wave, one area per dispatch
  uint64_t stamp_next = 0, stamp_areas = 0;
  bool profiling = false;
  hsa_signal_t prof_sig[kProfSlots];
  uint32_t nprof_sig = 0;
  bool prof_pending[kProfSlots] = {};
  double tick_us = 0;
  double prof_start[kProfLog];  // us, HSA system clock
  double prof_end[kProfLog];
  uint64_t prof_count = 0;
  uint32_t* d_tables = nullptr;
  uint32_t zcol[32];
  std::mutex mu;
  int ragged_spec = -1;     // lvkv_debug_engine_ragged_spec: -1 = by layout
  volatile int queue_error = 0;
  double stuck_s = 60.0;     // a wait gives up after this long without progress
  hsa_signal_t hold_sig{};   // lvkv_debug_engine_stall: queues blocked on it
  bool hold_ok = false;
};

namespace {

void queue_error_cb(hsa_status_t status, hsa_queue_t*, void* data) {
  static_cast<Engine*>(data)->queue_error = static_cast<int>(status);
}

void drop_probe(Engine& e) {
  if (e.probe_exe_ok) hsa_executable_destroy(e.probe_exe);
  if (e.probe_reader_ok) hsa_code_object_reader_destroy(e.probe_reader);
  e.probe_exe_ok = e.probe_reader_ok = e.probe_on = false;
}

int load_kernel(Engine& e, hsa_executable_t exe, const char* name, EngineKernel* k,
                size_t want_args = sizeof(UniformArgs)) {
  hsa_executable_symbol_t sym;
  if (hsa_executable_get_symbol_by_name(exe, name, &e.agent, &sym) != HSA_STATUS_SUCCESS)
    return LVKV_ERR_HIP;
  if (hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &k->object) !=
          HSA_STATUS_SUCCESS ||
      hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE,
                                     &k->kernarg_size) != HSA_STATUS_SUCCESS ||
      hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE,
                                     &k->group_size) != HSA_STATUS_SUCCESS ||
      hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE,
                                     &k->private_size) != HSA_STATUS_SUCCESS)
    return LVKV_ERR_HIP;
  // The kernarg segment must be exactly the argument struct: no hidden
  // arguments the engine would have to fill.
  if (k->kernarg_size != want_args || k->kernarg_size > kSlotBytes)
    return LVKV_ERR_HIP;
  return LVKV_OK;
}

void destroy(Engine* e) {
  for (hsa_queue_t* q : e->queues)
    if (q) hsa_queue_destroy(q);
  for (uint32_t i = 0; i < e->nprof_sig; ++i) hsa_signal_destroy(e->prof_sig[i]);
  if (e->fence_ok) hsa_signal_destroy(e->fence_sig);
  if (e->fin_ok) hsa_signal_destroy(e->fin_sig);
  if (e->hold_ok) hsa_signal_destroy(e->hold_sig);
  if (e->kernarg) {
    if (e->kernarg_vram)
      hsa_amd_memory_pool_free(e->kernarg);
    else
      hsa_memory_free(e->kernarg);
  }
  delete[] e->ka_cache;
  drop_probe(*e);
  if (e->exe_ok) hsa_executable_destroy(e->exe);
  if (e->reader_ok) hsa_code_object_reader_destroy(e->reader);
  delete e;
}

// Kernarg ring: VRAM through the BAR when the host may map it and the HDP
// flush register is exposed, else the agent's system-memory kernarg region.
bool alloc_kernargs(Engine& e) {
  PoolFind pf{{}, false};
  hsa_agent_t cpu{};
  hsa_amd_hdp_flush_t hdp{nullptr, nullptr};
  hsa_amd_agent_iterate_memory_pools(e.agent, find_vram_pool, &pf);
  hsa_iterate_agents(find_cpu, &cpu);
  void* p = nullptr;
  if (pf.found && cpu.handle != 0 &&
      hsa_agent_get_info(e.agent, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_HDP_FLUSH),
                         &hdp) == HSA_STATUS_SUCCESS &&
      hdp.HDP_MEM_FLUSH_CNTL != nullptr &&
      hsa_amd_memory_pool_allocate(pf.pool, (kSlots + kCacheSlots) * kSlotBytes, 0, &p) ==
          HSA_STATUS_SUCCESS) {
    if (hsa_amd_agents_allow_access(1, &cpu, nullptr, p) == HSA_STATUS_SUCCESS) {
      e.kernarg = static_cast<uint8_t*>(p);
      e.kernarg_vram = true;
      e.hdp_flush = hdp.HDP_MEM_FLUSH_CNTL;
      e.ka_cache = new Engine::CachedArgs[kCacheSlots];
      return true;
    }
    hsa_amd_memory_pool_free(p);
  }
  hsa_region_t karg{};
  karg.handle = 0;
  if (hsa_agent_iterate_regions(e.agent, find_kernarg_region, &karg) == HSA_STATUS_ERROR ||
      karg.handle == 0)
    return false;
  return hsa_memory_allocate(karg, kSlots * kSlotBytes, reinterpret_cast<void**>(&e.kernarg)) ==
         HSA_STATUS_SUCCESS;
}

int create(int device, Engine** out) {
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return LVKV_ERR_NO_DEVICE;
  if (device < 0 || device >= ndev) return LVKV_ERR_INVALID;
  std::call_once(g_hsa_once, [] { g_hsa_status = hsa_init(); });
  if (g_hsa_status != HSA_STATUS_SUCCESS) return LVKV_ERR_NO_DEVICE;
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof(bus), device) != hipSuccess) return LVKV_ERR_HIP;
  unsigned dom = 0, b = 0, d = 0, f = 0;
  if (sscanf(bus, "%x:%x:%x.%x", &dom, &b, &d, &f) != 4) return LVKV_ERR_HIP;
  AgentMatch m{dom, (b << 8) | (d << 3) | f, {}, false};
  hsa_iterate_agents(match_agent, &m);
  if (!m.found) return LVKV_ERR_NO_DEVICE;

  // The per-device tables of the HIP path (lane columns, zpow) serve the
  // engine too: allocate them on that device.
  int prev = -1;
  if (hipGetDevice(&prev) != hipSuccess) return LVKV_ERR_HIP;
  if (prev != device && hipSetDevice(device) != hipSuccess) return LVKV_ERR_HIP;
  int rc = LVKV_OK;
  uint32_t* tables = device_tables(&rc);
  int ncu = 0;
  if (rc == LVKV_OK &&
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess)
    rc = LVKV_ERR_HIP;
  if (prev != device) (void)hipSetDevice(prev);
  if (rc != LVKV_OK) return rc;

  Engine* e = new Engine();
  e->device = device;
  e->agent = m.agent;
  e->d_tables = tables;
  e->cus = ncu;
  const Gf2Op z = gf2_zero_advance(kRowBytes);
  memcpy(e->zcol, z.col, sizeof(e->zcol));
  uint64_t freq = 0;
  hsa_system_get_info(HSA_SYSTEM_INFO_TIMESTAMP_FREQUENCY, &freq);
  e->tick_us = freq ? 1e6 / static_cast<double>(freq) : 0.0;

  const size_t co_size = static_cast<size_t>(lvkv_engine_co_end - lvkv_engine_co);
  bool ok =
      hsa_code_object_reader_create_from_memory(lvkv_engine_co, co_size, &e->reader) ==
      HSA_STATUS_SUCCESS;
  e->reader_ok = ok;
  ok = ok && hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT,
                                       nullptr, &e->exe) == HSA_STATUS_SUCCESS;
  e->exe_ok = ok;
  ok = ok && hsa_executable_load_agent_code_object(e->exe, e->agent, e->reader, nullptr,
                                                   nullptr) == HSA_STATUS_SUCCESS;
  ok = ok && hsa_executable_freeze(e->exe, nullptr) == HSA_STATUS_SUCCESS;
  for (int i = 0; ok && i < kNumSpecs; ++i) {
    const size_t want = args_size(kSpecs[i].kind);
    ok = load_kernel(*e, e->exe, kSpecs[i].name, &e->kern[i], want) == LVKV_OK &&
         load_kernel(*e, e->exe, kSpecs[i].stamps ? kSpecs[i].stamps : kSpecs[i].name,
                     &e->kern_stamps[i], want) == LVKV_OK;
    for (EngineKernel* k : {&e->kern[i], &e->kern_stamps[i]}) {
      k->waves = kSpecs[i].waves;
      k->chains = kSpecs[i].chains;
      k->per_cu = kSpecs[i].per_cu;
    }
  }
  ok = ok && alloc_kernargs(*e);
  ok = ok && hsa_signal_create(0, 0, nullptr, &e->fence_sig) == HSA_STATUS_SUCCESS;
  e->fence_ok = ok;
  ok = ok && hsa_signal_create(0, 0, nullptr, &e->fin_sig) == HSA_STATUS_SUCCESS;
  e->fin_ok = ok;
  for (uint32_t i = 0; ok && i < kProfSlots; ++i) {
    ok = hsa_signal_create(0, 0, nullptr, &e->prof_sig[i]) == HSA_STATUS_SUCCESS;
    if (ok) e->nprof_sig = i + 1;
  }
  for (int i = 0; ok && i < kQueues; ++i)
    ok = hsa_queue_create(e->agent, kQueuePackets, HSA_QUEUE_TYPE_MULTI, queue_error_cb, e,
                          UINT32_MAX, UINT32_MAX, &e->queues[i]) == HSA_STATUS_SUCCESS &&
         // Timestamps are written only for packets that carry a completion
         // signal (profiled dispatches); the queue property is set before
         // the first packet because the packet processor may not see a later
         // change.
         hsa_amd_profiling_set_profiler_enabled(e->queues[i], 1) == HSA_STATUS_SUCCESS;
  if (!ok) {
    destroy(e);
    return LVKV_ERR_HIP;
  }
  *out = e;
  return LVKV_OK;
}

// A wait the engine gives up on: the device never hangs the caller. A
// queue error (the runtime's callback sets queue_error) ends every wait at
// once; a signal that does not move for e.stuck_s (60 s) marks the engine broken
// (queue_error = kStuck) and every later call returns LVKV_ERR_HIP.
constexpr int kStuck = -1;

double now_s() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return static_cast<double>(ts.tv_sec) + 1e-9 * static_cast<double>(ts.tv_nsec);
}

// Waits until `sig` < 1; false on a queue error or a stuck device.
bool wait_signal(Engine& e, hsa_signal_t sig) {
  // short active waits (a completion is normally µs away), each bounded so
  // the error flag and the deadline are re-checked
  const uint64_t hint = e.tick_us > 0 ? static_cast<uint64_t>(1000.0 / e.tick_us) : 1000000;
  double deadline = 0;
  hsa_signal_value_t seen = 0;
  for (;;) {
    const hsa_signal_value_t v =
        hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, hint, HSA_WAIT_STATE_ACTIVE);
    if (v < 1) return true;
    if (e.queue_error) return false;
    const double t = now_s();
    // the cutoff counts from the last progress: a fence over many queues
    // decrements its signal once per queue, and each decrement restarts it
    if (deadline == 0 || v != seen) {
      deadline = t + e.stuck_s;
      seen = v;
    } else if (t > deadline) {
      e.queue_error = kStuck;
      return false;
    }
  }
}

// Next free packet of queue e.cur (the caller holds e.mu); nullptr when the
// queue faulted or never drains.
void* packet_slot(Engine& e, uint64_t* idx) {
  hsa_queue_t* q = e.queues[e.cur];
  *idx = hsa_queue_add_write_index_screlease(q, 1);
  double deadline = 0;
  uint64_t seen = 0;
  for (uint64_t spin = 0; *idx - hsa_queue_load_read_index_scacquire(q) >= q->size; ++spin) {
    if (e.queue_error) return nullptr;
    if ((spin & 1023u) == 1023u) {
      const double t = now_s();
      const uint64_t rd = hsa_queue_load_read_index_relaxed(q);
      if (deadline == 0 || rd != seen) {  // the queue still advances: restart the cutoff
        deadline = t + e.stuck_s;
        seen = rd;
      } else if (t > deadline) {
        e.queue_error = kStuck;
        return nullptr;
      }
    }
  }
  return static_cast<hsa_kernel_dispatch_packet_t*>(q->base_address) + (*idx & (q->size - 1));
}

void publish(Engine& e, void* p, uint16_t header, uint16_t setup, uint64_t idx) {
  __atomic_store_n(static_cast<uint32_t*>(p), header | (static_cast<uint32_t>(setup) << 16),
                   __ATOMIC_RELEASE);
  hsa_signal_store_screlease(e.queues[e.cur]->doorbell_signal,
                             static_cast<hsa_signal_value_t>(idx));
}

// Reads the finished profiled dispatch of signal slot s into the log.
void collect_profile(Engine& e, uint32_t s) {
  if (!e.prof_pending[s]) return;
  if (!wait_signal(e, e.prof_sig[s])) {
    e.prof_pending[s] = false;
    return;
  }
  hsa_amd_profiling_dispatch_time_t t{};
  const hsa_status_t st = hsa_amd_profiling_get_dispatch_time(e.agent, e.prof_sig[s], &t);
  if (st == HSA_STATUS_SUCCESS) {
    const uint64_t i = e.prof_count++ % kProfLog;
    e.prof_start[i] = static_cast<double>(t.start) * e.tick_us;
    e.prof_end[i] = static_cast<double>(t.end) * e.tick_us;
  }
  e.prof_pending[s] = false;
}

// Every dispatch so far complete and its results visible to the host and to
// copy engines. A queue whose last dispatch since the previous fence was a
// LVKV_FLAG_FINAL one needs nothing more (that dispatch starts after the
// queue's earlier ones end and releases at system scope into fin_sig); every
// other queue with dispatches since then gets a barrier-AND packet with the
// barrier bit (it completes after every earlier packet of its queue and
// releases at system scope into fence_sig). Then the host spins on both.
// Caller holds e.mu. LVKV_ERR_HIP if a queue faulted or the device stopped
// (the wait ends instead of spinning forever).
int fence(Engine& e) {
  if (e.queue_error) return LVKV_ERR_HIP;
  int need = 0;
  for (int q = 0; q < kQueues; ++q)
    if (e.q_last[q] != 0 && e.q_final[q] != e.q_last[q]) ++need;
  hsa_signal_store_relaxed(e.fence_sig, need);
  const int keep = e.cur;
  for (int q = 0; q < kQueues; ++q) {
    if (e.q_last[q] == 0 || e.q_final[q] == e.q_last[q]) continue;
    e.cur = q;
    uint64_t idx;
    hsa_barrier_and_packet_t* p = static_cast<hsa_barrier_and_packet_t*>(packet_slot(e, &idx));
    if (p == nullptr) {
      e.cur = keep;
      return LVKV_ERR_HIP;
    }
    p->reserved0 = 0;
    p->reserved1 = 0;
    for (int i = 0; i < 5; ++i) p->dep_signal[i].handle = 0;
    p->reserved2 = 0;
    p->completion_signal = e.fence_sig;
    const uint16_t header =
        static_cast<uint16_t>((HSA_PACKET_TYPE_BARRIER_AND << HSA_PACKET_HEADER_TYPE) |
                              (1 << HSA_PACKET_HEADER_BARRIER) |
                              (e.fence_acq << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                              (e.fence_rel << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE));
    publish(e, p, header, 0, idx);
  }
  e.cur = keep;
  if (need && !wait_signal(e, e.fence_sig)) return LVKV_ERR_HIP;
  if (!wait_signal(e, e.fin_sig)) return LVKV_ERR_HIP;
  for (int q = 0; q < kQueues; ++q) e.q_last[q] = e.q_final[q] = 0;
  e.fenced = e.next;
  // oldest first: dispatch n used slot n % kProfSlots
  for (uint32_t i = 0; i < kProfSlots; ++i)
    collect_profile(e, static_cast<uint32_t>((e.next + i) % kProfSlots));
  return e.queue_error ? LVKV_ERR_HIP : LVKV_OK;
}

// The kernarg copy dispatch n points at: a cached slot holding exactly
// args[0, size) (its BAR write and HDP flush done by an earlier dispatch), a
// cache slot no unfinished dispatch uses (written now), or ring slot
// n % kSlots (written now). Caller holds e.mu.
uint8_t* kernarg_slot(Engine& e, uint64_t n, const void* args, size_t size) {
  uint8_t* ka = e.kernarg + static_cast<size_t>(n % kSlots) * kSlotBytes;
  if (e.kernarg_vram) {
    // FNV-1a over the argument bytes picks the set
    uint64_t h = 1469598103934665603ull;
    const uint8_t* b = static_cast<const uint8_t*>(args);
    for (size_t i = 0; i < size; ++i) h = (h ^ b[i]) * 1099511628211ull;
    const uint32_t set = static_cast<uint32_t>(h % kCacheSets);
    Engine::CachedArgs* ways = e.ka_cache + static_cast<size_t>(set) * kCacheWays;
    int victim = -1;
    for (uint32_t w = 0; w < kCacheWays; ++w) {
      Engine::CachedArgs& c = ways[w];
      if (c.last != 0 && c.hash == h && c.size == size && memcmp(c.bytes, args, size) == 0) {
        c.last = n + 1;
        ++e.ka_hits;
        return e.kernarg + (kSlots + static_cast<size_t>(set) * kCacheWays + w) * kSlotBytes;
      }
      // a slot no unfinished dispatch reads: the least recently used
      if (c.last <= e.fenced && (victim < 0 || c.last < ways[victim].last)) victim = static_cast<int>(w);
    }
    ++e.ka_misses;
    if (victim >= 0) {
      Engine::CachedArgs& c = ways[victim];
      c.hash = h;
      c.size = static_cast<uint32_t>(size);
      c.last = n + 1;
      memcpy(c.bytes, args, size);
      ka = e.kernarg + (kSlots + static_cast<size_t>(set) * kCacheWays + victim) * kSlotBytes;
    }
  }
  memcpy(ka, args, size);
  if (e.kernarg_vram) {
    // BAR writes are write-combined and may sit in the HDP write cache: fence
    // them, flush the HDP and read the register back (the read completes
    // only behind the posted writes) before the packet can be seen.
    __builtin_ia32_sfence();
    *reinterpret_cast<volatile uint32_t*>(e.hdp_flush) = 1u;
    (void)*reinterpret_cast<volatile uint32_t*>(e.hdp_flush);
  }
  return ka;
}

// One kernel-dispatch packet of `ngroups` workgroups whose kernel arguments
// are args[0, size); the caller holds e.mu. queue < 0: dispatch n goes to
// queue n % nq (consecutive dispatches side by side); else that queue.
int dispatch(Engine& e, const EngineKernel& k, const void* args, size_t size, uint32_t ngroups,
             bool acquire, bool barrier, bool system_acquire, int queue = -1,
             bool final = false) {
  if (e.queue_error) return LVKV_ERR_HIP;
  const uint64_t n = e.next;
  // Kernarg slot n % kSlots was last used by dispatch n - kSlots.
  if (n - e.fenced >= kSlots && fence(e) != LVKV_OK) return LVKV_ERR_HIP;
  e.cur = queue >= 0 ? queue : static_cast<int>(n % static_cast<uint64_t>(e.nq));
  hsa_signal_t done{};
  // (profiled dispatches carry their own signals: FINAL is ignored then)
  final = final && !e.profiling;
  if (final) {
    hsa_signal_add_relaxed(e.fin_sig, 1);
    done = e.fin_sig;
    barrier = true;
  }
  if (e.profiling) {
    const uint32_t s = static_cast<uint32_t>(n % kProfSlots);
    collect_profile(e, s);
    hsa_signal_store_relaxed(e.prof_sig[s], 1);
    e.prof_pending[s] = true;
    done = e.prof_sig[s];
  }
  uint8_t* ka = kernarg_slot(e, n, args, size);
  uint64_t idx;
  hsa_kernel_dispatch_packet_t* p = static_cast<hsa_kernel_dispatch_packet_t*>(packet_slot(e, &idx));
  if (p == nullptr) return LVKV_ERR_HIP;
  const uint32_t wg = 64u * k.waves;
  p->workgroup_size_x = static_cast<uint16_t>(wg);
  p->workgroup_size_y = 1;
  p->workgroup_size_z = 1;
  p->reserved0 = 0;
  p->grid_size_x = ngroups * wg;
  p->grid_size_y = 1;
  p->grid_size_z = 1;
  p->private_segment_size = k.private_size;
  p->group_segment_size = k.group_size;
  p->kernel_object = k.object;
  p->kernarg_address = ka;
  p->reserved2 = 0;
  p->completion_signal = done;
  const uint16_t header = static_cast<uint16_t>(
      (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
      ((barrier ? 1 : 0) << HSA_PACKET_HEADER_BARRIER) |
      ((acquire ? (system_acquire ? HSA_FENCE_SCOPE_SYSTEM : e.dispatch_acq)
                 : HSA_FENCE_SCOPE_NONE)
       << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
      ((final ? HSA_FENCE_SCOPE_SYSTEM : HSA_FENCE_SCOPE_NONE)
       << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE));
  publish(e, p, header, 1u << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS, idx);
  e.q_last[e.cur] = n + 1;
  if (final) e.q_final[e.cur] = n + 1;
  e.next = n + 1;
  return LVKV_OK;
}

// A general-layout batch (KernelArgs as the HIP path builds it: offsets or
// the uniform stride, a mode) through the engine's ragged kernels; the
// same ordering and acquire rules as the uniform submit. The kernel, by the
// measurements of tools/probe/engine_shapes.py:
//   * blocks of more than 17 rows in a uniform layout (config 3's 32 KiB WAL
//     blocks): the persistent 8 x 2 x 24 walk (0.77 of 8 TB/s overlapped on
//     16,384 x 32 KiB);
//   * WAL records (log verify / fill), uniform blocks of up to 8 rows and
//     ragged batches submitted with LVKV_FLAG_SMALL_BLOCKS (the caller knows
//     its blocks are small: log::Writer's records): the persistent 8 x 4 x 8
//     walk (0.29 overlapped on 62,000 x 0-2000 B where the burst gets 0.21;
//     on SST-sized blocks it gets 0.50 against the burst's 0.63);
//   * other ragged batches (SST blocks, ~4.1 KiB, the sizes being unknown to
//     the host) and uniform blocks of 9-17 rows: the 8 x 4 x 17 burst, whose
//     batch is cut into dispatches of one round (cus x 32 blocks, one
//     workgroup per CU) rotating over the queues like separate batches, so
//     consecutive rounds overlap on the device (0.62-0.64 overlapped on
//     16,384 x 4271 B, the persistent walk 0.53).
int submit_general(Engine& eng, KernelArgs a, size_t nblocks, uint32_t flags) {
  Engine* e = &eng;
  if (nblocks == 0) return LVKV_OK;
  const bool log = a.mode == kModeLogVerify || a.mode == kModeLogFill;
  a.long_split = log ? kLogLongBytes : kLongBytes;
  a.row_tab = e->d_tables;
  a.lane_tab = e->d_tables + kRowTabDwords;
  std::lock_guard<std::mutex> lk(e->mu);
  const bool ordered = (flags & LVKV_FLAG_ORDERED) != 0;
  if (ordered && e->nq > 1 && e->fenced != e->next && fence(*e) != LVKV_OK) return LVKV_ERR_HIP;
  const int queue = ordered ? static_cast<int>(e->next % static_cast<uint64_t>(e->nq)) : -1;
  int spec;
  if (a.offsets == nullptr) {
    const uint64_t rows = (uint64_t{a.length} + 3u + 255u) / 256u;  // upper bound, any alignment
    spec = rows > kBurstRows ? kRaggedSpec : rows <= kBurstSmallRows ? kRaggedSmallSpec : kBurstSpec;
  } else {
    spec = log || (flags & LVKV_FLAG_SMALL_BLOCKS) ? kRaggedSmallSpec : kBurstSpec;
  }
  // An ordered batch runs alone: the burst's one-round dispatches would run
  // one after another (16k SST-sized blocks: 0.31 of 8 TB/s, against 0.44
  // for the persistent 8 x 2 x 24 walk in one dispatch)
  if (ordered && spec == kBurstSpec) spec = kRaggedSpec;
  if (e->ragged_spec >= 0) spec = e->ragged_spec;
  const EngineKernel& k = e->kern[spec];
  const uint64_t per_round = uint64_t{k.waves} * k.chains;
  const uint64_t max_groups = static_cast<uint64_t>(e->cus) * k.per_cu;
  const bool burst = spec == kBurstSpec || spec == kBurstSmallSpec;
  // the kernel indexes blocks with u32; a burst dispatch holds one round
  const uint64_t max_per = burst ? max_groups * per_round : uint64_t{1} << 30;
  for (uint64_t done = 0; done < nblocks;) {
    const uint64_t n = std::min<uint64_t>(nblocks - done, max_per);
    EngineRaggedArgs r;
    memset(&r, 0, sizeof(r));
    r.k = a;
    r.k.nblocks = static_cast<uint32_t>(n);
    if (a.offsets != nullptr) {
      r.k.offsets = a.offsets + done;
      if (a.lengths != nullptr) r.k.lengths = a.lengths + done;
    } else {
      r.k.base = a.base + done * a.stride;
    }
    if (a.inits != nullptr) r.k.inits = a.inits + done;
    if (a.out_crc != nullptr) r.k.out_crc = a.out_crc + done;
    if (a.out_status != nullptr) r.k.out_status = a.out_status + done;
    r.zpow = e->d_tables + kZPowOffset;
    r.lane_cols = e->d_tables + kRowTabDwords + kLaneTabDwords;
    r.ngroups = static_cast<uint32_t>(std::min(max_groups, (n + per_round - 1) / per_round));
    const int rc = dispatch(*e, k, &r, sizeof(r), r.ngroups, /*acquire=*/true,
                            /*barrier=*/ordered, (flags & LVKV_FLAG_SYSTEM_ACQUIRE) != 0, queue,
                            (flags & LVKV_FLAG_FINAL) != 0 && done + n == nblocks);
    if (rc != LVKV_OK) return rc;
    done += n;
  }
  return LVKV_OK;
}

}  // namespace
}  // namespace lvkv

using namespace lvkv;

extern "C" {

int lvkv_engine_create(int device, lvkv_engine** out) {
  if (out == nullptr) return LVKV_ERR_INVALID;
  Engine* e = nullptr;
  const int rc = create(device, &e);
  *out = reinterpret_cast<lvkv_engine*>(e);
  return rc;
}

void lvkv_engine_destroy(lvkv_engine* eng) {
  if (eng == nullptr) return;
  (void)lvkv_engine_wait(eng);
  destroy(reinterpret_cast<Engine*>(eng));
}

int lvkv_engine_crc32c_uniform(lvkv_engine* eng, const void* d_base, uint64_t stride,
                               uint32_t length, uint32_t init, uint32_t* d_out, size_t nblocks,
                               uint32_t flags) {
  if (eng == nullptr) return LVKV_ERR_INVALID;
  if (nblocks == 0) return LVKV_OK;
  if (!d_base || !d_out || nblocks > (size_t{1} << 40)) return LVKV_ERR_INVALID;
  Engine* e = reinterpret_cast<Engine*>(eng);
  if (length < 4 || length > kRowsPerChunk * kRowBytes || stride % 4 != 0 ||
      (reinterpret_cast<uintptr_t>(d_base) + length) % 4 != 0) {
    // beyond the burst kernel (> 16 rows, < 4 bytes, block ends not 4-byte
    // aligned): the general walk in its uniform layout
    KernelArgs a;
    memset(&a, 0, sizeof(a));
    a.base = static_cast<const uint8_t*>(d_base);
    a.stride = stride;
    a.length = length;
    a.init = init;
    a.out_crc = d_out;
    a.mode = kModeCompute;
    a.mask = (flags & LVKV_FLAG_MASK) ? 1u : 0u;
    return submit_general(*e, a, nblocks, flags);
  }
  std::lock_guard<std::mutex> lk(e->mu);
  const bool ordered = (flags & LVKV_FLAG_ORDERED) != 0;
  // An ordered batch runs alone: the other queues drain first (the barrier
  // bit orders a packet only within its own queue), all of its dispatches go
  // to ONE queue with the barrier bit, so they run one after another, and it
  // gets the kernel shaped for the whole chip.
  if (ordered && e->nq > 1 && e->fenced != e->next && fence(*e) != LVKV_OK) return LVKV_ERR_HIP;
  const int queue = ordered ? static_cast<int>(e->next % static_cast<uint64_t>(e->nq)) : -1;
  const int v = ordered ? e->ordered_variant
                : ((flags & LVKV_FLAG_FINAL) && e->final_variant >= 0) ? e->final_variant
                                                                      : e->variant;
  const EngineKernel& k = (e->probe_on && ordered != e->probe_overlapped) ? e->probe
                          : e->stamps                ? e->kern_stamps[v]
                                                     : e->kern[v];
  const uint64_t groups = static_cast<uint64_t>(e->cus) * k.per_cu;
  const uint64_t cap = groups * k.waves * k.chains;
  // A batch beyond one dispatch's capacity goes out as several dispatches of
  // equal size, rotating over the queues like separate batches.
  const uint64_t nd = (nblocks + cap - 1) / cap;
  const uint64_t per = nblocks / nd, extra = nblocks % nd;
  uint64_t done = 0;
  for (uint64_t i = 0; i < nd; ++i) {
    const uint64_t n = per + (i < extra ? 1 : 0);
    UniformArgs a;
    memset(&a, 0, sizeof(a));
    a.base = static_cast<const uint8_t*>(d_base) + done * stride;
    a.stride = stride;
    a.out = d_out + done;
    a.lane_tab = e->d_tables + kRowTabDwords;
    a.lane_cols = e->d_tables + kRowTabDwords + kLaneTabDwords;
    a.zpow = e->d_tables + kZPowOffset;
    a.length = length;
    a.init = init;
    a.nblocks = static_cast<uint32_t>(n);
    a.mask = (flags & LVKV_FLAG_MASK) ? 1u : 0u;
    // at least 3 blocks per workgroup (as the HIP path)
    a.ngroups = static_cast<uint32_t>(std::min<uint64_t>(groups, (n + 2) / 3));
    memcpy(a.zcol, e->zcol, sizeof(a.zcol));
    if (e->stamps) {
      const uint64_t area = groups * k.waves * 8;
      a.stamps = e->stamps + (e->stamp_next++ % e->stamp_areas) * area;
    }
    // every dispatch acquires: overlapped ones rotate over queues, so
    // dispatch i > 0 may start before (or during) dispatch 0's acquire on
    // another queue
    const int rc = dispatch(*e, k, &a, sizeof(a), a.ngroups, /*acquire=*/true,
                            /*barrier=*/ordered, (flags & LVKV_FLAG_SYSTEM_ACQUIRE) != 0, queue,
                            (flags & LVKV_FLAG_FINAL) != 0 && i + 1 == nd);
    if (rc != LVKV_OK) return rc;
    done += n;
  }
  return LVKV_OK;
}

int lvkv_engine_wait(lvkv_engine* eng) {
  if (eng == nullptr) return LVKV_ERR_INVALID;
  Engine* e = reinterpret_cast<Engine*>(eng);
  std::lock_guard<std::mutex> lk(e->mu);
  if (e->fenced != e->next && fence(*e) != LVKV_OK) return LVKV_ERR_HIP;
  return e->queue_error ? LVKV_ERR_HIP : LVKV_OK;
}

int lvkv_engine_crc32c_batch(lvkv_engine* eng, const void* d_base, const uint64_t* d_offsets,
                             const uint32_t* d_lengths, const uint32_t* d_init, uint32_t init,
                             uint32_t* d_out, size_t nblocks, uint32_t flags) {
  if (eng == nullptr) return LVKV_ERR_INVALID;
  if (nblocks == 0) return LVKV_OK;
  if (!d_base || !d_offsets || !d_lengths || !d_out) return LVKV_ERR_INVALID;
  KernelArgs a;
  memset(&a, 0, sizeof(a));
  a.base = static_cast<const uint8_t*>(d_base);
  a.offsets = d_offsets;
  a.lengths = d_lengths;
  a.inits = d_init;
  a.init = init;
  a.out_crc = d_out;
  a.mode = kModeCompute;
  a.mask = (flags & LVKV_FLAG_MASK) ? 1u : 0u;
  return submit_general(*reinterpret_cast<Engine*>(eng), a, nblocks, flags);
}

int lvkv_engine_sst_verify(lvkv_engine* eng, const void* d_file, const uint64_t* d_offsets,
                           const uint32_t* d_sizes, uint32_t* d_actual, uint8_t* d_status,
                           size_t nblocks, uint32_t flags) {
  if (eng == nullptr) return LVKV_ERR_INVALID;
  if (nblocks == 0) return LVKV_OK;
  if (!d_file || !d_offsets || !d_sizes || !d_actual || !d_status) return LVKV_ERR_INVALID;
  KernelArgs a;
  memset(&a, 0, sizeof(a));
  a.base = static_cast<const uint8_t*>(d_file);
  a.offsets = d_offsets;
  a.lengths = d_sizes;
  a.out_crc = d_actual;
  a.out_status = d_status;
  a.mode = kModeSstVerify;
  return submit_general(*reinterpret_cast<Engine*>(eng), a, nblocks, flags);
}

int lvkv_engine_log_verify(lvkv_engine* eng, const void* d_file, const uint64_t* d_hdr_offsets,
                           uint32_t* d_actual, uint8_t* d_status, size_t nrecords,
                           uint32_t flags) {
  if (eng == nullptr) return LVKV_ERR_INVALID;
  if (nrecords == 0) return LVKV_OK;
  if (!d_file || !d_hdr_offsets || !d_actual || !d_status) return LVKV_ERR_INVALID;
  KernelArgs a;
  memset(&a, 0, sizeof(a));
  a.base = static_cast<const uint8_t*>(d_file);
  a.offsets = d_hdr_offsets;
  a.out_crc = d_actual;
  a.out_status = d_status;
  a.mode = kModeLogVerify;
  return submit_general(*reinterpret_cast<Engine*>(eng), a, nrecords, flags);
}

int lvkv_engine_sst_fill_trailers(lvkv_engine* eng, void* d_file, const uint64_t* d_offsets,
                                  const uint32_t* d_sizes, uint32_t* d_crc, size_t nblocks,
                                  uint32_t flags) {
  if (eng == nullptr) return LVKV_ERR_INVALID;
  if (nblocks == 0) return LVKV_OK;
  if (!d_file || !d_offsets || !d_sizes) return LVKV_ERR_INVALID;
  KernelArgs a;
  memset(&a, 0, sizeof(a));
  a.base = static_cast<const uint8_t*>(d_file);
  a.offsets = d_offsets;
  a.lengths = d_sizes;
  a.out_crc = d_crc;
  a.mode = kModeSstFill;
  return submit_general(*reinterpret_cast<Engine*>(eng), a, nblocks, flags);
}

int lvkv_engine_log_fill_headers(lvkv_engine* eng, void* d_file, const uint64_t* d_hdr_offsets,
                                 uint32_t* d_crc, size_t nrecords, uint32_t flags) {
  if (eng == nullptr) return LVKV_ERR_INVALID;
  if (nrecords == 0) return LVKV_OK;
  if (!d_file || !d_hdr_offsets) return LVKV_ERR_INVALID;
  KernelArgs a;
  memset(&a, 0, sizeof(a));
  a.base = static_cast<const uint8_t*>(d_file);
  a.offsets = d_hdr_offsets;
  a.out_crc = d_crc;
  a.mode = kModeLogFill;
  return submit_general(*reinterpret_cast<Engine*>(eng), a, nrecords, flags);
}

int lvkv_engine_queues(lvkv_engine* eng, int nq) {
  if (eng == nullptr || nq < 0 || nq > kQueues) return LVKV_ERR_INVALID;
  Engine* e = reinterpret_cast<Engine*>(eng);
  std::lock_guard<std::mutex> lk(e->mu);
  if (nq == 0) return e->nq;
  if (e->fenced != e->next && fence(*e) != LVKV_OK) return LVKV_ERR_HIP;
  e->nq = nq;
  return nq;
}

int lvkv_engine_profile(lvkv_engine* eng, int enable) {
  if (eng == nullptr) return LVKV_ERR_INVALID;
  Engine* e = reinterpret_cast<Engine*>(eng);
  std::lock_guard<std::mutex> lk(e->mu);
  if (e->fenced != e->next && fence(*e) != LVKV_OK) return LVKV_ERR_HIP;
  e->profiling = enable != 0;
  e->prof_count = 0;
  return LVKV_OK;
}

long lvkv_engine_profile_read(lvkv_engine* eng, double* start_us, double* end_us, size_t n) {
  if (eng == nullptr || ((start_us == nullptr || end_us == nullptr) && n != 0))
    return LVKV_ERR_INVALID;
  Engine* e = reinterpret_cast<Engine*>(eng);
  std::lock_guard<std::mutex> lk(e->mu);
  if (e->fenced != e->next && fence(*e) != LVKV_OK) return LVKV_ERR_HIP;
  const uint64_t have = std::min<uint64_t>(e->prof_count, kProfLog);
  const uint64_t take = std::min<uint64_t>(have, n);
  for (uint64_t i = 0; i < take; ++i) {
    const uint64_t j = (e->prof_count - take + i) % kProfLog;
    start_us[i] = e->prof_start[j];
    end_us[i] = e->prof_end[j];
  }
  e->prof_count = 0;
  return static_cast<long>(take);
}

int lvkv_engine_set_stamps(lvkv_engine* eng, uint64_t* d_stamps, uint64_t areas) {
  if (eng == nullptr || (d_stamps != nullptr && areas == 0)) return LVKV_ERR_INVALID;
  Engine* e = reinterpret_cast<Engine*>(eng);
  std::lock_guard<std::mutex> lk(e->mu);
  if (e->fenced != e->next && fence(*e) != LVKV_OK) return LVKV_ERR_HIP;
  e->stamps = d_stamps;
  e->stamp_areas = areas;
  e->stamp_next = 0;
  return LVKV_OK;
}

int lvkv_engine_set_variant(lvkv_engine* eng, int variant, int ordered_variant) {
  if (eng == nullptr || variant < 0 || variant >= kNumUniformSpecs || ordered_variant < 0 ||
      ordered_variant >= kNumUniformSpecs)
    return LVKV_ERR_INVALID;
  Engine* e = reinterpret_cast<Engine*>(eng);
  std::lock_guard<std::mutex> lk(e->mu);
  if (e->fenced != e->next && fence(*e) != LVKV_OK) return LVKV_ERR_HIP;
  e->variant = variant;
  e->ordered_variant = ordered_variant;
  return LVKV_OK;
}

int lvkv_engine_set_final_variant(lvkv_engine* eng, int variant) {
  if (eng == nullptr || variant < -1 || variant >= kNumUniformSpecs) return LVKV_ERR_INVALID;
  Engine* e = reinterpret_cast<Engine*>(eng);
  std::lock_guard<std::mutex> lk(e->mu);
  e->final_variant = variant;
  return LVKV_OK;
}

int lvkv_engine_load_probe(lvkv_engine* eng, const void* code_object, size_t size,
                           const char* kernel, uint32_t waves, uint32_t chains, uint32_t per_cu,
                           int overlapped) {
  if (eng == nullptr) return LVKV_ERR_INVALID;
  Engine* e = reinterpret_cast<Engine*>(eng);
  std::lock_guard<std::mutex> lk(e->mu);
  if (e->fenced != e->next && fence(*e) != LVKV_OK) return LVKV_ERR_HIP;
  drop_probe(*e);
  if (code_object == nullptr) return LVKV_OK;
  if (kernel == nullptr || waves == 0 || waves > 16 || chains == 0 || per_cu == 0)
    return LVKV_ERR_INVALID;
  bool ok = hsa_code_object_reader_create_from_memory(code_object, size, &e->probe_reader) ==
            HSA_STATUS_SUCCESS;
  e->probe_reader_ok = ok;
  ok = ok && hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT,
                                       nullptr, &e->probe_exe) == HSA_STATUS_SUCCESS;
  e->probe_exe_ok = ok;
  ok = ok && hsa_executable_load_agent_code_object(e->probe_exe, e->agent, e->probe_reader,
                                                   nullptr, nullptr) == HSA_STATUS_SUCCESS;
  ok = ok && hsa_executable_freeze(e->probe_exe, nullptr) == HSA_STATUS_SUCCESS;
  ok = ok && load_kernel(*e, e->probe_exe, kernel, &e->probe) == LVKV_OK;
  if (!ok) {
    drop_probe(*e);
    return LVKV_ERR_HIP;
  }
  e->probe.waves = waves;
  e->probe.chains = chains;
  e->probe.per_cu = per_cu;
  e->probe_overlapped = overlapped != 0;
  e->probe_on = true;
  return LVKV_OK;
}

int lvkv_engine_set_scopes(lvkv_engine* eng, int dispatch_acquire, int fence_acquire,
                           int fence_release) {
  if (eng == nullptr) return LVKV_ERR_INVALID;
  for (int v : {dispatch_acquire, fence_acquire, fence_release})
    if (v < HSA_FENCE_SCOPE_NONE || v > HSA_FENCE_SCOPE_SYSTEM) return LVKV_ERR_INVALID;
  Engine* e = reinterpret_cast<Engine*>(eng);
  std::lock_guard<std::mutex> lk(e->mu);
  if (e->fenced != e->next && fence(*e) != LVKV_OK) return LVKV_ERR_HIP;
  e->dispatch_acq = dispatch_acquire;
  e->fence_acq = fence_acquire;
  e->fence_rel = fence_release;
  return LVKV_OK;
}

int lvkv_engine_set_priority(lvkv_engine* eng, int priority) {
  if (eng == nullptr || priority < 0 || priority > 2) return LVKV_ERR_INVALID;
  Engine* e = reinterpret_cast<Engine*>(eng);
  std::lock_guard<std::mutex> lk(e->mu);
  if (e->fenced != e->next && fence(*e) != LVKV_OK) return LVKV_ERR_HIP;
  for (hsa_queue_t* q : e->queues)
    if (hsa_amd_queue_set_priority(q, static_cast<hsa_amd_queue_priority_t>(priority)) !=
        HSA_STATUS_SUCCESS)
      return LVKV_ERR_HIP;
  return LVKV_OK;
}

int lvkv_debug_engine_stall(lvkv_engine* eng, int stall, double stuck_seconds) {
  if (eng == nullptr || stuck_seconds <= 0) return LVKV_ERR_INVALID;
  Engine* e = reinterpret_cast<Engine*>(eng);
  std::lock_guard<std::mutex> lk(e->mu);
  e->stuck_s = stuck_seconds;
  if (!stall) {
    if (e->hold_ok) hsa_signal_store_screlease(e->hold_sig, 0);
    return LVKV_OK;
  }
  if (!e->hold_ok) {
    if (hsa_signal_create(1, 0, nullptr, &e->hold_sig) != HSA_STATUS_SUCCESS) return LVKV_ERR_HIP;
    e->hold_ok = true;
  }
  hsa_signal_store_screlease(e->hold_sig, 1);
  // a barrier-AND packet on every queue that waits for the hold signal: the
  // queues stop behind it as they would behind a faulted or endless kernel
  const int keep = e->cur;
  for (int q = 0; q < e->nq; ++q) {
    e->cur = q;
    uint64_t idx;
    hsa_barrier_and_packet_t* p = static_cast<hsa_barrier_and_packet_t*>(packet_slot(*e, &idx));
    if (p == nullptr) {
      e->cur = keep;
      return LVKV_ERR_HIP;
    }
    p->reserved0 = 0;
    p->reserved1 = 0;
    for (int i = 0; i < 5; ++i) p->dep_signal[i].handle = 0;
    p->dep_signal[0] = e->hold_sig;
    p->reserved2 = 0;
    p->completion_signal.handle = 0;
    publish(*e, p,
            static_cast<uint16_t>((HSA_PACKET_TYPE_BARRIER_AND << HSA_PACKET_HEADER_TYPE) |
                                  (1 << HSA_PACKET_HEADER_BARRIER)),
            0, idx);
  }
  e->cur = keep;
  return LVKV_OK;
}

int lvkv_debug_engine_ragged_spec(lvkv_engine* eng, int spec) {
  if (eng == nullptr || spec < -1 || spec >= kNumSpecs || (spec >= 0 && spec < kRaggedSpec))
    return LVKV_ERR_INVALID;
  Engine* e = reinterpret_cast<Engine*>(eng);
  std::lock_guard<std::mutex> lk(e->mu);
  e->ragged_spec = spec;
  return LVKV_OK;
}

int lvkv_debug_engine_kernarg_cache(lvkv_engine* eng, uint64_t* hits, uint64_t* misses) {
  if (eng == nullptr || hits == nullptr || misses == nullptr) return LVKV_ERR_INVALID;
  Engine* e = reinterpret_cast<Engine*>(eng);
  std::lock_guard<std::mutex> lk(e->mu);
  *hits = e->ka_hits;
  *misses = e->ka_misses;
  return LVKV_OK;
}

int lvkv_engine_shape(lvkv_engine* eng, uint32_t* waves, uint32_t* chains, uint32_t* groups) {
  if (eng == nullptr) return LVKV_ERR_INVALID;
  Engine* e = reinterpret_cast<Engine*>(eng);
  std::lock_guard<std::mutex> lk(e->mu);
  const EngineKernel& k = e->kern[e->variant];
  if (waves) *waves = k.waves;
  if (chains) *chains = k.chains;
  if (groups) *groups = static_cast<uint32_t>(e->cus) * k.per_cu;
  return LVKV_OK;
}

}  // extern "C"
