// Timing probes for the headline kernel (NOT part of the product library).
//
// Built by tools/probe/build.sh into tools/probe/libprobe.so. Instantiates
// variants of crc32c_burst_kernel (csrc/crc32c_burst.h) and times them, and
// the product entry lvkv_crc32c_uniform_device, with the launch loop in C++
// so host launch cost does not pace the GPU:
//   res[0] single stream, HIP events around K launches: us per launch
//   res[1] `nstreams` streams (step i on stream i % S): us per launch period
//   res[2] bench-style host-timed region of 20 steps (sync, t0, launches,
//          sync, t1): us per step, median of 7 repetitions
//   res[3] the same with K steps
// Consecutive launches read different windows of a rotation (MALL-cold).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <vector>

#include "crc32c_burst.h"
#include "lvkv_crc32c.h"
#include "lvkv_kernel_args.h"
#include "lvkv_tables.h"

namespace lvkv {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) probe_read_kernel(const u32x4* p, uint64_t n16,
                                                         uint32_t* out) {
  uint32_t x = 0;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
    const u32x4 v = __builtin_nontemporal_load(p + i);
    x ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (x == 0x12345678u) out[0] = x;
}

}  // namespace lvkv

using namespace lvkv;

namespace {

struct Ctx {
  bool ready = false;
  int cus = 0;
  uint32_t* d_lane_cols = nullptr;
  uint32_t* d_zpow = nullptr;
  uint32_t zcol[32];
} g;

int init() {
  if (g.ready) return 0;
  if (hipDeviceGetAttribute(&g.cus, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess)
    return -1;
  std::vector<uint32_t> cols(kLaneColDwords), zp(kZPowDwords);
  build_lane_columns(cols.data());
  build_zpow_tables(zp.data());
  if (hipMalloc(&g.d_lane_cols, cols.size() * 4) != hipSuccess) return -2;
  if (hipMalloc(&g.d_zpow, zp.size() * 4) != hipSuccess) return -2;
  hipMemcpy(g.d_lane_cols, cols.data(), cols.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(g.d_zpow, zp.data(), zp.size() * 4, hipMemcpyHostToDevice);
  const Gf2Op z = gf2_zero_advance(kRowBytes);
  memcpy(g.zcol, z.col, sizeof(g.zcol));
  g.ready = true;
  return 0;
}

struct Shape {
  int w, nch, occ;
};

// cfg -> (flags, W, NCH, OCC); cfg >= 100: product entry / read kernel.
Shape shape_of(int cfg) {
  switch (cfg) {
    case 7: case 8: case 17: case 18: return {8, 5, 2};
    case 9: case 10: return {16, 3, 1};
    case 13: case 14: return {8, 4, 2};
    default: return {8, 3, 2};
  }
}

hipError_t launch_cfg(int cfg, int groups, const UniformArgs& a, hipStream_t s) {
#define C(id, f, w, n, o)                                                                  \
  case id:                                                                                 \
    hipLaunchKernelGGL((crc32c_burst_kernel<f, w, n, o>), dim3(groups), dim3(64 * w), 0, s, a); \
    break;
  switch (cfg) {
    C(0, 0, 8, 3, 2)
    C(1, kBurstLate, 8, 3, 2)
    C(2, kBurstBare, 8, 3, 2)
    C(3, kBurstNoBuild, 8, 3, 2)
    C(4, kBurstNoWalk, 8, 3, 2)
    C(5, kBurstRowsHbm, 8, 3, 2)
    C(6, kBurstDefaultPolicy, 8, 3, 2)
    C(7, 0, 8, 5, 2)
    C(8, kBurstBare, 8, 5, 2)
    C(9, 0, 16, 3, 1)
    C(10, kBurstBare, 16, 3, 1)
    C(11, kBurstStamps, 8, 3, 2)
    C(12, kBurstNoBuild | kBurstNoWalk, 8, 3, 2)
    C(13, 0, 8, 4, 2)
    C(14, kBurstLate, 8, 4, 2)
    C(15, kBurstSplit2, 8, 3, 2)
    C(16, kBurstSplit4, 8, 3, 2)
    C(17, kBurstSplit2, 8, 5, 2)
    C(18, kBurstSplit4, 8, 5, 2)
    C(19, kBurstSplit2 | kBurstLate, 8, 3, 2)
    default:
      return hipErrorInvalidValue;
  }
#undef C
  return hipGetLastError();
}

struct Job {
  int cfg, groups;
  const uint8_t* base;
  uint64_t win_bytes;
  int nrot;
  uint32_t len, nb;
  uint32_t* out;
  uint64_t* stamps;
};

hipError_t launch_one(const Job& j, int i, hipStream_t s) {
  const uint8_t* b = j.base + static_cast<uint64_t>(i % j.nrot) * j.win_bytes;
  uint32_t* out = j.out + static_cast<uint64_t>(i & 1) * j.nb;
  if (j.cfg == 100) {
    const int rc = lvkv_crc32c_uniform_device(b, j.len, j.len, 0, out, j.nb, 0, s);
    return rc == 0 ? hipSuccess : hipErrorUnknown;
  }
  if (j.cfg == 101) {
    const int grid = j.groups > 0 ? j.groups : g.cus * 8;
    hipLaunchKernelGGL(probe_read_kernel, dim3(grid), dim3(256), 0, s,
                       reinterpret_cast<const u32x4*>(b),
                       static_cast<uint64_t>(j.nb) * j.len / 16, out);
    return hipGetLastError();
  }
  UniformArgs a;
  memset(&a, 0, sizeof(a));
  a.base = b;
  a.stride = j.len;
  a.out = out;
  a.lane_cols = g.d_lane_cols;
  a.zpow = g.d_zpow;
  a.stamps = j.stamps;
  a.length = j.len;
  a.nblocks = j.nb;
  memcpy(a.zcol, g.zcol, sizeof(a.zcol));
  return launch_cfg(j.cfg, j.groups, a, s);
}

double now_us() {
  return std::chrono::duration<double, std::micro>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

}  // namespace

extern "C" {

// Launch cfg once (parity checks, stamps). groups <= 0: CUs * OCC.
int probe_launch(int cfg, int groups, const void* base, uint32_t len, uint32_t nb, uint32_t* out,
                 uint64_t* stamps, void* stream) {
  if (init() != 0) return -1;
  const Shape sh = shape_of(cfg);
  if (groups <= 0) groups = g.cus * sh.occ;
  if (cfg < 100 && static_cast<uint64_t>(groups) * sh.w * sh.nch < nb) return -3;
  Job j{cfg, groups, static_cast<const uint8_t*>(base), 0, 1, len, nb, out, stamps};
  return launch_one(j, 0, static_cast<hipStream_t>(stream)) == hipSuccess ? 0 : -4;
}

int probe_cus() { return init() == 0 ? g.cus : -1; }

// out must hold 2 * nb u32. Returns 0 or a negative code.
int probe_time(int cfg, int groups, const void* base, uint64_t win_bytes, int nrot, uint32_t len,
               uint32_t nb, uint32_t* out, int K, int nstreams, double warm_ms, double* res) {
  if (init() != 0) return -1;
  const Shape sh = shape_of(cfg);
  if (groups <= 0) groups = g.cus * sh.occ;
  if (cfg < 100 && static_cast<uint64_t>(groups) * sh.w * sh.nch < nb) return -3;
  Job j{cfg, groups, static_cast<const uint8_t*>(base), win_bytes, nrot, len, nb, out, nullptr};
  nstreams = std::max(1, std::min(nstreams, 4));
  std::vector<hipStream_t> st(nstreams);
  std::vector<hipEvent_t> join(nstreams);
  for (int s = 0; s < nstreams; ++s) {
    hipStreamCreateWithFlags(&st[s], hipStreamNonBlocking);
    hipEventCreateWithFlags(&join[s], hipEventDisableTiming);
  }
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  int rot = 0;
  auto warm = [&](double ms) {
    const double t_end = now_us() + ms * 1000.0;
    while (now_us() < t_end)
      for (int k = 0; k < 32; ++k) {
        const int i = rot++;
        launch_one(j, i, st[i % nstreams]);
      }
    hipDeviceSynchronize();
  };
  auto multi = [&](int n) {  // fork from st[0], n launches over the streams, join
    hipEventRecord(join[0], st[0]);
    for (int s = 1; s < nstreams; ++s) hipStreamWaitEvent(st[s], join[0], 0);
    for (int i = 0; i < n; ++i) launch_one(j, rot++, st[i % nstreams]);
    for (int s = 1; s < nstreams; ++s) {
      hipEventRecord(join[s], st[s]);
      hipStreamWaitEvent(st[0], join[s], 0);
    }
  };
  float ms = 0;
  // single stream
  warm(warm_ms);
  hipEventRecord(e0, st[0]);
  for (int i = 0; i < K; ++i) launch_one(j, rot++, st[0]);
  hipEventRecord(e1, st[0]);
  hipEventSynchronize(e1);
  hipEventElapsedTime(&ms, e0, e1);
  res[0] = 1000.0 * ms / K;
  // S streams, device period
  warm(warm_ms);
  hipEventRecord(e0, st[0]);
  multi(K);
  hipEventRecord(e1, st[0]);
  hipEventSynchronize(e1);
  hipEventElapsedTime(&ms, e0, e1);
  res[1] = 1000.0 * ms / K;
  // host-timed regions
  for (int pass = 0; pass < 2; ++pass) {
    const int n = pass == 0 ? 20 : K;
    std::vector<double> t;
    for (int rep = 0; rep < 7; ++rep) {
      warm(pass == 0 ? std::min(warm_ms, 100.0) : 20.0);
      const double t0 = now_us();
      multi(n);
      hipDeviceSynchronize();
      t.push_back((now_us() - t0) / n);
    }
    std::sort(t.begin(), t.end());
    res[2 + pass] = t[t.size() / 2];
  }
  const hipError_t err = hipGetLastError();
  for (int s = 0; s < nstreams; ++s) {
    hipStreamDestroy(st[s]);
    hipEventDestroy(join[s]);
  }
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  return err == hipSuccess ? 0 : -5;
}

// Host-timed regions of K steps for each K in ks[0..nk): median us per
// region over 7 repetitions, each after a 50 ms warm-up. mode bit 0: spin on
// hipEventQuery of the end event before hipDeviceSynchronize; bit 1: one
// stream, no fork/join.
int probe_host_sweep(int cfg, int groups, const void* base, uint64_t win_bytes, int nrot,
                     uint32_t len, uint32_t nb, uint32_t* out, int nstreams, int mode,
                     const int* ks, int nk, double* res) {
  if (init() != 0) return -1;
  const Shape sh = shape_of(cfg);
  if (groups <= 0) groups = g.cus * sh.occ;
  if (cfg < 100 && static_cast<uint64_t>(groups) * sh.w * sh.nch < nb) return -3;
  Job j{cfg, groups, static_cast<const uint8_t*>(base), win_bytes, nrot, len, nb, out, nullptr};
  nstreams = (mode & 2) ? 1 : std::max(1, std::min(nstreams, 4));
  std::vector<hipStream_t> st(nstreams);
  std::vector<hipEvent_t> join(nstreams);
  for (int s = 0; s < nstreams; ++s) {
    hipStreamCreateWithFlags(&st[s], hipStreamNonBlocking);
    hipEventCreateWithFlags(&join[s], hipEventDisableTiming);
  }
  hipEvent_t fin;
  hipEventCreateWithFlags(&fin, hipEventDisableTiming);
  int rot = 0;
  for (int q = 0; q < nk; ++q) {
    std::vector<double> t;
    for (int rep = 0; rep < 7; ++rep) {
      const double t_end = now_us() + 50000.0;
      while (now_us() < t_end)
        for (int k = 0; k < 32; ++k) {
          const int i = rot++;
          launch_one(j, i, st[i % nstreams]);
        }
      hipDeviceSynchronize();
      const double t0 = now_us();
      hipEventRecord(join[0], st[0]);
      for (int s = 1; s < nstreams; ++s) hipStreamWaitEvent(st[s], join[0], 0);
      for (int i = 0; i < ks[q]; ++i) launch_one(j, rot++, st[i % nstreams]);
      for (int s = 1; s < nstreams; ++s) {
        hipEventRecord(join[s], st[s]);
        hipStreamWaitEvent(st[0], join[s], 0);
      }
      hipEventRecord(fin, st[0]);
      if (mode & 1)
        while (hipEventQuery(fin) == hipErrorNotReady) {
        }
      hipDeviceSynchronize();
      t.push_back(now_us() - t0);
    }
    std::sort(t.begin(), t.end());
    res[q] = t[t.size() / 2];
  }
  for (int s = 0; s < nstreams; ++s) {
    hipStreamDestroy(st[s]);
    hipEventDestroy(join[s]);
  }
  hipEventDestroy(fin);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

__global__ void probe_empty_kernel(uint32_t* p);

// Timed region anatomy, single stream, K steps of cfg: for prep in
// {0: none, 1: 50 ms warm-up + sync, 2: warm-up + sync + one empty kernel
// + sync, 3: warm-up + sync + 2 ms idle}: res[prep*4 + {0,1,2,3}] = median
// host total, host issue time, device e0->e1 time, host wait after issue.
int probe_region(int cfg, int groups, const void* base, uint64_t win_bytes, int nrot, uint32_t len,
                 uint32_t nb, uint32_t* out, int K, double* res) {
  if (init() != 0) return -1;
  const Shape sh = shape_of(cfg);
  if (groups <= 0) groups = g.cus * sh.occ;
  Job j{cfg, groups, static_cast<const uint8_t*>(base), win_bytes, nrot, len, nb, out, nullptr};
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  int rot = 0;
  for (int prep = 0; prep < 4; ++prep) {
    std::vector<double> t[4];
    for (int rep = 0; rep < 9; ++rep) {
      if (prep >= 1) {
        const double t_end = now_us() + 50000.0;
        while (now_us() < t_end)
          for (int k = 0; k < 32; ++k) launch_one(j, rot++, s);
      }
      hipDeviceSynchronize();
      if (prep == 2) {
        hipLaunchKernelGGL(probe_empty_kernel, dim3(1), dim3(64), 0, s, nullptr);
        hipDeviceSynchronize();
      }
      if (prep == 3) {
        const double t_end = now_us() + 2000.0;
        while (now_us() < t_end) {
        }
      }
      const double t0 = now_us();
      hipEventRecord(e0, s);
      for (int i = 0; i < K; ++i) launch_one(j, rot++, s);
      hipEventRecord(e1, s);
      const double t1 = now_us();
      hipDeviceSynchronize();
      const double t2 = now_us();
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      t[0].push_back(t2 - t0);
      t[1].push_back(t1 - t0);
      t[2].push_back(1000.0 * ms);
      t[3].push_back(t2 - t1);
    }
    for (int k = 0; k < 4; ++k) {
      std::sort(t[k].begin(), t[k].end());
      res[prep * 4 + k] = t[k][t[k].size() / 2];
    }
  }
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  hipStreamDestroy(s);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

// Graph replay: K launches of cfg (windows start..start+K-1 of the rotation)
// captured once on `nstreams` forked streams, then timed as a bench region:
// warm-up (50 ms of direct launches on other windows), sync, t0, one
// hipGraphLaunch, sync, t1. res[0] = median host us per step, res[1] =
// device us per step (events around the graph launch), res[2] = host us of
// the hipGraphLaunch call, res[3] = instantiate ms.
int probe_graph(int cfg, int groups, const void* base, uint64_t win_bytes, int nrot, uint32_t len,
                uint32_t nb, uint32_t* out, int K, int nstreams, double* res) {
  if (init() != 0) return -1;
  const Shape sh = shape_of(cfg);
  if (groups <= 0) groups = g.cus * sh.occ;
  Job j{cfg, groups, static_cast<const uint8_t*>(base), win_bytes, nrot, len, nb, out, nullptr};
  nstreams = std::max(1, std::min(nstreams, 4));
  std::vector<hipStream_t> st(nstreams);
  std::vector<hipEvent_t> join(nstreams);
  for (int s = 0; s < nstreams; ++s) {
    hipStreamCreateWithFlags(&st[s], hipStreamNonBlocking);
    hipEventCreateWithFlags(&join[s], hipEventDisableTiming);
  }
  // warm the launch path and the device context before capturing
  launch_one(j, 0, st[0]);
  hipDeviceSynchronize();
  const int first = nrot / 2;  // the graph's windows
  hipGraph_t graph;
  if (hipStreamBeginCapture(st[0], hipStreamCaptureModeThreadLocal) != hipSuccess) return -6;
  hipEventRecord(join[0], st[0]);
  for (int s = 1; s < nstreams; ++s) hipStreamWaitEvent(st[s], join[0], 0);
  for (int i = 0; i < K; ++i) launch_one(j, first + i, st[i % nstreams]);
  for (int s = 1; s < nstreams; ++s) {
    hipEventRecord(join[s], st[s]);
    hipStreamWaitEvent(st[0], join[s], 0);
  }
  if (hipStreamEndCapture(st[0], &graph) != hipSuccess) return -7;
  hipGraphExec_t exec;
  double ti = now_us();
  if (hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0) != hipSuccess) return -8;
  res[3] = (now_us() - ti) / 1000.0;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  std::vector<double> th, td, tl;
  int rot = first + K;
  for (int rep = 0; rep < 9; ++rep) {
    const double t_end = now_us() + 50000.0;
    while (now_us() < t_end)
      for (int k = 0; k < 32; ++k) {
        const int i = rot++;
        if (i % nrot >= first && i % nrot < first + K) continue;
        launch_one(j, i, st[0]);
      }
    hipDeviceSynchronize();
    const double t0 = now_us();
    hipEventRecord(e0, st[0]);
    hipGraphLaunch(exec, st[0]);
    const double t1 = now_us();
    hipEventRecord(e1, st[0]);
    hipDeviceSynchronize();
    const double t2 = now_us();
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    th.push_back((t2 - t0) / K);
    td.push_back(1000.0 * ms / K);
    tl.push_back(t1 - t0);
  }
  std::sort(th.begin(), th.end());
  std::sort(td.begin(), td.end());
  std::sort(tl.begin(), tl.end());
  res[0] = th[th.size() / 2];
  res[1] = td[td.size() / 2];
  res[2] = tl[tl.size() / 2];
  hipGraphExecDestroy(exec);
  hipGraphDestroy(graph);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  for (int s = 0; s < nstreams; ++s) {
    hipStreamDestroy(st[s]);
    hipEventDestroy(join[s]);
  }
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

// K launches of cfg on one stream after a 20 ms warm-up (profiling runs).
int probe_single(int cfg, int groups, const void* base, uint64_t win_bytes, int nrot, uint32_t len,
                 uint32_t nb, uint32_t* out, int K) {
  if (init() != 0) return -1;
  const Shape sh = shape_of(cfg);
  if (groups <= 0) groups = g.cus * sh.occ;
  Job j{cfg, groups, static_cast<const uint8_t*>(base), win_bytes, nrot, len, nb, out, nullptr};
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  int rot = 0;
  const double t_end = now_us() + 20000.0;
  while (now_us() < t_end) launch_one(j, rot++, s);
  for (int i = 0; i < K; ++i) launch_one(j, rot++, s);
  hipStreamSynchronize(s);
  hipStreamDestroy(s);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

__global__ void probe_empty_kernel(uint32_t* p) {
  if (p != nullptr && threadIdx.x == 1023u) p[0] = 0;
}

// Latency components (us, medians of 200): [0] hipDeviceSynchronize on an
// idle device, [1] hipStreamSynchronize on an idle stream, [2] one empty
// kernel launched and waited for by spinning on hipEventQuery, [3] the same
// waited for by hipDeviceSynchronize, [4] host cost of one launch call,
// [5] one empty kernel + hipStreamSynchronize.
int probe_latency(double* res) {
  if (init() != 0) return -1;
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipEvent_t ev;
  hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  std::vector<double> t[6];
  for (int i = 0; i < 200; ++i) {
    double t0 = now_us();
    hipDeviceSynchronize();
    t[0].push_back(now_us() - t0);
    t0 = now_us();
    hipStreamSynchronize(s);
    t[1].push_back(now_us() - t0);
    t0 = now_us();
    hipLaunchKernelGGL(probe_empty_kernel, dim3(512), dim3(512), 0, s, nullptr);
    const double t1 = now_us();
    hipEventRecord(ev, s);
    while (hipEventQuery(ev) == hipErrorNotReady) {
    }
    t[2].push_back(now_us() - t0);
    t[4].push_back(t1 - t0);
    t0 = now_us();
    hipLaunchKernelGGL(probe_empty_kernel, dim3(512), dim3(512), 0, s, nullptr);
    hipDeviceSynchronize();
    t[3].push_back(now_us() - t0);
    t0 = now_us();
    hipLaunchKernelGGL(probe_empty_kernel, dim3(512), dim3(512), 0, s, nullptr);
    hipStreamSynchronize(s);
    t[5].push_back(now_us() - t0);
  }
  for (int k = 0; k < 6; ++k) {
    std::sort(t[k].begin(), t[k].end());
    res[k] = t[k][t[k].size() / 2];
  }
  hipEventDestroy(ev);
  hipStreamDestroy(s);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

}  // extern "C"
