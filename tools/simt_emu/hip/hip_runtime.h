// A host-side SIMT emulation of the few HIP device facilities the codec
// kernels use, for debugging them on the CPU (tools/simt_emu/README in the
// header of emu_build.sh). NOT part of the product: a workgroup is 64
// std::threads, one per lane; every cross-lane operation (ballot, shuffle,
// readlane, bpermute, __syncthreads) is a barrier over the 64, so the
// kernel's wave-uniform code runs in lock step at those points; LDS is a
// malloc'd buffer of exactly the launch's size (AddressSanitizer sees
// every byte past it).
#pragma once
#include <stdint.h>
#include <string.h>

#include <atomic>
#include <barrier>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <thread>
#include <vector>

#define __device__
#define __global__
#define __host__
#define __forceinline__ inline
#define __launch_bounds__(x)
#define __constant__ static const

struct dim3 {
  uint32_t x, y, z;
  dim3(uint32_t a = 1, uint32_t b = 1, uint32_t c = 1) : x(a), y(b), z(c) {}
};
typedef int hipError_t;
typedef void* hipStream_t;
#define hipSuccess 0

namespace emu {
inline thread_local dim3 tid;
inline dim3 bid;
inline uint8_t* lds_base = nullptr;
inline std::barrier<>* bar = nullptr;
inline uint64_t slot[64];
inline void sync() { bar->arrive_and_wait(); }
template <typename T>
inline T xread(T v, uint32_t src) {
  uint64_t raw = 0;
  memcpy(&raw, &v, sizeof(T) < 8 ? sizeof(T) : 8);
  slot[tid.x] = raw;
  sync();
  const uint64_t r = slot[src & 63u];
  sync();
  T out;
  memcpy(&out, &r, sizeof(T) < 8 ? sizeof(T) : 8);
  return out;
}
inline uint64_t ballot(bool p) {
  slot[tid.x] = p ? 1u : 0u;
  sync();
  uint64_t m = 0;
  for (int i = 0; i < 64; ++i) m |= (slot[i] & 1u) << i;
  sync();
  return m;
}
template <typename T>
inline T shfl_up(T v, uint32_t d) {
  const uint32_t l = tid.x;
  return xread(v, l >= d ? l - d : l);
}
template <typename T>
inline T shfl_down(T v, uint32_t d) {
  const uint32_t l = tid.x;
  return xread(v, l + d < 64 ? l + d : l);
}
template <typename T>
inline T shfl_xor(T v, uint32_t m) {
  return xread(v, (tid.x ^ m) & 63u);
}
template <typename T>
inline T amin(T* p, T v) {
  T old = __atomic_load_n(p, __ATOMIC_SEQ_CST);
  while (v < old && !__atomic_compare_exchange_n(p, &old, v, false, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST)) {
  }
  return old;
}
template <typename T>
inline T amax(T* p, T v) {
  T old = __atomic_load_n(p, __ATOMIC_SEQ_CST);
  while (v > old && !__atomic_compare_exchange_n(p, &old, v, false, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST)) {
  }
  return old;
}

template <typename K, typename... A>
inline void launch(K kernel, dim3 grid, size_t lds, A... args) {
  for (uint32_t b = 0; b < grid.x; ++b) {
    bid = dim3(b);
    lds_base = static_cast<uint8_t*>(malloc(lds ? lds : 16));
    memset(lds_base, 0xA5, lds);  // (LDS is not zeroed on the device either)
    std::barrier<> br(64);
    bar = &br;
    std::vector<std::thread> th;
    for (uint32_t l = 0; l < 64; ++l)
      th.emplace_back([=]() {
        tid = dim3(l);
        kernel(args...);
      });
    for (auto& t : th) t.join();
    free(lds_base);
  }
}
}  // namespace emu

#define threadIdx (emu::tid)
#define blockIdx (emu::bid)
#define __syncthreads() emu::sync()
#define __ballot(p) emu::ballot(p)
#define __shfl(v, s) emu::xread((v), static_cast<uint32_t>(s))
#define __shfl_up(v, d) emu::shfl_up((v), static_cast<uint32_t>(d))
#define __shfl_down(v, d) emu::shfl_down((v), static_cast<uint32_t>(d))
#define __shfl_xor(v, m) emu::shfl_xor((v), static_cast<uint32_t>(m))
#define __builtin_amdgcn_readlane(v, l) emu::xread((v), static_cast<uint32_t>(l))
#define __builtin_amdgcn_readfirstlane(v) emu::xread((v), 0u)
#define __builtin_amdgcn_writelane(v, l, old) \
  (emu::tid.x == static_cast<uint32_t>(l) ? static_cast<uint32_t>(v) : static_cast<uint32_t>(old))
#define __builtin_amdgcn_ds_bpermute(a, v) emu::xread((v), static_cast<uint32_t>((a) >> 2))
#define __builtin_amdgcn_alignbyte(hi, lo, s) \
  static_cast<uint32_t>(((static_cast<uint64_t>(hi) << 32) | static_cast<uint32_t>(lo)) >> (8u * ((s) & 3u)))
#define __builtin_amdgcn_rcpf(x) (1.0f / (x))
#define __builtin_amdgcn_s_memtime() 0ull
#define __builtin_amdgcn_wave_barrier() ((void)0)
#define __builtin_amdgcn_s_waitcnt(x) ((void)0)
#define __popcll(x) __builtin_popcountll(x)
#define __lane_id() (emu::tid.x)
#define atomicMin(p, v) emu::amin((p), (v))
#define atomicMax(p, v) emu::amax((p), (v))
#define atomicAdd(p, v) __atomic_fetch_add((p), (v), __ATOMIC_SEQ_CST)
#define atomicOr(p, v) __atomic_fetch_or((p), (v), __ATOMIC_SEQ_CST)
#define hipLaunchKernelGGL(k, grid, block, lds, stream, ...) emu::launch(k, grid, lds, __VA_ARGS__)
#define hipGetLastError() 0
