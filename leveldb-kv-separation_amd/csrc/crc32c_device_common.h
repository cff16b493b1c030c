// Device helpers shared by the batch kernels (gfx950): scalar loads, the
// LDS table walk (row step, lane end shift) and the wave reduction.
#ifndef LVKV_CRC32C_DEVICE_COMMON_H_
#define LVKV_CRC32C_DEVICE_COMMON_H_

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lvkv_kernel_args.h"

namespace lvkv {
namespace {

typedef __attribute__((address_space(4))) const uint32_t ConstU32;

constexpr uint32_t kBufferDword3 = 0x00020000u;  // gfx9 raw buffer config
constexpr uint32_t kOobOffset = 0x80000000u;     // >= any num_records

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

typedef __attribute__((address_space(4))) const uint64_t ConstU64;

// Wave-uniform dword load through the scalar cache. `addr` must be 4-aligned.
__device__ __forceinline__ uint32_t sload32(uint64_t addr) {
  return *reinterpret_cast<ConstU32*>(addr);
}
typedef __attribute__((address_space(1))) const uint32_t GlobalU32;
// Dword vector load from global memory (vmcnt only: a flat load would also
// count in lgkmcnt and hold up the next LDS wait). `addr` must be 4-aligned.
__device__ __forceinline__ uint32_t gload32(uint64_t addr) {
  return *reinterpret_cast<GlobalU32*>(addr);
}

// Wave-uniform element loads of the descriptor arrays (s_load, lgkmcnt).
__device__ __forceinline__ uint32_t sload_u32(const uint32_t* p, uint32_t i) {
  return reinterpret_cast<ConstU32*>(reinterpret_cast<uint64_t>(p))[i];
}
__device__ __forceinline__ uint64_t sload_u64(const uint64_t* p, uint32_t i) {
  return reinterpret_cast<ConstU64*>(reinterpret_cast<uint64_t>(p))[i];
}

// Wave-uniform little-endian load of n (1..4) bytes at any address, touching
// only the dwords that contain [addr, addr + n).
__device__ __forceinline__ uint32_t sload_le(uint64_t addr, uint32_t n) {
  const uint64_t a0 = addr & ~uint64_t{3};
  const uint64_t a1 = (addr + n - 1) & ~uint64_t{3};
  const uint32_t lo = sload32(a0);
  const uint32_t hi = (a1 != a0) ? sload32(a1) : 0u;
  const uint32_t sh = static_cast<uint32_t>(addr & 3u) * 8u;
  const uint64_t v = (static_cast<uint64_t>(hi) << 32) | lo;
  uint32_t r = static_cast<uint32_t>(v >> sh);
  if (n < 4) r &= (1u << (8u * n)) - 1u;
  return r;
}

__device__ __forceinline__ uint32_t crc_mask(uint32_t c) {
  return ((c >> 15) | (c << 17)) + kMaskDelta;
}
__device__ __forceinline__ uint32_t crc_unmask(uint32_t m) {
  const uint32_t r = m - kMaskDelta;
  return (r >> 17) | (r << 15);
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

__device__ __forceinline__ uint32_t lds_ld(const uint32_t* lds,
                                           uint32_t byte_addr) {
  return *reinterpret_cast<const uint32_t*>(
      reinterpret_cast<const char*>(lds) + byte_addr);
}

// S -> Z_256(S): one bank-private LDS lookup per byte of S.
// k0 = (lane & 31) * 4, k1 = k0 | 0x10000. v_perm_b32 builds
// {k.byte0, S.byte_t, k.byte2, 0} = S.byte_t * 256 + copy*4 + region.
__device__ __forceinline__ uint32_t row_advance(const uint32_t* lds,
                                                uint32_t s, uint32_t k0,
                                                uint32_t k1) {
  const uint32_t a0 = __builtin_amdgcn_perm(s, k0, 0x0C020400u);
  const uint32_t a1 = __builtin_amdgcn_perm(s, k0, 0x0C020500u);
  const uint32_t a2 = __builtin_amdgcn_perm(s, k1, 0x0C020600u);
  const uint32_t a3 = __builtin_amdgcn_perm(s, k1, 0x0C020700u);
  return xor3(lds_ld(lds, a0), lds_ld(lds, a1 + 128u), lds_ld(lds, a2)) ^
         lds_ld(lds, a3 + 128u);
}

// S -> Z_256(S) ^ w with two 3-input xors (v_bitop3_b32, truth table 0x96).
__device__ __forceinline__ uint32_t row_step(const uint32_t* lds, uint32_t s,
                                             uint32_t w, uint32_t k0,
                                             uint32_t k1) {
  const uint32_t a0 = __builtin_amdgcn_perm(s, k0, 0x0C020400u);
  const uint32_t a1 = __builtin_amdgcn_perm(s, k0, 0x0C020500u);
  const uint32_t a2 = __builtin_amdgcn_perm(s, k1, 0x0C020600u);
  const uint32_t a3 = __builtin_amdgcn_perm(s, k1, 0x0C020700u);
  const uint32_t t = xor3(lds_ld(lds, a0), lds_ld(lds, a1 + 128u), w);
  return xor3(t, lds_ld(lds, a2), lds_ld(lds, a3 + 128u));
}

// S -> Z_{256-4s}(S) for this lane s: eight lane-private nibble lookups.
__device__ __forceinline__ uint32_t lane_end_shift(const uint32_t* lds,
                                                   uint32_t s,
                                                   uint32_t lane_base) {
  uint32_t r = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint32_t nib = (s >> (4 * k)) & 15u;
    r ^= lds_ld(lds, (lane_base | (nib << 8)) + 4096u * k);
  }
  return r;
}

// XOR over the 64 lanes, result wave-uniform. DPP row ops fold each 16-lane
// row (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror: VALU, no
// LDS traffic), then four v_readlane_b32 + scalar xors combine the rows.
__device__ __forceinline__ uint32_t wave_xor_dpp(uint32_t v) {
  v ^= static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(v), 0xB1, 0xF, 0xF, false));
  v ^= static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(v), 0x4E, 0xF, 0xF, false));
  v ^= static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(v), 0x141, 0xF, 0xF, false));
  v ^= static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(v), 0x140, 0xF, 0xF, false));
  return __builtin_amdgcn_readlane(v, 0) ^ __builtin_amdgcn_readlane(v, 16) ^
         __builtin_amdgcn_readlane(v, 32) ^ __builtin_amdgcn_readlane(v, 48);
}

// Integer sums and scans over a wave with every lane active, the same way:
// DPP row ops (a few VALU cycles each) and v_readlane for the four rows,
// where __shfl_xor / __shfl_up are ds_bpermute round trips through the LDS
// unit (~100 cycles, six of them in a row for a 64-lane sum).
template <int Ctrl>
__device__ __forceinline__ uint32_t dpp32(uint32_t v) {
  return static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(v), Ctrl, 0xF, 0xF, false));
}
// row_shr:n with the lanes that have no source reading 0
template <int N>
__device__ __forceinline__ uint32_t dpp_shr0(uint32_t v) {
  return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x110 + N, 0xF, 0xF, false));
}
__device__ __forceinline__ uint32_t lane_u32(uint32_t v, uint32_t l) {
  return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), static_cast<int>(l)));
}
__device__ __forceinline__ uint64_t lane_u64(uint64_t v, uint32_t l) {
  return uint64_t{lane_u32(static_cast<uint32_t>(v), l)} |
         uint64_t{lane_u32(static_cast<uint32_t>(v >> 32), l)} << 32;
}
template <int Ctrl, typename T>
__device__ __forceinline__ T dpp_any(T v) {
  if constexpr (sizeof(T) == 8) {
    return static_cast<T>(uint64_t{dpp32<Ctrl>(static_cast<uint32_t>(v))} |
                          uint64_t{dpp32<Ctrl>(static_cast<uint32_t>(static_cast<uint64_t>(v) >> 32))} << 32);
  } else {
    return static_cast<T>(dpp32<Ctrl>(static_cast<uint32_t>(v)));
  }
}
template <int N, typename T>
__device__ __forceinline__ T dpp_shr0_any(T v) {
  if constexpr (sizeof(T) == 8) {
    return static_cast<T>(uint64_t{dpp_shr0<N>(static_cast<uint32_t>(v))} |
                          uint64_t{dpp_shr0<N>(static_cast<uint32_t>(static_cast<uint64_t>(v) >> 32))} << 32);
  } else {
    return static_cast<T>(dpp_shr0<N>(static_cast<uint32_t>(v)));
  }
}
template <typename T>
__device__ __forceinline__ T lane_any(T v, uint32_t l) {
  if constexpr (sizeof(T) == 8) return static_cast<T>(lane_u64(static_cast<uint64_t>(v), l));
  else return static_cast<T>(lane_u32(static_cast<uint32_t>(v), l));
}

// The sum over the 64 lanes, wave-uniform.
template <typename T>
__device__ __forceinline__ T wave_sum_dpp(T v) {
  v += dpp_any<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_any<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_any<0x141>(v);  // row_half_mirror
  v += dpp_any<0x140>(v);  // row_mirror
  return lane_any(v, 0) + lane_any(v, 16) + lane_any(v, 32) + lane_any(v, 48);
}

// The minimum over the 64 lanes, wave-uniform.
__device__ __forceinline__ uint32_t wave_min_dpp(uint32_t v) {
  v = min(v, dpp32<0xB1>(v));
  v = min(v, dpp32<0x4E>(v));
  v = min(v, dpp32<0x141>(v));
  v = min(v, dpp32<0x140>(v));
  return min(min(lane_u32(v, 0), lane_u32(v, 16)), min(lane_u32(v, 32), lane_u32(v, 48)));
}

// The inclusive prefix sum over lanes 0..lane: the 16-lane rows scanned by
// row_shr 1, 2, 4, 8, then each row adds the totals of the rows below it.
template <typename T>
__device__ __forceinline__ T wave_scan_dpp(T v, uint32_t lane) {
  v += dpp_shr0_any<1>(v);
  v += dpp_shr0_any<2>(v);
  v += dpp_shr0_any<4>(v);
  v += dpp_shr0_any<8>(v);
  const T r0 = lane_any(v, 15), r1 = lane_any(v, 31), r2 = lane_any(v, 47);
  const uint32_t row = lane >> 4;
  const T add = row == 0 ? T(0) : row == 1 ? r0 : row == 2 ? T(r0 + r1) : T(r0 + r1 + r2);
  return v + add;
}

// Same reduction through ds_bpermute shuffles (probe variant kProbeShflReduce).
__device__ __forceinline__ uint32_t wave_xor_shfl(uint32_t v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v ^= __shfl_xor(v, m, 64);
  return v;
}

}  // namespace
}  // namespace lvkv

#endif  // LVKV_CRC32C_DEVICE_COMMON_H_
