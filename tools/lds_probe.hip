// LDS table-walk microbenchmark: the batch kernel's row step (4 x v_perm +
// 4 x bank-private ds_read_b32 + xors) in isolation, for CHAINS independent
// chains per wave and WAVES waves per workgroup (one workgroup per CU, 160 KiB
// LDS). Prints lookups per CU per ns.
// Build: hipcc --offload-arch=gfx950 -O3 tools/lds_probe.hip -o lds_probe
#include <hip/hip_runtime.h>

#include <cstdio>

__device__ __forceinline__ uint32_t lds_ld(const uint32_t* lds, uint32_t a) {
  return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(lds) + a);
}

template <int MODE>
__device__ __forceinline__ uint32_t step(const uint32_t* lds, uint32_t s, uint32_t k0, uint32_t k1) {
  if (MODE == 0) {  // production: v_perm addresses, 4 lookups, xor
    const uint32_t a0 = __builtin_amdgcn_perm(s, k0, 0x0C020400u);
    const uint32_t a1 = __builtin_amdgcn_perm(s, k0, 0x0C020500u);
    const uint32_t a2 = __builtin_amdgcn_perm(s, k1, 0x0C020600u);
    const uint32_t a3 = __builtin_amdgcn_perm(s, k1, 0x0C020700u);
    return lds_ld(lds, a0) ^ lds_ld(lds, a1 + 128u) ^ lds_ld(lds, a2) ^ lds_ld(lds, a3 + 128u);
  } else if (MODE == 1) {  // same addresses for all lanes of a row (broadcast)
    const uint32_t a0 = (s & 0xff) << 8;
    return lds_ld(lds, a0) ^ lds_ld(lds, a0 + 128u) ^ lds_ld(lds, a0 + 65536u) ^ lds_ld(lds, a0 + 65536u + 128u);
  } else {  // VALU only: same perms, xor instead of lookups
    const uint32_t a0 = __builtin_amdgcn_perm(s, k0, 0x0C020400u);
    const uint32_t a1 = __builtin_amdgcn_perm(s, k0, 0x0C020500u);
    const uint32_t a2 = __builtin_amdgcn_perm(s, k1, 0x0C020600u);
    const uint32_t a3 = __builtin_amdgcn_perm(s, k1, 0x0C020700u);
    return (a0 * 0x9E3779B1u) ^ a1 ^ (a2 >> 3) ^ a3;
  }
}

template <int CHAINS, int MODE>
__global__ void __launch_bounds__(1024) probe(uint32_t* out, int steps) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[40960];
  for (int i = threadIdx.x; i < 40960; i += blockDim.x) lds[i] = i * 0x9E3779B1u;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t k0 = (lane & 31) * 4, k1 = k0 | 0x10000;
  uint32_t s[CHAINS];
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) s[c] = lane * 7919u + c * 104729u + blockIdx.x;
  for (int i = 0; i < steps; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s[c] = step<MODE>(lds, s[c], k0, k1) ^ static_cast<uint32_t>(i);
  }
  uint32_t r = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) r ^= s[c];
  if (r == 0x12345678u) out[0] = r;
}

template <int CHAINS, int MODE>
void run(int waves, int ncu, int steps, uint32_t* out, const char* name) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  probe<CHAINS, MODE><<<ncu, waves * 64>>>(out, steps);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(a);
  const int reps = 10;
  for (int r = 0; r < reps; ++r) probe<CHAINS, MODE><<<ncu, waves * 64>>>(out, steps);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  const double us = ms * 1000.0 / reps;
  const double lookups_per_cu = 4.0 * CHAINS * steps * waves * 64;  // lane-lookups
  const double wave_instr_per_cu = 4.0 * CHAINS * steps * waves;    // ds_read wave-instructions
  printf("%-22s chains=%d waves=%2d  %8.1f us  %6.2f lane-lookups/ns/CU  %6.3f ds_read/ns/CU\n", name,
         CHAINS, waves, us, lookups_per_cu / (us * 1000.0), wave_instr_per_cu / (us * 1000.0));
}

int main() {
  int ncu = 0;
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  uint32_t* out;
  (void)hipMalloc(&out, 64);
  const int steps = 4096;
  for (int w : {4, 8, 16}) {
    run<1, 0>(w, ncu, steps, out, "perm+lds");
    run<2, 0>(w, ncu, steps, out, "perm+lds");
    run<4, 0>(w, ncu, steps, out, "perm+lds");
  }
  run<2, 1>(16, ncu, steps, out, "broadcast lds");
  run<2, 2>(16, ncu, steps, out, "valu only");
  run<4, 2>(16, ncu, steps, out, "valu only");
  return 0;
}
