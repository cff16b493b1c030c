// LDS round-trip latency as the WAL header walk sees it: one wave chases a
// chain of dependent LDS reads (uniform address, the next offset read from
// LDS), alone or beside 7 busy waves. Prints ns and shader cycles per step.
// Build: hipcc --offload-arch=gfx950 -O3 tools/lds_latency.hip -o build/lds_latency
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kSteps = 4096;

template <int kBusy>
__global__ void __launch_bounds__(512) chase(uint64_t* out, uint32_t seed) {
  __shared__ uint32_t lds[8192];
  for (uint32_t i = threadIdx.x; i < 8192; i += blockDim.x)
    lds[i] = ((i * 2654435761u + seed) & 8191u) * 4u;  // a byte offset
  __syncthreads();
  const uint32_t wave = threadIdx.x >> 6;
  if (wave == 1) {
    uint32_t p = 0;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < kSteps; ++i)
      p = __builtin_amdgcn_readfirstlane(
          *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(lds) + p));
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    const uint64_t c1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 64 && blockIdx.x == 0) {
      out[0] = t1 - t0;
      out[1] = c1 - c0;
      out[2] = p;
    }
  } else if (kBusy) {
    // the other waves: independent LDS reads (the record CRCs' load)
    uint32_t acc = threadIdx.x, q = threadIdx.x * 4u;
    for (int i = 0; i < kSteps; ++i) {
      acc ^= *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(lds) + (q & 32767u));
      q += 260u;
    }
    if (acc == 0x12345678u) out[3] = acc;
  }
}

int main() {
  uint64_t* d;
  (void)hipMalloc(&d, 64);
  uint64_t h[4];
  for (int busy = 0; busy < 2; ++busy) {
    for (int rep = 0; rep < 3; ++rep) {
      if (busy) hipLaunchKernelGGL(chase<1>, dim3(256), dim3(512), 0, 0, d, 12345u);
      else hipLaunchKernelGGL(chase<0>, dim3(256), dim3(512), 0, 0, d, 12345u);
      (void)hipDeviceSynchronize();
    }
    (void)hipMemcpy(h, d, 32, hipMemcpyDeviceToHost);
    std::printf("busy=%d: %.1f ns/step, %.1f memtime ticks/step\n", busy,
                h[0] * 10.0 / kSteps, static_cast<double>(h[1]) / kSteps);
  }
  return 0;
}
