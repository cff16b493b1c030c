// Launch-cost probe: empty kernels of different shapes, timed back to back
// with hipEvents; run under `rocprofv3 --kernel-trace --stats` for device
// times. Build: hipcc --offload-arch=gfx950 -O3 tools/launch_probe.hip -o launch_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

template <int kThreads, int kLdsDwords>
__global__ void __launch_bounds__(kThreads) empty_kernel(int flag, int* out) {
  if constexpr (kLdsDwords > 0) {
    __shared__ uint32_t lds[kLdsDwords];
    if (flag == 12345) {
      lds[threadIdx.x] = threadIdx.x;
      __syncthreads();
      out[0] = lds[(threadIdx.x + 1) % kThreads];
    }
  } else {
    if (flag == 12345) out[0] = 1;
  }
}

template <int T, int L>
float time_it(int groups, int* out, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int i = 0; i < 5; ++i) empty_kernel<T, L><<<groups, T>>>(0, out);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(a);
  for (int i = 0; i < reps; ++i) empty_kernel<T, L><<<groups, T>>>(0, out);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms * 1000.0f / reps;
}

int main() {
  int* out;
  (void)hipMalloc(&out, 64);
  const int reps = 200;
  printf("back-to-back average (us per launch):\n");
  printf("  256 thr x 2048 WG, no LDS      %.2f\n", time_it<256, 0>(2048, out, reps));
  printf("  256 thr x 256 WG, no LDS       %.2f\n", time_it<256, 0>(256, out, reps));
  printf("  1024 thr x 256 WG, no LDS      %.2f\n", time_it<1024, 0>(256, out, reps));
  printf("  1024 thr x 256 WG, 64 KiB LDS  %.2f\n", time_it<1024, 16384>(256, out, reps));
  printf("  1024 thr x 256 WG, 160 KiB LDS %.2f\n", time_it<1024, 40960>(256, out, reps));
  printf("  512 thr x 256 WG, 160 KiB LDS  %.2f\n", time_it<512, 40960>(256, out, reps));
  printf("  256 thr x 256 WG, 160 KiB LDS  %.2f\n", time_it<256, 40960>(256, out, reps));
  printf("  1024 thr x 512 WG, 80 KiB LDS  %.2f\n", time_it<1024, 20480>(512, out, reps));
  return 0;
}
