// Prints what xpose_rows (crc32c_wide.hip) does to lane/register ids on the GPU.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* o) {
  const unsigned L = threadIdx.x;
  unsigned v0 = L * 4 + 0, v1 = L * 4 + 1, v2 = L * 4 + 2, v3 = L * 4 + 3;  // word ids
  const auto a = __builtin_amdgcn_permlane32_swap(v0, v2, false, false);
  const auto b = __builtin_amdgcn_permlane32_swap(v1, v3, false, false);
  const auto c = __builtin_amdgcn_permlane16_swap(a[0], b[0], false, false);
  const auto d = __builtin_amdgcn_permlane16_swap(a[1], b[1], false, false);
  o[L * 4 + 0] = c[0]; o[L * 4 + 1] = c[1]; o[L * 4 + 2] = d[0]; o[L * 4 + 3] = d[1];
  const auto e = __builtin_amdgcn_permlane32_swap(L, 100 + L, false, false);
  o[256 + L * 2] = e[0]; o[256 + L * 2 + 1] = e[1];
  const auto f = __builtin_amdgcn_permlane16_swap(L, 100 + L, false, false);
  o[384 + L * 2] = f[0]; o[384 + L * 2 + 1] = f[1];
}
int main() {
  unsigned* d; unsigned h[512];
  (void)hipMalloc(&d, sizeof(h));
  k<<<1, 64>>>(d);
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  int bad = 0;
  for (unsigned L = 0; L < 64; ++L)
    for (unsigned q = 0; q < 4; ++q) {
      unsigned want = 64 * q + 4 * (L & 15) + (L >> 4);
      if (h[L * 4 + q] != want) ++bad;
    }
  printf("xpose mismatches: %d\n", bad);
  for (unsigned L = 0; L < 64; L += 5) printf("L=%2u regs: %3u %3u %3u %3u\n", L, h[L*4], h[L*4+1], h[L*4+2], h[L*4+3]);
  printf("permlane32_swap(L, 100+L): ");
  for (unsigned L = 0; L < 64; L += 9) printf("[%u: %u %u] ", L, h[256 + 2*L], h[257 + 2*L]);
  printf("\npermlane16_swap(L, 100+L): ");
  for (unsigned L = 0; L < 64; L += 9) printf("[%u: %u %u] ", L, h[384 + 2*L], h[385 + 2*L]);
  printf("\n");
  return 0;
}
