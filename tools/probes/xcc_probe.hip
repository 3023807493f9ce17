#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
__global__ __launch_bounds__(256) void k(unsigned* out, int spin) {
  unsigned x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  if (threadIdx.x == 0) out[blockIdx.x] = x & 0xF;
  // keep blocks resident a while so the dispatcher fills every CU
  unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)spin) {}
}
int main() {
  const int nb = 1280;
  unsigned* d; (void)hipMalloc(&d, nb * 4);
  hipLaunchKernelGGL(k, dim3(nb), dim3(256), 0, 0, d, 10000);
  std::vector<unsigned> h(nb);
  (void)hipMemcpy(h.data(), d, nb * 4, hipMemcpyDeviceToHost);
  int match = 0; int hist[8][8] = {};
  for (int b = 0; b < nb; ++b) { match += (h[b] == (unsigned)(b % 8)); hist[b % 8][h[b] & 7]++; }
  printf("blocks %d: xcc == blockIdx %% 8 for %d\n", nb, match);
  for (int g = 0; g < 8; ++g) { printf("label %d ->", g); for (int x = 0; x < 8; ++x) printf(" %d", hist[g][x]); printf("\n"); }
  printf("first 24: "); for (int b = 0; b < 24; ++b) printf("%u ", h[b]); printf("\n");
  return 0;
}
