// How much LDS a block may take so that n blocks of 256 lanes still run together on every CU (gfx950).
// n * 256 blocks each wait ~2 ms; a launch that takes ~2 ms ran them together, ~4 ms means a CU held
// fewer (hipOccupancyMaxActiveBlocksPerMultiprocessor's answer is printed beside it).  Build: hipcc --offload-arch=gfx950 -O2 -o tools/probes/lds_fit tools/probes/lds_fit.hip
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void hold(int* sink, long long cycles) {
  extern __shared__ int lds[];
  lds[threadIdx.x] = threadIdx.x;
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < cycles) __builtin_amdgcn_s_sleep(8);
  __syncthreads();
  if (lds[(threadIdx.x + 1) & 255] == -1) sink[0] = 1;  // keeps the LDS use
}

int main() {
  int* sink;
  (void)hipMalloc(&sink, 4);
  int dev = 0, cus = 0, rate = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  (void)hipDeviceGetAttribute(&rate, hipDeviceAttributeWallClockRate, dev);  // kHz
  const long long cycles = (long long)rate * 2;                               // ~2 ms
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  // n blocks per CU, each asking floor(128 / n) * 1280 bytes (the largest multiple of 1/128 of the CU's 160 KB
  // that n blocks share) and one byte more; and the 5-block sweep the round-6 region experiment ran into
  struct Run { int per, lds; };
  Run runs[64];
  int nr = 0;
  for (int per = 2; per <= 8; ++per) {
    const int fit = (128 / per) * 1280;
    runs[nr++] = {per, fit};
    if (fit + 1 <= 65536) runs[nr++] = {per, fit + 1};
  }
  const int sweep[] = {31744, 32000, 32001, 32256, 32512, 32768};
  for (int v : sweep) runs[nr++] = {5, v};
  printf("{\"cus\": %d, \"wall_clock_khz\": %d, \"runs\": [\n", cus, rate);
  for (int k = 0; k < nr; ++k) {
    int occ = 0;
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, hold, 256, runs[k].lds);
    float best = 1e9f;
    for (int rep = 0; rep < 3; ++rep) {
      (void)hipEventRecord(a);
      hipLaunchKernelGGL(hold, dim3(cus * runs[k].per), dim3(256), runs[k].lds, 0, sink, cycles);
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, a, b);
      if (ms < best) best = ms;
    }
    printf("  {\"blocks_per_cu\": %d, \"lds_bytes\": %d, \"api_blocks_per_cu\": %d, \"ms\": %.3f, \"together\": %s}%s\n",
           runs[k].per, runs[k].lds, occ, best, best < 3.0f ? "true" : "false", k + 1 == nr ? "" : ",");
  }
  printf("]}\n");
  return 0;
}
