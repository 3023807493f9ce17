// rcp_exhaustive.hip -- exhaustive check of the 3-instruction reciprocal
// (v_rcp_f32 + one FMA Newton step) against the correctly rounded 1.0f / a,
// over all 2^32 fp32 bit patterns, bucketed by exponent.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt
//        -fno-gpu-flush-denormals-to-zero tools/rcp_exhaustive.hip -o rcp_exhaustive
// Output: one line per exponent bucket with mismatches, then "TOTAL <n>".
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

__device__ __forceinline__ float rcp_newton(float a) {
  const float r = __builtin_amdgcn_rcpf(a);
  const float e = __builtin_fmaf(-a, r, 1.0f);
  return __builtin_fmaf(e, r, r);
}

__global__ void check(unsigned long long* bucket, unsigned* first, unsigned long long base, unsigned long long n) {
  const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
  for (unsigned long long i = base + blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; i < base + n;
       i += stride) {
    const unsigned bits = (unsigned)i;
    const float a = __uint_as_float(bits);
    const float exact = 1.0f / a;
    const float fast = rcp_newton(a);
    const bool both_nan = exact != exact && fast != fast;
    if (!both_nan && __float_as_uint(exact) != __float_as_uint(fast)) {
      const unsigned e = (bits >> 23) & 0xFF;
      atomicAdd(&bucket[e], 1ull);
      atomicCAS(&first[e], 0u, bits);
    }
  }
}

int main() {
  unsigned long long* d_bucket;
  unsigned* d_first;
  hipMalloc(&d_bucket, 256 * sizeof(unsigned long long));
  hipMalloc(&d_first, 256 * sizeof(unsigned));
  hipMemset(d_bucket, 0, 256 * sizeof(unsigned long long));
  hipMemset(d_first, 0, 256 * sizeof(unsigned));
  const unsigned long long total = 1ull << 32, chunk = 1ull << 30;
  for (unsigned long long b = 0; b < total; b += chunk) hipLaunchKernelGGL(check, dim3(4096), dim3(256), 0, 0, d_bucket, d_first, b, chunk);
  if (hipDeviceSynchronize() != hipSuccess) {
    std::printf("HIP error\n");
    return 2;
  }
  unsigned long long h[256];
  unsigned f[256];
  hipMemcpy(h, d_bucket, sizeof h, hipMemcpyDeviceToHost);
  hipMemcpy(f, d_first, sizeof f, hipMemcpyDeviceToHost);
  unsigned long long sum = 0;
  for (int e = 0; e < 256; ++e) {
    if (!h[e]) continue;
    float a;
    std::memcpy(&a, &f[e], 4);
    std::printf("exp %3d (2^%d): %llu mismatches, e.g. 0x%08x = %g\n", e, e - 127, h[e], f[e], a);
    sum += h[e];
  }
  std::printf("TOTAL %llu\n", sum);
  return 0;
}
