// pow5_exhaustive.hip -- exhaustive checks of pow5_f (pt_math.hpp), the
// contract's pow(x, 5.0), over all 2^32 fp32 inputs on the GPU:
//   (a) against x^5 rounded to nearest-even from its exact value (m^5 in
//       128-bit integers), for every input whose result is a normal float;
//   (b) against the general pow_f(x, 5.0f) = exp2(5 * log2(x)) in double.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt
//        -fno-gpu-flush-denormals-to-zero -I simple-ray-tracer_amd/csrc tools/pow5_exhaustive.hip -o pow5_exhaustive
// Output: "EXACT_MISMATCH <n> CHECKED <n>", "POW_MISMATCH <n>", then up to 8 examples of (b).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

#include "pt_math.hpp"

using namespace srt::dev;
typedef unsigned __int128 u128;

// x^5 rounded to nearest-even, as fp32 bits; false when the result is not a
// normal float (zero, subnormal, overflow) or x is not a positive finite number
__device__ bool pow5_exact(float x, unsigned& out) {
  const unsigned b = __float_as_uint(x);
  const unsigned be = (b >> 23) & 0xFF;
  if ((b >> 31) || be == 0xFF || (b & 0x7FFFFFFF) == 0) return false;
  unsigned m = b & 0x7FFFFF;
  int e;  // x = m * 2^e
  if (be == 0) {
    e = -149;
  } else {
    m |= 0x800000;
    e = (int)be - 150;
  }
  u128 p = m;
  for (int i = 0; i < 4; ++i) p *= m;
  int len = 0;
  for (u128 t = p; t; t >>= 1) ++len;
  int shift = len - 24;  // keep 24 significant bits
  u128 q = p, rem = 0;
  bool half = false, above = false;
  if (shift > 0) {
    q = p >> shift;
    rem = p & ((((u128)1) << shift) - 1);
    const u128 h = ((u128)1) << (shift - 1);
    half = rem == h;
    above = rem > h;
  } else {
    q = p << (-shift);
  }
  if (above || (half && (q & 1))) ++q;
  if (q == (((u128)1) << 24)) {
    q >>= 1;
    ++shift;
  }
  const int exp2 = shift + 5 * e + 23;  // value = 1.xxx * 2^exp2
  const int biased = exp2 + 127;
  if (biased < 1 || biased > 254) return false;
  out = ((unsigned)biased << 23) | ((unsigned)q & 0x7FFFFF);
  return true;
}

__global__ void check(unsigned long long* cnt, unsigned* ex, unsigned long long base, unsigned long long n) {
  const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
  for (unsigned long long i = base + blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; i < base + n;
       i += stride) {
    const unsigned bits = (unsigned)i;
    const float x = __uint_as_float(bits);
    const float got = pow5_f(x);
    unsigned want;
    if (pow5_exact(x, want)) {
      atomicAdd(&cnt[1], 1ull);
      if (__float_as_uint(got) != want) atomicAdd(&cnt[0], 1ull);
    }
    const float ref = pow_f(x, 5.0f);
    if (!(ref != ref && got != got) && __float_as_uint(ref) != __float_as_uint(got)) {
      const unsigned long long k = atomicAdd(&cnt[2], 1ull);
      if (k < 8) ex[k] = bits;
    }
  }
}

int main() {
  unsigned long long* d_cnt = nullptr;
  unsigned* d_ex = nullptr;
  if (hipMalloc(&d_cnt, 3 * sizeof(unsigned long long)) != hipSuccess || hipMalloc(&d_ex, 8 * sizeof(unsigned)) != hipSuccess ||
      hipMemset(d_cnt, 0, 3 * sizeof(unsigned long long)) != hipSuccess || hipMemset(d_ex, 0, 8 * sizeof(unsigned)) != hipSuccess) {
    std::printf("HIP error\n");
    return 2;
  }
  const unsigned long long total = 1ull << 32, chunk = 1ull << 30;
  for (unsigned long long b = 0; b < total; b += chunk)
    hipLaunchKernelGGL(check, dim3(4096), dim3(256), 0, 0, d_cnt, d_ex, b, chunk);
  unsigned long long h[3];
  unsigned ex[8];
  if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(h, d_cnt, sizeof h, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(ex, d_ex, sizeof ex, hipMemcpyDeviceToHost) != hipSuccess) {
    std::printf("HIP error\n");
    return 2;
  }
  std::printf("EXACT_MISMATCH %llu CHECKED %llu\n", h[0], h[1]);
  std::printf("POW_MISMATCH %llu\n", h[2]);
  for (int k = 0; k < 8 && k < (int)h[2]; ++k) {
    float x;
    std::memcpy(&x, &ex[k], 4);
    std::printf("  e.g. 0x%08x = %.9g\n", ex[k], x);
  }
  return 0;
}
