// sin_probe.hip -- how gfx950's v_sin_f32 evaluates GLSL sin as AMD's GPU compilers emit it
// (v_mul_f32 by 1/(2 pi), then v_sin_f32 on the argument in revolutions; contract F, DESIGN.md
// section 3).  The reference's RNG (raytrace_utils.glsl:28-30) takes sin of dot(seed, (12.9898,
// 78.233)) with |x| up to ~1e4, i.e. up to ~1600 revolutions.  For |x| in decades 1e0..1e5 this prints
// the max / mean absolute error against sin in double, and how many results are exactly 0.
// Build + run (GPU box): hipcc -O2 --offload-arch=gfx950 tools/probes/sin_probe.hip -o /tmp/sin_probe && /tmp/sin_probe
// TEST INFRASTRUCTURE (a measurement probe).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

__global__ void probe(const float* x, float* s, float* c, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float r = x[i] * 0x1.45f306p-3f;
  s[i] = __builtin_amdgcn_sinf(r);
  c[i] = __builtin_amdgcn_cosf(r);
}

int main() {
  const int per = 1 << 20;
  const double decades[][2] = {{1, 10}, {10, 100}, {100, 1000}, {1000, 1e4}, {1e4, 1e5}};
  const int nd = 5, n = per * nd;
  std::vector<float> x(n), s(n), c(n);
  unsigned long long st = 0x9E3779B97F4A7C15ull;
  for (int d = 0; d < nd; ++d)
    for (int i = 0; i < per; ++i) {
      st ^= st << 13; st ^= st >> 7; st ^= st << 17;
      const double u = (double)(st >> 11) * 0x1p-53;
      const double v = decades[d][0] * std::pow(decades[d][1] / decades[d][0], u);
      x[(size_t)d * per + i] = (float)((i & 1) ? -v : v);
    }
  float *dx, *ds, *dc;
  if (hipMalloc(&dx, n * 4) || hipMalloc(&ds, n * 4) || hipMalloc(&dc, n * 4)) return 1;
  if (hipMemcpy(dx, x.data(), n * 4, hipMemcpyHostToDevice)) return 1;
  hipLaunchKernelGGL(probe, dim3((n + 255) / 256), dim3(256), 0, 0, dx, ds, dc, n);
  if (hipMemcpy(s.data(), ds, n * 4, hipMemcpyDeviceToHost) || hipMemcpy(c.data(), dc, n * 4, hipMemcpyDeviceToHost))
    return 1;
  std::printf("{\"probe\": \"v_sin_f32/v_cos_f32 of (float)(x * 1/(2 pi)) vs double sin/cos of x\", \"decades\": [");
  for (int d = 0; d < nd; ++d) {
    double emax = 0, esum = 0, cmax = 0;
    long zeros = 0;
    for (int i = 0; i < per; ++i) {
      const size_t k = (size_t)d * per + i;
      const double e = std::fabs((double)s[k] - std::sin((double)x[k]));
      const double ec = std::fabs((double)c[k] - std::cos((double)x[k]));
      emax = std::fmax(emax, e);
      cmax = std::fmax(cmax, ec);
      esum += e;
      zeros += s[k] == 0.0f;
    }
    std::printf("%s{\"abs_x\": [%g, %g], \"sin_err_max\": %.3e, \"sin_err_mean\": %.3e, \"cos_err_max\": %.3e, "
                "\"sin_exact_zero\": %ld}",
                d ? ", " : "", decades[d][0], decades[d][1], emax, esum / per, cmax, zeros);
  }
  std::printf("]}\n");
  return 0;
}
