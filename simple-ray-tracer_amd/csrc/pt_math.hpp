// pt_math.hpp -- device arithmetic contract of the path tracer (gfx950).
//
// The reference kernel's results are chaotic in its inputs: every random
// number is fract(sin(dot(hit_position, k)) * 43758.5453) indexing a noise
// buffer (shaders/raytrace_utils.glsl:28-54), so one ULP anywhere changes the
// path.  The kernel therefore follows a fixed arithmetic contract (DESIGN.md
// section 3) that the CPU oracle (oracle/srt_oracle.c) restates independently:
//   * IEEE fp32, source-order evaluation, no FMA contraction (-ffp-contract=off),
//     correctly rounded '/' and sqrt, denormals preserved;
//   * GLSL min/max/clamp with IEEE minNum/maxNum NaN handling;
//   * sin/cos: fp32 Cody-Waite reduction with FMA + minimax polynomials (below);
//     pow(x, y) = exp2(y * log2(x)) in double (x < 0 -> NaN);
//   * pow(x, 5.0) = x^5 rounded to nearest-even (pow5_f).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace srt {
namespace dev {

struct f3 {
  float x, y, z;
};

// ---- fast correctly rounded reciprocal ---------------------------------------
// 1.0f / b, correctly rounded.  v_rcp_f32 plus one FMA Newton step equals the
// correctly rounded reciprocal for every 2^-126 <= |b| < 2^126 (all 2^32 inputs
// checked on gfx950: tools/rcp_exhaustive.hip, tests/test_gpu_exhaustive_math.py);
// other b take the division on a branch skipped unless some lane needs it.
__device__ __forceinline__ float recip_newton(float b) {
  const float r = __builtin_amdgcn_rcpf(b);
  return __builtin_fmaf(__builtin_fmaf(-b, r, 1.0f), r, r);
}
__device__ __forceinline__ float recip_exact(float b) {
  float r = recip_newton(b);
  const float m = __builtin_fabsf(b);
  if (__builtin_expect(!(m >= 0x1p-126f && m < 0x1p126f), 0)) r = 1.0f / b;
  return r;
}

// ---- correctly rounded division ---------------------------------------------
// a / b, correctly rounded (the contract's '/').  SRT_FAST_DIV: the verified Newton reciprocal r of
// b, q = a * r, and one Markstein correction q + (a - b*q) * r with the residual exact in an FMA;
// equal to the IEEE quotient for every a, b inside the range checked below (2^-62 <= |a|, |b| <= 2^62,
// or a == 0: no intermediate over- or underflows, so the result is the same for every exponent
// pair), all 2^46 mantissa pairs checked on gfx950 (tools/div_exhaustive.hip); other inputs take
// the division on a branch that is skipped unless some lane needs it.  An exact quotient (zero
// residual) is q itself, which keeps the sign of a zero quotient.
#ifndef SRT_FAST_DIV
#define SRT_FAST_DIV 0
#endif
__device__ __forceinline__ float div_rn(float a, float b) {
#if SRT_FAST_DIV
  const float r = recip_newton(b);
  const float q = a * r;
  const float e = __builtin_fmaf(-b, q, a);
  float res = (e == 0.0f) ? q : __builtin_fmaf(e, r, q);
  const float ma = __builtin_fabsf(a), mb = __builtin_fabsf(b);
  const bool ok = (ma <= 0x1p62f) & ((ma >= 0x1p-62f) | (a == 0.0f)) & (mb >= 0x1p-62f) & (mb <= 0x1p62f);
  if (__builtin_expect(!ok, 0)) res = a / b;
  return res;
#else
  return a / b;
#endif
}

__device__ __forceinline__ f3 mk(float x, float y, float z) { return f3{x, y, z}; }
__device__ __forceinline__ f3 operator+(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ f3 operator-(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ f3 operator*(f3 a, f3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ f3 operator*(f3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ f3 operator*(float s, f3 a) { return mk(s * a.x, s * a.y, s * a.z); }
__device__ __forceinline__ f3 operator/(f3 a, float s) { return mk(div_rn(a.x, s), div_rn(a.y, s), div_rn(a.z, s)); }
__device__ __forceinline__ f3 operator-(f3 a) { return mk(-a.x, -a.y, -a.z); }
// GLSL dot / cross built-ins with fused multiply-adds, as GPU compilers evaluate
// them: dot = fma(z, z', fma(y, y', x * x')),
// cross_i = fma(a_j, b_k, -(a_k * b_j)); every other expression stays unfused.
__device__ __forceinline__ float dot(f3 a, f3 b) { return __builtin_fmaf(a.z, b.z, __builtin_fmaf(a.y, b.y, a.x * b.x)); }
__device__ __forceinline__ f3 cross(f3 a, f3 b) {
  return mk(__builtin_fmaf(a.y, b.z, -(a.z * b.y)), __builtin_fmaf(a.z, b.x, -(a.x * b.z)),
            __builtin_fmaf(a.x, b.y, -(a.y * b.x)));
}
__device__ __forceinline__ float length(f3 a) { return __builtin_sqrtf(dot(a, a)); }
__device__ __forceinline__ f3 normalize(f3 a) {
  const float inv = recip_exact(__builtin_sqrtf(dot(a, a)));
  return a * inv;
}
__device__ __forceinline__ float fmn(float a, float b) { return (b < a || a != a) ? b : a; }
__device__ __forceinline__ float fmx(float a, float b) { return (a < b || a != a) ? b : a; }
__device__ __forceinline__ float clampf(float x, float lo, float hi) { return fmn(fmx(x, lo), hi); }
__device__ __forceinline__ float sat(float x) { return clampf(x, 0.0f, 1.0f); }
__device__ __forceinline__ float fractf(float x) { return x - __builtin_floorf(x); }
__device__ __forceinline__ int f2i(float x) {
  if (x != x) return 0;
  if (x >= 2147483648.0f) return 2147483647;
  if (x <= -2147483648.0f) return (-2147483647 - 1);
  return (int)x;
}
__device__ __forceinline__ bool isinf_f(float x) { return __builtin_fabsf(x) == __builtin_inff(); }

#ifndef SRT_CONTRACT_HW
#define SRT_CONTRACT_HW 0
#endif
#if SRT_CONTRACT_HW
// ---- contract F: GLSL transcendentals as AMD's GPU compilers lower them ------
// A measurement build, never the default (make CONTRACT=F: libsrt_amd_F.so; DESIGN.md section 3,
// "Tolerance").  A GL/Vulkan driver on gfx9+ lowers GLSL sin/cos to the hardware instructions on the
// argument in revolutions -- v_mul_f32 by 1/(2 pi), then v_sin_f32 / v_cos_f32, with no further range
// reduction (LLVM AMDGPU LowerTrig; only GFX8 inserts v_fract_f32) -- and pow(x, y) to
// v_exp_f32(y * v_log_f32(x)).  The random numbers of raytrace_utils.glsl:28-54 go through that sin at
// |x| ~ 1e3-1e4, so F moves every path; the oracle cannot restate these instructions, so F is
// compared with contract A on the GPU (tools/contract_f.py).
__device__ __forceinline__ float sin_f(float x) { return __builtin_amdgcn_sinf(x * 0x1.45f306p-3f); }
__device__ __forceinline__ float cos_f(float x) { return __builtin_amdgcn_cosf(x * 0x1.45f306p-3f); }
__device__ __forceinline__ float pow_f(float x, float y) {
  return __builtin_amdgcn_exp2f(y * __builtin_amdgcn_logf(x));
}
__device__ __forceinline__ float pow5_f(float x) { return pow_f(x, 5.0f); }
#else
// ---- sin / cos ------------------------------------------------------------
// The contract's sin/cos, in fp32 with fused multiply-adds:
// k = rint(x * 2/pi); r = x - k * pi/2 with pi/2 = P1 + P2 + P3 (each product
// exact inside its FMA); then minimax polynomials on [-pi/4, pi/4] (Cephes
// sinf/cosf coefficients) and the quadrant's sign/selection.  |x| >= 2^30
// gives 0, NaN and Inf give NaN.  oracle/srt_oracle.c evaluates the same
// expressions with fmaf/rintf.
__device__ __forceinline__ float sincos_kernel(float x, int want_cos) {
  if (x != x || isinf_f(x)) return __builtin_nanf("");
  if (__builtin_fabsf(x) >= 0x1p30f) return 0.0f;
  const float kf = __builtin_rintf(x * 0x1.45f306p-1f);
  float r = __builtin_fmaf(-kf, 0x1.921fb6p+0f, x);
  r = __builtin_fmaf(-kf, -0x1.777a5cp-25f, r);
  r = __builtin_fmaf(-kf, -0x1.ee59dap-50f, r);
  const float z = r * r;
  const float ps = __builtin_fmaf(__builtin_fmaf(-0x1.9943f2p-13f, z, 0x1.11073cp-7f), z, -0x1.555546p-3f);
  const float s = __builtin_fmaf(ps * z, r, r);
  const float pc = __builtin_fmaf(__builtin_fmaf(0x1.99eb9cp-16f, z, -0x1.6c0c34p-10f), z, 0x1.55554ap-5f);
  const float c = __builtin_fmaf(pc * z, z, __builtin_fmaf(-0.5f, z, 1.0f));
  const int q = ((int)kf + want_cos) & 3;
  const float v = (q & 1) ? c : s;
  return (q & 2) ? -v : v;
}
__device__ __forceinline__ float sin_f(float x) { return sincos_kernel(x, 0); }
__device__ __forceinline__ float cos_f(float x) { return sincos_kernel(x, 1); }

// ---- pow ------------------------------------------------------------------
__constant__ static const double kInvC[32] = {
  0x1.f81f81f81f820p-1, 0x1.e9131abf0b767p-1, 0x1.dae6076b981dbp-1, 0x1.cd85689039b0bp-1,
  0x1.c0e070381c0e0p-1, 0x1.b4e81b4e81b4fp-1, 0x1.a98ef606a63bep-1, 0x1.9ec8e951033d9p-1,
  0x1.948b0fcd6e9e0p-1, 0x1.8acb90f6bf3aap-1, 0x1.8181818181818p-1, 0x1.78a4c8178a4c8p-1,
  0x1.702e05c0b8170p-1, 0x1.6816816816817p-1, 0x1.6058160581606p-1, 0x1.58ed2308158edp-1,
  0x1.51d07eae2f815p-1, 0x1.4afd6a052bf5bp-1, 0x1.446f86562d9fbp-1, 0x1.3e22cbce4a902p-1,
  0x1.3813813813814p-1, 0x1.323e34a2b10bfp-1, 0x1.2c9fb4d812ca0p-1, 0x1.27350b8812735p-1,
  0x1.21fb78121fb78p-1, 0x1.1cf06ada2811dp-1, 0x1.1811811811812p-1, 0x1.135c81135c811p-1,
  0x1.0ecf56be69c90p-1, 0x1.0a6810a6810a7p-1, 0x1.0624dd2f1a9fcp-1, 0x1.0204081020408p-1};
__constant__ static const double kLog2C[32] = {
  0x1.6e79685c2d22ap-6, 0x1.0eb389fa29f9bp-4, 0x1.bc84240adabbap-4, 0x1.32ae9e278ae1ap-3,
  0x1.84c2bd02f03b3p-3, 0x1.d49ee4c325970p-3, 0x1.11307dad30b76p-2, 0x1.37124cea4cdedp-2,
  0x1.5c01a39fbd688p-2, 0x1.800a563161c54p-2, 0x1.a33760a7f6051p-2, 0x1.c592fad295b56p-2,
  0x1.e726aa1e754d2p-2, 0x1.03fda8b97997fp-1, 0x1.140c9faa1e544p-1, 0x1.23c41d42727c8p-1,
  0x1.3327c6ab49ca7p-1, 0x1.423b07e986aa9p-1, 0x1.510118708a8f9p-1, 0x1.5f7cff41e09afp-1,
  0x1.6db196a76194ap-1, 0x1.7ba18f93502e4p-1, 0x1.894f74b06ef8bp-1, 0x1.96bdad2acb5f6p-1,
  0x1.a3ee7f38e181fp-1, 0x1.b0e4126bcc86cp-1, 0x1.bda071cc67e6ep-1, 0x1.ca258dca93316p-1,
  0x1.d6753e032ea0fp-1, 0x1.e29142e0e0140p-1, 0x1.ee7b471b3a950p-1, 0x1.fa34e1177c233p-1};

__device__ __forceinline__ double log2_pos(float xf) {
  uint32_t b = __builtin_bit_cast(uint32_t, xf);
  int e = (int)(b >> 23) - 127;
  uint32_t m = b & 0x7FFFFFu;
  if ((b >> 23) == 0) {
    const int lz = __builtin_clz(m) - 8;  // shifts to bring the leading one to bit 23
    m = (m << lz) & 0x7FFFFFu;
    e = -126 - lz;
  }
  const double md = 1.0 + (double)m * 0x1p-23;
  const int j = (int)(m >> 18);
  const double f = md * kInvC[j] - 1.0;
  const double p = f * (1.0 + f * (-0x1.0000000000000p-1 + f * (0x1.5555555555555p-2 + f * (-0x1.0000000000000p-2 +
                   f * (0x1.999999999999ap-3 + f * (-0x1.5555555555555p-3 + f * (0x1.2492492492492p-3 +
                   f * (-0x1.0000000000000p-3 + f * 0x1.c71c71c71c71cp-4))))))));
  return ((double)e + kLog2C[j]) + p * 0x1.71547652b82fep+0;
}
__device__ __forceinline__ double exp2_d(double t) {
  if (t != t) return t;
  if (t > 130.0) return __builtin_inf();
  if (t < -160.0) return 0.0;
  const double n = __builtin_rint(t);
  const double g = (t - n) * 0x1.62e42fefa39efp-1;
  const double p = 1.0 + g * (1.0 + g * (0x1.0000000000000p-1 + g * (0x1.5555555555555p-3 + g * (0x1.5555555555555p-5 +
                   g * (0x1.1111111111111p-7 + g * (0x1.6c16c16c16c17p-10 + g * (0x1.a01a01a01a01ap-13 +
                   g * (0x1.a01a01a01a01ap-16 + g * (0x1.71de3a556c734p-19 + g * (0x1.27e4fb7789f5cp-22 +
                   g * (0x1.ae64567f544e4p-26 + g * 0x1.1eed8eff8d898p-29)))))))))));
  const uint64_t eb = (uint64_t)((long long)n + 1023) << 52;
  return p * __builtin_bit_cast(double, eb);
}
__device__ __forceinline__ float pow_f(float x, float y) {
  if (x != x || y != y) return __builtin_nanf("");
  if (x < 0.0f) return __builtin_nanf("");
  if (x == 0.0f) return (y > 0.0f) ? 0.0f : (y == 0.0f ? __builtin_nanf("") : __builtin_inff());
  if (x == __builtin_inff()) return (y > 0.0f) ? __builtin_inff() : (y == 0.0f ? __builtin_nanf("") : 0.0f);
  return (float)exp2_d((double)y * log2_pos(x));
}

// pow(x, 5.0) (the Fresnel terms, brdf.glsl): x^5 by multiplication in
// double -- x^2 exact, x^4 and x^5 rounded to double -- then rounded to float.
// GLSL domain as pow_f: x < 0 and NaN give NaN, +-0 gives +0.  It differs from
// pow_f(x, 5.0f) = exp2(5 * log2(x)) in 92 of 2^32 inputs, all exact float
// midpoints such as x = 1.8125, where this form rounds half to even
// (tools/pow5_exhaustive.hip).
__device__ __forceinline__ float pow5_f(float x) {
  if (!(x >= 0.0f)) return __builtin_nanf("");
  const double d = (double)x;
  const double d2 = d * d;
  return x == 0.0f ? 0.0f : (float)((d2 * d2) * d);
}
#endif  // SRT_CONTRACT_HW

}  // namespace dev
}  // namespace srt
