/*
 * srt_oracle.c -- TEST INFRASTRUCTURE ONLY (see srt_oracle.h).
 *
 * Scalar C restatement of the reference GLSL path tracer.  Every function
 * cites the reference file:line it follows.  Arithmetic contract (DESIGN.md
 * section 3): IEEE fp32, source-order evaluation, no FMA contraction
 * (-ffp-contract=off) outside the dot/cross built-ins, correctly rounded '/'
 * and sqrt, GLSL min/max/clamp with IEEE minNum/maxNum NaN handling, sin/cos/pow
 * by the procedures below (shared specification with the HIP kernel, written
 * out independently here).
 *
 * ORACLE_CONTRACT selects a contract variant (oracle/Makefile builds one
 * library per variant).  Only the tolerance measurement uses the variants
 * (tools/contract_tolerance.py, tests/test_contract_tolerance.py): GLSL leaves
 * these choices to the implementation, so how far the converged image moves
 * between them bounds what "matches the GLSL render" can mean.
 *   0 (A) the kernel's contract (the default library, liboracle.so);
 *   1 (B) no FMA anywhere in expressions: dot/cross/luminance and the RNG
 *         seed's dot unfused (SURVEY.md 8a's original contract);
 *   2 (C) every a*b+c contracted, as a fusing GLSL compiler does: A compiled
 *         with -ffp-contract=fast -mfma (GetRay's pixelSample, the hit point
 *         dist*dir+origin, SampleDiffuse's sums, the BRDF terms, ...);
 *   3 (D) sin/cos in double precision rounded to float (correctly rounded
 *         unless the double result lies within 2^-29 ulp of a float midpoint);
 *   4 (E) B and D together: the round-1 contract (tests/golden/
 *         contract_e_renders.json pins it against that round's golden renders).
 */
#include "srt_oracle.h"

#include <math.h>
#include <string.h>
#include <stdint.h>
#include <stdlib.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------ */
/* scalar primitives                                                   */
/* ------------------------------------------------------------------ */
typedef struct { float x, y, z; } v3;

static inline v3 V(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 add(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 sub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 mul(v3 a, v3 b) { return V(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 muls(v3 a, float s) { return V(a.x * s, a.y * s, a.z * s); }
static inline v3 smul(float s, v3 a) { return V(s * a.x, s * a.y, s * a.z); }
static inline v3 divs(v3 a, float s) { return V(a.x / s, a.y / s, a.z / s); }
static inline v3 neg(v3 a) { return V(-a.x, -a.y, -a.z); }
#ifndef ORACLE_CONTRACT
#define ORACLE_CONTRACT 0
#endif
#define CTR_UNFUSED (ORACLE_CONTRACT == 1 || ORACLE_CONTRACT == 4)  /* B, E */
#define CTR_DSIN (ORACLE_CONTRACT == 3 || ORACLE_CONTRACT == 4)     /* D, E */
#if CTR_UNFUSED
/* variants B, E: the built-ins as written, left to right, every product rounded */
static inline float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline v3 cross(v3 a, v3 b) {
  return V(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
#else
/* GLSL dot / cross built-ins with fused multiply-adds:
 * dot = fma(z, z', fma(y, y', x * x')), cross_i = fma(a_j, b_k, -(a_k * b_j)). */
static inline float dot(v3 a, v3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
static inline v3 cross(v3 a, v3 b) {
  return V(fmaf(a.y, b.z, -(a.z * b.y)), fmaf(a.z, b.x, -(a.x * b.z)), fmaf(a.x, b.y, -(a.y * b.x)));
}
#endif
static inline float length3(v3 a) { return sqrtf(dot(a, a)); }
static inline v3 normalize3(v3 a) { float inv = 1.0f / sqrtf(dot(a, a)); return muls(a, inv); }
/* GLSL min/max with IEEE minNum/maxNum NaN handling (the non-NaN operand wins). */
static inline float fmn(float a, float b) { return (b < a || a != a) ? b : a; }
static inline float fmx(float a, float b) { return (a < b || a != a) ? b : a; }
static inline float clampf(float x, float lo, float hi) { return fmn(fmx(x, lo), hi); }
static inline float sat(float x) { return clampf(x, 0.0f, 1.0f); }
static inline float fractf(float x) { return x - floorf(x); }
/* float -> int32 as the hardware converts (NaN -> 0, saturating) */
static inline int f2i(float x) {
  if (x != x) return 0;
  if (x >= 2147483648.0f) return 2147483647;
  if (x <= -2147483648.0f) return (-2147483647 - 1);
  return (int)x;
}
static inline v3 vload(const float* p) { return V(p[0], p[1], p[2]); }

/* ---- sin / cos -----------------------------------
 * fp32 with fused multiply-adds: k = rint(x * 2/pi); r = x - k * pi/2 with
 * pi/2 = P1 + P2 + P3 (each product exact inside its fmaf); then the Cephes
 * sinf/cosf minimax polynomials on [-pi/4, pi/4] and the quadrant's
 * sign/selection.  |x| >= 2^30 gives 0, NaN and Inf give NaN.  The kernel
 * (simple-ray-tracer_amd/csrc/pt_math.hpp) evaluates the same expressions. */
#if CTR_DSIN
/* variants D, E: double-precision Cody-Waite reduction (pi/2 in two parts) and
 * the fdlibm kernel polynomials, rounded once to float (the round-1 contract) */
static void sincos_kernel(float xf, int want_cos, float* out) {
  if (xf != xf || xf == INFINITY || xf == -INFINITY) { *out = NAN; return; }
  if (fabsf(xf) >= 0x1p30f) { *out = 0.0f; return; }
  const double x = (double)xf;
  const double kd = rint(x * 0x1.45f306dc9c883p-1);
  const long long k = (long long)kd;
  const double r = (x - kd * 0x1.921fb54400000p+0) - kd * 0x1.0b4611a626331p-34;
  const double z = r * r;
  const double s = r + (r * z) * (-1.66666666666666324348e-01 + z * (8.33333333332248946124e-03 +
                   z * (-1.98412698298579493134e-04 + z * (2.75573137070700676789e-06 +
                   z * (-2.50507602534068634195e-08 + z * 1.58969099521155010221e-10)))));
  const double c = (1.0 - 0.5 * z) + (z * z) * (4.16666666666666019037e-02 + z * (-1.38888888888741095749e-03 +
                   z * (2.48015872894767294178e-05 + z * (-2.75573143513906633035e-07 +
                   z * (2.08757232129817482790e-09 + z * -1.13596475577881948265e-11)))));
  const int q = (int)((k + (want_cos ? 1 : 0)) & 3);
  const double v = (q == 0) ? s : (q == 1) ? c : (q == 2) ? -s : -c;
  *out = (float)v;
}
#else
static void sincos_kernel(float x, int want_cos, float* out) {
  if (x != x || x == INFINITY || x == -INFINITY) { *out = NAN; return; }
  if (fabsf(x) >= 0x1p30f) { *out = 0.0f; return; }
  const float kf = rintf(x * 0x1.45f306p-1f);
  float r = fmaf(-kf, 0x1.921fb6p+0f, x);
  r = fmaf(-kf, -0x1.777a5cp-25f, r);
  r = fmaf(-kf, -0x1.ee59dap-50f, r);
  const float z = r * r;
  const float ps = fmaf(fmaf(-0x1.9943f2p-13f, z, 0x1.11073cp-7f), z, -0x1.555546p-3f);
  const float s = fmaf(ps * z, r, r);
  const float pc = fmaf(fmaf(0x1.99eb9cp-16f, z, -0x1.6c0c34p-10f), z, 0x1.55554ap-5f);
  const float c = fmaf(pc * z, z, fmaf(-0.5f, z, 1.0f));
  const int q = ((int)kf + (want_cos ? 1 : 0)) & 3;
  const float v = (q & 1) ? c : s;
  *out = (q & 2) ? -v : v;
}
#endif
float oracle_sin(float x) { float r; sincos_kernel(x, 0, &r); return r; }
float oracle_cos(float x) { float r; sincos_kernel(x, 1, &r); return r; }

/* ---- pow(x, y) = exp2(y * log2(x)) in double (GLSL pow definition) ---- */
static const double kInvC[32] = {
  0x1.f81f81f81f820p-1, 0x1.e9131abf0b767p-1, 0x1.dae6076b981dbp-1, 0x1.cd85689039b0bp-1,
  0x1.c0e070381c0e0p-1, 0x1.b4e81b4e81b4fp-1, 0x1.a98ef606a63bep-1, 0x1.9ec8e951033d9p-1,
  0x1.948b0fcd6e9e0p-1, 0x1.8acb90f6bf3aap-1, 0x1.8181818181818p-1, 0x1.78a4c8178a4c8p-1,
  0x1.702e05c0b8170p-1, 0x1.6816816816817p-1, 0x1.6058160581606p-1, 0x1.58ed2308158edp-1,
  0x1.51d07eae2f815p-1, 0x1.4afd6a052bf5bp-1, 0x1.446f86562d9fbp-1, 0x1.3e22cbce4a902p-1,
  0x1.3813813813814p-1, 0x1.323e34a2b10bfp-1, 0x1.2c9fb4d812ca0p-1, 0x1.27350b8812735p-1,
  0x1.21fb78121fb78p-1, 0x1.1cf06ada2811dp-1, 0x1.1811811811812p-1, 0x1.135c81135c811p-1,
  0x1.0ecf56be69c90p-1, 0x1.0a6810a6810a7p-1, 0x1.0624dd2f1a9fcp-1, 0x1.0204081020408p-1};
static const double kLog2C[32] = {
  0x1.6e79685c2d22ap-6, 0x1.0eb389fa29f9bp-4, 0x1.bc84240adabbap-4, 0x1.32ae9e278ae1ap-3,
  0x1.84c2bd02f03b3p-3, 0x1.d49ee4c325970p-3, 0x1.11307dad30b76p-2, 0x1.37124cea4cdedp-2,
  0x1.5c01a39fbd688p-2, 0x1.800a563161c54p-2, 0x1.a33760a7f6051p-2, 0x1.c592fad295b56p-2,
  0x1.e726aa1e754d2p-2, 0x1.03fda8b97997fp-1, 0x1.140c9faa1e544p-1, 0x1.23c41d42727c8p-1,
  0x1.3327c6ab49ca7p-1, 0x1.423b07e986aa9p-1, 0x1.510118708a8f9p-1, 0x1.5f7cff41e09afp-1,
  0x1.6db196a76194ap-1, 0x1.7ba18f93502e4p-1, 0x1.894f74b06ef8bp-1, 0x1.96bdad2acb5f6p-1,
  0x1.a3ee7f38e181fp-1, 0x1.b0e4126bcc86cp-1, 0x1.bda071cc67e6ep-1, 0x1.ca258dca93316p-1,
  0x1.d6753e032ea0fp-1, 0x1.e29142e0e0140p-1, 0x1.ee7b471b3a950p-1, 0x1.fa34e1177c233p-1};
static const double kInvLn2 = 0x1.71547652b82fep+0;
static const double kLn2 = 0x1.62e42fefa39efp-1;

/* log2 of a positive finite float, in double */
static double log2_pos(float xf) {
  uint32_t b; memcpy(&b, &xf, 4);
  int e = (int)(b >> 23) - 127;
  uint32_t m = b & 0x7FFFFFu;
  if ((b >> 23) == 0) {           /* subnormal: normalise the mantissa */
    int sh = 0;
    while ((m & 0x800000u) == 0) { m <<= 1; sh++; }
    m &= 0x7FFFFFu;
    e = -126 - sh;
  }
  double md = 1.0 + (double)m * 0x1p-23;
  int j = (int)(m >> 18);
  double f = md * kInvC[j] - 1.0;
  double p = f * (1.0 + f * (-0x1.0000000000000p-1 + f * (0x1.5555555555555p-2 + f * (-0x1.0000000000000p-2 +
             f * (0x1.999999999999ap-3 + f * (-0x1.5555555555555p-3 + f * (0x1.2492492492492p-3 +
             f * (-0x1.0000000000000p-3 + f * 0x1.c71c71c71c71cp-4))))))));
  return ((double)e + kLog2C[j]) + p * kInvLn2;
}
static double exp2_d(double t) {
  if (t != t) return t;
  if (t > 130.0) return INFINITY;
  if (t < -160.0) return 0.0;
  double n = rint(t);
  double g = (t - n) * kLn2;
  double p = 1.0 + g * (1.0 + g * (0x1.0000000000000p-1 + g * (0x1.5555555555555p-3 + g * (0x1.5555555555555p-5 +
             g * (0x1.1111111111111p-7 + g * (0x1.6c16c16c16c17p-10 + g * (0x1.a01a01a01a01ap-13 +
             g * (0x1.a01a01a01a01ap-16 + g * (0x1.71de3a556c734p-19 + g * (0x1.27e4fb7789f5cp-22 +
             g * (0x1.ae64567f544e4p-26 + g * 0x1.1eed8eff8d898p-29)))))))))));
  uint64_t eb = (uint64_t)((long long)n + 1023) << 52;
  double sc; memcpy(&sc, &eb, 8);
  return p * sc;
}
float oracle_pow(float x, float y) {
  if (x != x || y != y) return NAN;
  if (x < 0.0f) return NAN;
  if (x == 0.0f) return (y > 0.0f) ? 0.0f : (y == 0.0f ? NAN : INFINITY);
  if (x == INFINITY) return (y > 0.0f) ? INFINITY : (y == 0.0f ? NAN : 0.0f);
  return (float)exp2_d((double)y * log2_pos(x));
}

/* pow(x, 5.0) of the Fresnel terms (brdf.glsl:34-41): x^5 by multiplication in
 * double (x^2 exact, x^4 and x^5 rounded), then rounded to float.  This is x^5
 * rounded to nearest-even for every x whose result is a normal float (checked
 * over all 2^32 inputs against the exact value: tools/pow5_exhaustive.hip).
 * GLSL domain as oracle_pow: x < 0 and NaN -> NaN, +-0 -> +0. */
/* variant tag of this build: 'A' + ORACLE_CONTRACT */
int oracle_contract(void) { return 'A' + ORACLE_CONTRACT; }

float oracle_pow5(float x) {
  if (!(x >= 0.0f)) return NAN;
  if (x == 0.0f) return 0.0f;
  const double d = (double)x;
  const double d2 = d * d;
  return (float)((d2 * d2) * d);
}

/* ------------------------------------------------------------------ */
/* per-invocation context                                              */
/* ------------------------------------------------------------------ */
typedef struct {
  v3 albedo, specular;
  float roughness, metalness;
  int useSpec;
} Material;     /* raytrace_types.glsl:4-10 */

typedef struct {
  int hit;
  v3 p, normal;
  float t;
  int frontFace;
  Material mat;
} HitRecord;    /* raytrace_types.glsl:109-116 */

typedef struct {
  v3 pos; float radius; Material mat;
} Sphere;       /* raytrace_types.glsl:96-100 */

typedef struct {
  v3 pos; float intensity; v3 color;
} Light;

typedef struct {
  const OrScene* s;
  const OrFrame* f;
  int x, y;             /* gl_GlobalInvocationID.xy */
  OrStats* st;
  Sphere world[5];
} Ctx;

#define M_PI_F 3.1415926535897f   /* raytrace_compute.glsl:6 */
#define INF_F INFINITY

/* raytrace_utils.glsl:28-30 */
float oracle_rand_float(float sx, float sy) {
#if CTR_UNFUSED
  float d = sx * 12.9898f + sy * 78.233f;
#else
  float d = fmaf(sy, 78.233f, sx * 12.9898f);  /* dot(seed, vec2(12.9898, 78.233)) */
#endif
  float m = oracle_sin(d) * 43758.5453f;
  return fractf(m);
}

/* raytrace_utils.glsl:44-54 randFloatSampleUniform (uses Height, not Width) */
static float randU(Ctx* c, float sx, float sy) {
  int W = c->f->width, H = c->f->height;
  int index = (c->y * H) + c->x;
  float r = oracle_rand_float(sx, sy) * (float)W * (float)H;
  int ri = f2i(r);
  index = (index + ri) % (W * H);
  c->st->rng_u++;
  return c->s->noise_u[(size_t)index * 3];
}

/* raytrace_utils.glsl:10-17 SampleSquare */
static v3 sample_square(Ctx* c, int samp) {
  int W = c->f->width, H = c->f->height;
  int index = (c->y * H) + c->x;
  index = (index + samp) % (W * H);
  c->st->rng_sq++;
  const float* n = c->s->noise + (size_t)index * 3;
  return V(n[0] - 0.5f, n[1] - 0.5f, 0.0f);
}

/* raytrace_utils.glsl:107-109 */
static inline float luminance(v3 c) { return dot(c, V(0.2126f, 0.7152f, 0.0722f)); }  /* raytrace_utils.glsl:107-109 */
/* raytrace_utils.glsl:111-113: mix(x, y, a) = x*(1-a) + y*a */
static inline v3 specularF0(v3 base, float metal) {
  float om = 1.0f - metal;
  return V(0.04f * om + base.x * metal, 0.04f * om + base.y * metal, 0.04f * om + base.z * metal);
}
/* raytrace_utils.glsl:123-129 */
static v3 perpendicular(v3 u) {
  v3 a = V(fabsf(u.x), fabsf(u.y), fabsf(u.z));
  unsigned xm = ((a.x - a.y) < 0 && (a.x - a.z) < 0) ? 1u : 0u;
  unsigned ym = (a.y - a.z) < 0 ? (1u ^ xm) : 0u;
  unsigned zm = 1u ^ (xm | ym);
  return cross(u, V((float)xm, (float)ym, (float)zm));
}
/* raytrace_utils.glsl:131-137 */
static inline float shadowedF90(v3 F0) {
  const float t = (1.0f / 0.04f);
  return fmn(1.0f, t * luminance(F0));
}
/* brdf.glsl:39-41 */
static inline v3 fresnelSchlickNew(v3 f0, float f90, float NdotS) {
  float p = oracle_pow5(1.0f - NdotS);
  return add(f0, muls(V(f90 - f0.x, f90 - f0.y, f90 - f0.z), p));
}
/* brdf.glsl:34-36 */
static inline v3 schlickFresnel(v3 f0, float u) {
  float p = oracle_pow5(fmx(0.001f, 1.0f - u));
  return add(f0, muls(sub(V(1.0f, 1.0f, 1.0f), f0), p));
}
/* raytrace_utils.glsl:177-184 */
static inline float linearToSrgb(float c) {
  if (c < 0.0031308f) return c * 12.92f;
  return 1.055f * oracle_pow(c, 1.0f / 2.4f) - 0.055f;
}

/* ------------------------------------------------------------------ */
/* intersection: ray_intersects.glsl                                   */
/* ------------------------------------------------------------------ */
/* ray_intersects.glsl:49-58 */
static float intersects_box(v3 o, v3 d, v3 mn, v3 mx) {
  v3 inv = V(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
  v3 t0 = mul(sub(mn, o), inv);
  v3 t1 = mul(sub(mx, o), inv);
  v3 tmin = V(fmn(t0.x, t1.x), fmn(t0.y, t1.y), fmn(t0.z, t1.z));
  v3 tmax = V(fmx(t0.x, t1.x), fmx(t0.y, t1.y), fmx(t0.z, t1.z));
  float tn = fmx(fmx(tmin.x, tmin.y), tmin.z);
  float tf = fmn(fmn(tmax.x, tmax.y), tmax.z);
  return tn <= tf ? ((tn >= 0.0f) ? tn : tf) : INF_F;
}

/* ray_intersects.glsl:61-96 */
static int intersects_triangle(v3 o, v3 d, v3 v0, v3 v1, v3 v2, float* dist, v3* tri_norm) {
  v3 e1 = sub(v1, v0);
  v3 e2 = sub(v2, v0);
  v3 h = cross(d, e2);
  float a = dot(e1, h);
  if (a > -0.0001f && a < 0.0001f) return 0;
  float f = 1.0f / a;
  v3 s = sub(o, v0);
  float u = f * dot(s, h);
  if (u < 0.0f || u > 1.0f) return 0;
  v3 q = cross(s, e1);
  float v = f * dot(d, q);
  if (v < 0.0f || u + v > 1.0f) return 0;
  float t = f * dot(e2, q);
  if (t > 0.00001f && t < *dist) {
    *tri_norm = normalize3(cross(e1, e2));
    *dist = t;
    return 1;
  }
  return 0;
}

static inline OrNode node_at(const OrScene* s, uint32_t i) {
  if (i < s->n_nodes) return s->nodes[i];
  OrNode z; memset(&z, 0, sizeof z); return z;   /* OOB SSBO read -> zeros */
}
static inline v3 vert_at(const OrScene* s, uint32_t i) {
  if (i < s->n_verts) return vload(s->verts[i].pos);
  return V(0, 0, 0);
}

/* ray_intersects.glsl:99-133 (stack[64], push first_child then first_child+1) */
static uint32_t intersects(const OrScene* s, uint32_t start, v3 o, v3 d, float* dist, v3* tri_norm,
                           OrStats* st) {
  uint32_t stack[64];
  int sp = 0;
  stack[sp++] = start;
  uint32_t out = 0xFFFFFFFFu;
  while (sp > 0) {
    uint32_t ni = stack[--sp];
    OrNode n = node_at(s, ni);
    st->nodes++;
    float b = intersects_box(o, d, vload(n.mn), vload(n.mx));
    if (b < *dist && !isinf(b)) {
      if (n.count > 0) {
        for (uint32_t i = 0; i < n.count; ++i) {
          uint32_t ti = n.first + i;
          OrTri tri;
          if (ti < s->n_tris) tri = s->tris[ti]; else memset(&tri, 0, sizeof tri);
          st->tris++;
          if (intersects_triangle(o, d, vert_at(s, tri.v[0]), vert_at(s, tri.v[1]), vert_at(s, tri.v[2]),
                                  dist, tri_norm))
            out = ti;
        }
      } else {
        if (sp + 2 > 64) { st->stack_overflow++; return out; }
        stack[sp++] = n.first;
        stack[sp++] = n.first + 1;
        if ((uint64_t)sp > st->max_stack) st->max_stack = (uint64_t)sp;
      }
    }
  }
  return out;
}

/* One 8-bit texel channel as GL reads it: c/255; GL_RED has no g/b, and the
 * reference uploads a 2-channel file as GL_RGB (read here as (r, g, 0)). */
static float texel_channel(const uint8_t* px, uint32_t ch, uint32_t k) {
  if (k >= ch || (ch == 2 && k == 2)) return 0.0f;
  return (float)px[k] / 255.0f;
}

/* texture(sampler2D, st).xyz for the reference's sampler state
 * (gpu_texture.h:52-58: GL_REPEAT, GL_LINEAR magnification; a compute shader
 * samples level 0).  Contract: non-finite coordinates
 * read as 0; wrap by st - floor(st); bilinear over texel centres
 * (i + 0.5)/size with weights (1-a)(1-b), a(1-b), (1-a)b, ab summed in that
 * order. */
static v3 texture_bilinear(const OrScene* s, uint32_t h, float sc, float tc) {
  const uint32_t* in = s->tex_info + 4 * (size_t)h;
  const int w = (int)in[1], hh = (int)in[2];
  const uint32_t ch = in[3];
  if (!isfinite(sc)) sc = 0.0f;
  if (!isfinite(tc)) tc = 0.0f;
  sc -= floorf(sc);
  tc -= floorf(tc);
  float x = sc * (float)w - 0.5f, y = tc * (float)hh - 0.5f;
  float xf = floorf(x), yf = floorf(y);
  float a = x - xf, b = y - yf;
  int xi[2] = {(int)xf, (int)xf + 1}, yi[2] = {(int)yf, (int)yf + 1};
  if (xi[0] < 0) xi[0] = w - 1;
  if (yi[0] < 0) yi[0] = hh - 1;
  if (xi[1] >= w) xi[1] = 0;
  if (yi[1] >= hh) yi[1] = 0;
  const float wt[4] = {(1.0f - a) * (1.0f - b), a * (1.0f - b), (1.0f - a) * b, a * b};
  float out[3];
  for (uint32_t k = 0; k < 3; k++) {
    float acc = 0.0f;
    for (int q = 0; q < 4; q++) {
      const uint8_t* px = s->tex_texels + in[0] + ((size_t)yi[q >> 1] * (size_t)w + (size_t)xi[q & 1]) * ch;
      const float term = wt[q] * texel_channel(px, ch, k);
      acc = q == 0 ? term : acc + term;
    }
    out[k] = acc;
  }
  return V(out[0], out[1], out[2]);
}

static OrVertex vertex_at(const OrScene* s, uint32_t i) {
  if (i < s->n_verts) return s->verts[i];
  OrVertex z; memset(&z, 0, sizeof z); return z;
}

/* raytrace_utils.glsl:140-175 TriangleToSupportedMat; model_p is the hit in
 * the hit BVH's frame (raytrace_compute.glsl:155) */
static Material tri_material(const OrScene* s, uint32_t tri_idx, v3 model_p, OrStats* st) {
  Material m;
  OrTri tri;
  if (tri_idx < s->n_tris) tri = s->tris[tri_idx]; else memset(&tri, 0, sizeof tri);
  OrMaterial in;
  if (tri.mat < s->n_mats) in = s->mats[tri.mat]; else memset(&in, 0, sizeof in);
  st->mat_reads++;
  if (in.use_texture == 0) {
    m.albedo = vload(in.diffuse);
  } else if (s->tex_albedo) {  /* every uv is (0,0) (types.h:105): the constant texture() result */
    m.albedo = vload(s->tex_albedo + (size_t)tri.mat * 3);
  } else {  /* :145-166 */
    OrVertex t0 = vertex_at(s, tri.v[0]), t1 = vertex_at(s, tri.v[1]), t2 = vertex_at(s, tri.v[2]);
    v3 v0v1 = sub(vload(t1.pos), vload(t0.pos));
    v3 v0v2 = sub(vload(t2.pos), vload(t0.pos));
    v3 v0p = sub(model_p, vload(t0.pos));
    float d00 = dot(v0v1, v0v1), d01 = dot(v0v1, v0v2), d11 = dot(v0v2, v0v2);
    float d20 = dot(v0p, v0v1), d21 = dot(v0p, v0v2);
    float denom = 1.0f / (d00 * d11 - d01 * d01);
    float v = (d11 * d20 - d01 * d21) * denom;
    float w = (d00 * d21 - d01 * d20) * denom;
    float u = 1.0f - v - w;
    float sc = u * t0.uv[0] + v * t1.uv[0] + w * t2.uv[0];
    float tc = u * t0.uv[1] + v * t1.uv[1] + w * t2.uv[1];
    uint64_t h = (uint64_t)in.handle[0] | ((uint64_t)in.handle[1] << 32);
    m.albedo = h < s->n_tex ? texture_bilinear(s, (uint32_t)h, sc, tc) : V(0, 0, 0);
  }
  m.specular = vload(in.Ks);
  m.roughness = 1.0f / (in.Ns + 0.0000001f);
  m.metalness = 0.1f;
  m.useSpec = 1;
  return m;
}

static OrBVH bvh_at(const OrScene* s, uint32_t i) {
  if (i < s->n_bvhs) return s->bvhs[i];
  OrBVH z; memset(&z, 0, sizeof z); return z;
}

/* mat4 * vec4, column-major: r[row] = sum_c m[c][row] * v[c] (left to right) */
static v3 xform(const float* m, v3 v, float w) {
  return V(((m[0] * v.x + m[4] * v.y) + m[8] * v.z) + m[12] * w,
           ((m[1] * v.x + m[5] * v.y) + m[9] * v.z) + m[13] * w,
           ((m[2] * v.x + m[6] * v.y) + m[10] * v.z) + m[14] * w);
}

/* raytrace_compute.glsl:93-120 SphereHit (pow(length(x), 2.0) folded to x*x) */
static int sphere_hit(v3 ro, v3 rd, const Sphere* sp, float mn, float mx, HitRecord* rec) {
  v3 oc = sub(sp->pos, ro);
  float ld = length3(rd);
  float a = ld * ld;
  float h = dot(rd, oc);
  float loc = length3(oc);
  float c = loc * loc - (sp->radius * sp->radius);
  float disc = h * h - a * c;
  if (disc < 0.0f) return 0;
  float sq = sqrtf(disc);
  float root = (h - sq) / a;
  if (!(mn < root && root < mx)) {
    root = (h + sq) / a;
    if (!(mn < root && root < mx)) return 0;
  }
  rec->t = root;
  rec->p = add(ro, muls(rd, rec->t));
  rec->mat = sp->mat;
  v3 outward = divs(sub(rec->p, sp->pos), sp->radius);
  /* raytrace_utils.glsl:23-26 SetFaceNormal */
  rec->frontFace = dot(rd, outward) < 0.0f;
  rec->normal = rec->frontFace ? outward : neg(outward);
  return 1;
}

/* raytrace_compute.glsl:122-165 CheckHit */
static HitRecord check_hit(Ctx* c, v3 ro, v3 rd, float mn, float mx) {
  HitRecord rec;
  memset(&rec, 0, sizeof rec);
  rec.hit = 0;
  rec.frontFace = 1;
  c->st->rays++;
  float dist = mx;
  if (!c->f->show_model) {
    for (int i = 0; i < 5; i++) {
      if (sphere_hit(ro, rd, &c->world[i], mn, dist, &rec)) {
        rec.hit = 1;
        dist = rec.t;
      }
    }
  }
  if (c->f->show_model) {
    for (uint32_t i = 0; i < c->f->bvh_count; i++) {
      OrBVH b = bvh_at(c->s, i);
      v3 to = xform(b.frame, ro, 1.0f);
      v3 td = xform(b.frame, rd, 0.0f);
      v3 tri_norm = V(0, 0, 0);
      uint32_t hit = intersects(c->s, b.first_index, to, td, &dist, &tri_norm, c->st);
      if (hit != 0xFFFFFFFFu) {
        rec.hit = 1;
        rec.p = add(smul(dist, rd), ro);
        rec.normal = tri_norm;
        rec.t = dist;
        v3 model_p = add(smul(dist, td), to);
        rec.mat = tri_material(c->s, hit, model_p, c->st);
      }
    }
  }
  return rec;
}

/* raytrace_compute.glsl:167-176 (full closest-hit query) */
static int light_occluded(Ctx* c, v3 pos, const Light* L) {
  v3 dir = normalize3(sub(L->pos, pos));
  float mx = length3(sub(L->pos, pos));
  c->st->shadow_rays++;
  HitRecord r = check_hit(c, pos, dir, 0.001f, mx);
  return r.hit;
}

/* brdf.glsl:147-152 */
static inline float light_falloff(v3 p, const Light* L) {
  v3 d = sub(L->pos, p);
  float d2 = dot(d, d);
  return 1.0f / ((0.01f * 0.01f) + d2);
}
/* brdf.glsl:2-5 */
static inline v3 light_dir(const Light* L, v3 p) {
  v3 ld = sub(L->pos, p);
  return length3(ld) > 0.0f ? normalize3(ld) : ld;
}

static Light light_at(Ctx* c, int i) {
  Light L;
  c->st->light_reads++;
  if (i >= 0 && (uint32_t)i < c->s->n_lights) {
    const OrLight* l = &c->s->lights[i];
    L.pos = vload(l->pos); L.intensity = l->intensity; L.color = vload(l->color);
  } else {
    L.pos = V(0, 0, 0); L.intensity = 0.0f; L.color = V(0, 0, 0);   /* OOB -> zeros */
  }
  return L;
}

/* raytrace_compute.glsl:179-206 SampleLights (literal loop) */
static int sample_lights(Ctx* c, const HitRecord* hit, float* weight, Light* sel) {
  float total = 0.0f, pdf = 0.0f;
  int selected = 0;
  int n = c->f->light_count;
  for (int i = 0; i < n; i++) {
    int idx = f2i(rintf(randU(c, hit->p.x, hit->p.y) * (float)n));
    float lw = (float)n;
    Light L = light_at(c, idx);
    float fo = light_falloff(hit->p, &L);
    float inten = L.intensity * fo;
    float lpdf = luminance(V(inten, inten, inten));
    float ris = lpdf * lw;
    total += ris;
    float r = randU(c, hit->p.y + (float)i, hit->p.z + (float)i);
    if (r < (ris / total)) {
      *sel = L;
      pdf = lpdf;
      selected = 1;
    }
  }
  *weight = (total / (float)n) / fmx(0.001f, pdf);
  return selected;
}

/* brdf.glsl:8-12 */
static inline float ggxD(float NdotH, float rough) {
  float a2 = rough * rough;
  float d = ((NdotH * a2 - NdotH) * NdotH + 1.0f);
  return a2 / fmx(0.001f, (d * d * M_PI_F));
}
/* brdf.glsl:15-18 */
static inline float ggxDNew(float NdotH, float alphaSquared) {
  float b = ((alphaSquared - 1.0f) * NdotH * NdotH + 1.0f);
  return alphaSquared / fmx(0.001f, (M_PI_F * b * b));
}
/* brdf.glsl:21-31 */
static inline float ggxSchlickMasking(float NdotL, float NdotV, float rough) {
  float k = rough * rough / 2.0f;
  float gv = NdotV / fmx(0.001f, (NdotV * (1.0f - k) + k));
  float gl = NdotL / fmx(0.001f, (NdotL * (1.0f - k) + k));
  return fabsf(gv * gl);
}
/* brdf.glsl:44-57 */
static inline float smithGAlpha(float alpha, float NdotS) {
  return NdotS / (fmx(0.0001f, alpha) * sqrtf(1.0f - fmn(0.99999f, NdotS * NdotS)));
}
static inline float smithLambda(float a) {
  return (-1.0f + sqrtf(1.0f + (1.0f / fmx(0.001f, a * a)))) * 0.5f;
}
static inline float smithG2(float alpha, float NdotL, float NdotV) {
  float aL = smithGAlpha(alpha, NdotL);
  float aV = smithGAlpha(alpha, NdotV);
  return 1.0f / (1.0f + smithLambda(aL) + smithLambda(aV));
}

/* brdf.glsl:200-224 SampleDirect (old GGX; used when useSpec) */
static v3 sample_direct(const HitRecord* hit, v3 Vv, const Light* L, float shadow) {
  v3 Ld = light_dir(L, hit->p);
  v3 vl = add(Vv, Ld);
  v3 H = length3(vl) > 0.0f ? normalize3(vl) : vl;
  v3 N = hit->normal;
  float NdotL = sat(dot(N, Ld));
  float NdotH = sat(dot(N, H));
  float LdotH = sat(dot(Ld, H));
  float NdotV = sat(dot(N, Vv));
  float rough = hit->mat.roughness;
  float D = ggxD(NdotH, rough);
  float G = ggxSchlickMasking(NdotL, NdotV, rough);
  v3 F = schlickFresnel(hit->mat.specular, LdotH);
  float fo = light_falloff(hit->p, L);
  float li = L->intensity * fo;
  v3 ggx = divs(muls(F, D * G), (4.0f * fmx(0.001f, NdotV)));
  v3 lt = muls(smul(shadow, L->color), li);
  v3 diff = divs(smul(NdotL, hit->mat.albedo), M_PI_F);
  return mul(lt, add(ggx, diff));
}

typedef struct { v3 specF0, diffRefl, F; float alpha, alphaSq, NdotL, NdotV, NdotH; } Brdf;

/* brdf.glsl:173-198 GetAllBRDFValues(N, L, V, hit) */
static Brdf brdf_values(v3 N, v3 L, v3 Vv, const HitRecord* hit) {
  Brdf b;
  v3 H = normalize3(add(L, Vv));
  b.NdotL = sat(dot(N, L));
  b.NdotV = sat(dot(N, Vv));
  float LdotH = sat(dot(L, H));
  b.NdotH = sat(dot(N, H));
  b.specF0 = specularF0(hit->mat.albedo, hit->mat.metalness);
  b.diffRefl = muls(hit->mat.albedo, (1.0f - hit->mat.metalness));
  b.alpha = hit->mat.roughness * hit->mat.roughness;
  b.alphaSq = b.alpha * b.alpha;
  b.F = fresnelSchlickNew(b.specF0, shadowedF90(b.specF0), LdotH);
  return b;
}

/* brdf.glsl:226-237 SampleDirectNew + EvalSpecular :139-145 + EvalDiffuse :134-137 */
static v3 sample_direct_new(const HitRecord* hit, v3 Vv, v3 L) {
  Brdf d = brdf_values(hit->normal, L, Vv, hit);
  /* EvalSpecular: ggxNormalDistributionNew(max(1e-5, alphaSq), NdotH) -- arguments swapped */
  float D = ggxDNew(fmx(0.00001f, d.alphaSq), d.NdotH);
  float G = smithG2(d.alpha, d.NdotL, d.NdotV);
  float denom = 4.0f * fmx(d.NdotL, 0.001f) * fmx(d.NdotV, 0.001f);
  v3 spec = muls(divs(muls(muls(d.F, G), D), fmx(denom, 0.001f)), d.NdotL);
  const float oneOverPi = 1.0f / M_PI_F;
  v3 diff = muls(d.diffRefl, (oneOverPi * d.NdotL));
  return add(mul(sub(V(1.0f, 1.0f, 1.0f), d.F), diff), spec);
}

/* brdf.glsl:279-288 */
static float brdf_probability(const Material* m, v3 Vv, v3 N) {
  float specF0 = luminance(specularF0(m->albedo, m->metalness));
  float diffRefl = luminance(muls(m->albedo, (1.0f - m->metalness)));
  v3 f0 = V(specF0, specF0, specF0);
  float F = sat(luminance(fresnelSchlickNew(f0, shadowedF90(f0), fmx(0.0f, dot(Vv, N)))));
  float specular = F;
  float diffuse = diffRefl * (1.0f - F);
  float p = (specular / fmx(0.0001f, (specular + diffuse)));
  return clampf(p, 0.1f, 0.9f);
}

/* brdf.glsl:60-74 */
static v3 sample_diffuse(Ctx* c, v3 point, v3 N) {
  float r1 = randU(c, point.x, point.y);
  float r2 = randU(c, point.y, point.z);
  v3 B = perpendicular(N);
  v3 T = cross(B, N);
  float r = sqrtf(fabsf(r1));
  float phi = 2.0f * M_PI_F * r2;
  return add(add(muls(T, (r * oracle_cos(phi))), muls(B, (r * oracle_sin(phi)))), muls(N, sqrtf(fabsf(1.0f - r1))));
}

/* brdf.glsl:81-99 */
static v3 sample_specular_half(Ctx* c, v3 point, float rough, v3 N) {
  float rx = randU(c, point.x, point.y);
  float ry = randU(c, point.y, point.z);
  v3 B = perpendicular(N);
  v3 T = cross(B, N);
  float a2 = rough * rough;
  float cosT = sqrtf(fmx(0.0f, (1.0f - rx) / ((a2 - 1.0f) * rx + 1.0f)));
  float sinT = sqrtf(fmx(0.0f, 1.0f - cosT * cosT));
  float phi = ry * M_PI_F * 2.0f;
  return add(add(muls(T, (sinT * oracle_cos(phi))), muls(B, (sinT * oracle_sin(phi)))), muls(N, cosT));
}

static inline v3 reflect3(v3 I, v3 N) { return sub(I, muls(N, 2.0f * dot(N, I))); }

/* brdf.glsl:76-78 */
static inline float specular_sample_weight(float alpha, float alphaSq, float NdotS, float NdotS2) {
  (void)alpha;
  return 2.0f / (sqrtf(((alphaSq * (1.0f - NdotS2)) + NdotS2) / NdotS2) + 1.0f);
}

/* brdf.glsl:102-132 */
static v3 sample_specular_microfacet(Ctx* c, const HitRecord* hit, v3 Vv, float alpha, float alphaSq,
                                     v3 specF0, v3* weight) {
  v3 H;
  if (alpha == 0.0f) {
    v3 Lt = reflect3(neg(Vv), hit->normal);
    H = normalize3(add(neg(Vv), Lt));
  } else {
    H = sample_specular_half(c, hit->p, hit->mat.roughness, hit->normal);
  }
  v3 L = reflect3(neg(Vv), H);
  v3 N = hit->normal;
  float HdotL = fmx(0.00001f, fmn(1.0f, dot(H, L)));
  float NdotL = fmx(0.00001f, fmn(1.0f, dot(N, L)));
  v3 F = fresnelSchlickNew(specF0, shadowedF90(specF0), HdotL);
  *weight = muls(F, specular_sample_weight(alpha, alphaSq, NdotL, NdotL * NdotL));
  return L;
}

#define DIFFUSE_BRDF 1
#define SPECULAR_BRDF 2

/* brdf.glsl:239-277 SampleIndirectNew */
static int sample_indirect(Ctx* c, const HitRecord* hit, v3 N, v3 Vv, const Material* m, int type,
                           v3* dir, v3* weight) {
  if (dot(N, Vv) <= 0.0f) return 0;
  v3 nd;
  if (type == DIFFUSE_BRDF) {
    nd = sample_diffuse(c, hit->p, N);
    Brdf d = brdf_values(N, nd, Vv, hit);
    *weight = d.diffRefl;
    v3 H = sample_specular_half(c, hit->p, m->roughness, N);
    float VdotH = fmx(0.00001f, fmn(1.0f, dot(Vv, H)));
    *weight = mul(*weight, sub(V(1.0f, 1.0f, 1.0f), fresnelSchlickNew(d.specF0, shadowedF90(d.specF0), VdotH)));
  } else {
    Brdf d = brdf_values(N, V(0.0f, 0.0f, 1.0f), Vv, hit);
    nd = sample_specular_microfacet(c, hit, Vv, d.alpha, d.alphaSq, d.specF0, weight);
  }
  if (luminance(*weight) == 0.0f) return 0;
  *dir = normalize3(nd);
  if (dot(N, *dir) <= 0.0f) return 0;
  return 1;
}

/* raytrace_compute.glsl:208-294 GetRayColor */
static v3 get_ray_color(Ctx* c, v3 ro, v3 rd, int maxDepth) {
  int randIndex = 0;
  int depth = maxDepth;
  v3 sky = V(0.05f, 0.05f, 0.05f);
  v3 T = V(1.0f, 1.0f, 1.0f);
  v3 color = V(0.0f, 0.0f, 0.0f);
  for (;;) {
    HitRecord rec = check_hit(c, ro, rd, 0.001f, INF_F);
    if (!rec.hit) break;
    float lw;
    Light L;
    memset(&L, 0, sizeof L);
    int sampled = sample_lights(c, &rec, &lw, &L);
    v3 Vv = neg(rd);
    if (sampled) {
      float shadow = light_occluded(c, rec.p, &L) ? 0.0f : 1.0f;
      v3 Ld = light_dir(&L, rec.p);
      if (rec.mat.useSpec) {
        color = add(color, muls(mul(T, sample_direct(&rec, neg(rd), &L, shadow)), lw));
      } else {
        float fo = light_falloff(rec.p, &L);
        v3 li = muls(muls(muls(L.color, fo), L.intensity), lw);
        color = add(color, mul(muls(mul(T, sample_direct_new(&rec, neg(rd), Ld)), shadow), li));
      }
    }
    int type;
    if (rec.mat.metalness == 1.0f && rec.mat.roughness == 0.0f) {
      type = SPECULAR_BRDF;
    } else {
      float bp = brdf_probability(&rec.mat, Vv, rec.normal);
      float r = randU(c, rec.p.x + (float)depth, rec.p.y + (float)depth);
      if (r < bp) { type = SPECULAR_BRDF; T = divs(T, bp); }
      else { type = DIFFUSE_BRDF; T = divs(T, (1.0f - bp)); }
    }
    if (depth <= 0) {
      float surv = clampf(luminance(T), 0.1f, 1.0f);
      if (randU(c, rec.p.x + (float)randIndex, rec.p.y + (float)randIndex) > surv) break;
      T = divs(T, surv);
      randIndex++;
    } else {
      depth--;
    }
    v3 dir, bw;
    if (!sample_indirect(c, &rec, rec.normal, Vv, &rec.mat, type, &dir, &bw)) break;
    T = mul(T, bw);
    rd = dir;
    ro = rec.p;
  }
  color = add(color, mul(T, sky));
  return color;
}

/* raytrace_compute.glsl:299-364 the five hard-coded spheres */
static void build_world(Sphere* w) {
  Material m1 = {V(0.2f, 0.8f, 0.8f), V(0.2f, 0.4f, 0.4f), 0.01f, 0.99f, 0};
  Material m2 = {V(0.8f, 0.3f, 0.3f), V(0.9f, 0.7f, 0.7f), 0.1f, 0.5f, 1};
  Material m3 = {V(0.2f, 0.9f, 0.3f), V(0.2f, 0.9f, 0.9f), 0.3f, 0.95f, 1};
  Material m4 = {V(0.2f, 0.4f, 1.0f), V(0.8f, 0.8f, 0.9f), 0.01f, 0.9f, 0};
  Material m5 = {V(0.9f, 0.8f, 0.1f), V(0.3f, 0.3f, 0.1f), 0.7f, 0.3f, 0};
  w[1].pos = V(0.0f, -100.5f, -1.0f); w[1].radius = 100.0f; w[1].mat = m1;
  w[0].pos = V(1.8f, 0.0f, -2.0f);    w[0].radius = 0.5f;   w[0].mat = m4;
  w[2].pos = V(0.55f, 0.0f, -2.0f);   w[2].radius = 0.5f;   w[2].mat = m3;
  w[3].pos = V(-0.55f, 0.0f, -2.0f);  w[3].radius = 0.5f;   w[3].mat = m2;
  w[4].pos = V(-1.8f, 0.0f, -2.0f);   w[4].radius = 0.5f;   w[4].mat = m5;
}

typedef struct { v3 center, p00, du, dv; } Cam;

/* raytrace_compute.glsl:47-76 GetCamera (focusDist = 1, :384) */
static Cam get_camera(const OrFrame* f) {
  Cam c;
  float aspect = (float)f->width / (float)f->height;
  int height = f2i((float)f->width / aspect);
  height = (height < 1) ? 1 : height;
  const float focus = 1.0f;
  c.center = vload(f->cam_origin);
  v3 w = neg(vload(f->cam_dir));
  v3 u = vload(f->cam_right);
  v3 v = vload(f->cam_up);
  v3 viewU = muls(u, focus);
  v3 viewV = muls(v, focus);
  c.du = divs(viewU, (float)f->width);
  c.dv = divs(viewV, (float)height);
  v3 ll = sub(sub(sub(c.center, smul(focus, w)), divs(viewU, 2.0f)), divs(viewV, 2.0f));
  c.p00 = add(ll, smul(0.5f, add(c.du, c.dv)));
  return c;
}

static inline uint8_t to_unorm8(float x) {
  if (x != x) return 0;
  float c = clampf(x, 0.0f, 1.0f);
  return (uint8_t)rintf(c * 255.0f);
}

/* raytrace_compute.glsl:296-414 main() for one invocation */
static void invocation(const OrScene* s, const OrFrame* f, const Cam* cam, int x, int y, float* accum,
                       uint8_t* out, OrStats* st) {
  size_t px = (size_t)y * (size_t)f->width + (size_t)x;
  if (f->reset) {
    accum[px * 4 + 0] = 0.0f; accum[px * 4 + 1] = 0.0f; accum[px * 4 + 2] = 0.0f; accum[px * 4 + 3] = 1.0f;
    return;
  }
  Ctx c;
  c.s = s; c.f = f; c.x = x; c.y = y; c.st = st;
  build_world(c.world);
  int samp = f->accum_frames % (f->width * f->height);
  v3 off = sample_square(&c, samp);
  v3 ps = add(add(cam->p00, muls(cam->du, ((float)x + off.x))), muls(cam->dv, ((float)y + off.y)));
  v3 rd = sub(ps, cam->center);
  st->samples++;
  v3 col = get_ray_color(&c, cam->center, rd, f->max_depth);
  v3 prev = vload(accum + px * 4);
  v3 acc = add(prev, col);
  accum[px * 4 + 0] = acc.x; accum[px * 4 + 1] = acc.y; accum[px * 4 + 2] = acc.z; accum[px * 4 + 3] = 1.0f;
  v3 o = divs(acc, (float)f->accum_frames);
  out[px * 4 + 0] = to_unorm8(linearToSrgb(o.x));
  out[px * 4 + 1] = to_unorm8(linearToSrgb(o.y));
  out[px * 4 + 2] = to_unorm8(linearToSrgb(o.z));
  out[px * 4 + 3] = 255;
}

void oracle_dispatch(const OrScene* s, const OrFrame* f, float* accum, uint8_t* out, int y0, int y1,
                     OrStats* st) {
  Cam cam = get_camera(f);
  for (int y = y0; y < y1; ++y)
    for (int x = 0; x < f->width; ++x) invocation(s, f, &cam, x, y, accum, out, st);
}

static void stats_add(OrStats* a, const OrStats* b) {
  a->rays += b->rays; a->nodes += b->nodes; a->tris += b->tris; a->rng_u += b->rng_u;
  a->rng_sq += b->rng_sq; a->light_reads += b->light_reads; a->mat_reads += b->mat_reads;
  a->samples += b->samples; a->stack_overflow += b->stack_overflow; a->shadow_rays += b->shadow_rays;
  if (b->max_stack > a->max_stack) a->max_stack = b->max_stack;
}

void oracle_render(const OrScene* s, const OrFrame* f, int frame_first, int nframes, float* accum,
                   uint8_t* out, int y0, int y1, int threads, OrStats* st) {
  OrStats total; memset(&total, 0, sizeof total);
#ifdef _OPENMP
  if (threads <= 0) threads = omp_get_max_threads();
  #pragma omp parallel num_threads(threads)
  {
    OrStats loc; memset(&loc, 0, sizeof loc);
    #pragma omp for schedule(dynamic, 1)
    for (int y = y0; y < y1; ++y) {
      for (int k = 0; k < nframes; ++k) {
        OrFrame fk = *f; fk.accum_frames = frame_first + k; fk.reset = 0;
        Cam cam = get_camera(&fk);
        for (int x = 0; x < f->width; ++x) invocation(s, &fk, &cam, x, y, accum, out, &loc);
      }
    }
    #pragma omp critical
    stats_add(&total, &loc);
  }
#else
  (void)threads;
  for (int y = y0; y < y1; ++y)
    for (int k = 0; k < nframes; ++k) {
      OrFrame fk = *f; fk.accum_frames = frame_first + k; fk.reset = 0;
      Cam cam = get_camera(&fk);
      for (int x = 0; x < f->width; ++x) invocation(s, &fk, &cam, x, y, accum, out, &total);
    }
#endif
  if (st) stats_add(st, &total);
}

void oracle_render_rows(const OrScene* s, const OrFrame* f, int frame_first, int nframes, float* accum,
                        uint8_t* out, const int* rows, int nrows, int threads, OrStats* st) {
  OrStats total; memset(&total, 0, sizeof total);
#ifdef _OPENMP
  if (threads <= 0) threads = omp_get_max_threads();
  #pragma omp parallel num_threads(threads)
  {
    OrStats loc; memset(&loc, 0, sizeof loc);
    /* pixels are independent and only each pixel's frames are ordered, so a row is split into
     * 64-pixel pieces that run their frames in order: a few rows at many frames use every thread */
    const int nxc = (f->width + 63) / 64;
    #pragma omp for schedule(dynamic, 1)
    for (int it = 0; it < nrows * nxc; ++it) {
      const int r = it / nxc, x0 = (it % nxc) * 64, x1 = x0 + 64 < f->width ? x0 + 64 : f->width;
      for (int k = 0; k < nframes; ++k) {
        OrFrame fk = *f; fk.accum_frames = frame_first + k; fk.reset = 0;
        Cam cam = get_camera(&fk);
        for (int x = x0; x < x1; ++x) invocation(s, &fk, &cam, x, rows[r], accum, out, &loc);
      }
    }
    #pragma omp critical
    stats_add(&total, &loc);
  }
#else
  (void)threads;
  for (int r = 0; r < nrows; ++r)
    for (int k = 0; k < nframes; ++k) {
      OrFrame fk = *f; fk.accum_frames = frame_first + k; fk.reset = 0;
      Cam cam = get_camera(&fk);
      for (int x = 0; x < f->width; ++x) invocation(s, &fk, &cam, x, rows[r], accum, out, &total);
    }
#endif
  if (st) stats_add(st, &total);
}

/* ray_intersects.glsl:135-161 (commented test kernel): per ray, hits = -1;
 * for each BVH: transform, Intersects(first_index, o', d', ray.t). */
void oracle_trace_closest(const OrScene* s, uint32_t bvh_count, const OrRay* rays, int n, uint32_t* hits,
                          float* t_out, float* n_out, OrStats* st) {
  for (int r = 0; r < n; ++r) {
    v3 o = vload(rays[r].o), d = vload(rays[r].d);
    float dist = rays[r].t;
    uint32_t hit = 0xFFFFFFFFu;
    v3 nrm = V(0, 0, 0);
    st->rays++;
    for (uint32_t i = 0; i < bvh_count; ++i) {
      OrBVH b = bvh_at(s, i);
      v3 to = xform(b.frame, o, 1.0f);
      v3 td = xform(b.frame, d, 0.0f);
      uint32_t h = intersects(s, b.first_index, to, td, &dist, &nrm, st);
      if (h != 0xFFFFFFFFu) hit = h;
    }
    hits[r] = hit;
    if (t_out) t_out[r] = dist;
    if (n_out) { n_out[r * 3] = nrm.x; n_out[r * 3 + 1] = nrm.y; n_out[r * 3 + 2] = nrm.z; }
  }
}
