// pathtrace.hip -- MI355X (gfx950) path-tracing kernels + the device context.
//
// One HIP thread traces one pixel.  A launch covers `nframes` consecutive
// frames of the reference's progressive loop (one dispatch of
// shaders/raytrace_compute.glsl per frame, src/main.cpp:657-718); the
// accumulation is carried in registers across frames (the same fp32 adds in
// the same order as per-frame image RMWs) and stored once.
//
// Device layout (re-laid from the std430 SSBOs):
//   nodes  : 32 B per node (min.xyz|first, max.xyz|count), base offset 32 B so
//            each sibling pair (2k+1, 2k+2) is one 64-B aligned block;
//   tris   : 48 B per triangle = v0, e1 = v1 - v0, e2 = v2 - v0, material id
//            (vertex gather and edge subtraction hoisted to upload time);
//   mats   : 32 B shading material (albedo|roughness, specular) precomputed
//            from MaterialFromOBJ (raytrace_utils.glsl:140-175);
//   lights : 32 B, one zero record appended (lights[lightCount] reads zero);
//   noise  : noiseTex as .xy float2 (8 B), noiseUniformTex as .x float (4 B):
//            the only channels the live kernel reads.
// Traversal stack: per-lane in LDS (3 dwords per entry), sized from the
// BVH's depth.  Shadow rays use an any-hit traversal, which returns exactly
// CheckHit(...).hit (first accepted triangle happens before any change of the
// running distance).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "pt_math.hpp"
#include "srt_internal.hpp"

using namespace srt::dev;

namespace srt {

// ---------------------------------------------------------------------------
// kernel parameters (kernarg segment -> scalar registers)
// ---------------------------------------------------------------------------
struct KParams {
  const float4* nodes;   // node i at nodes[2*i + 2], nodes[2*i + 3]
  const float4* tris;    // 3 float4 per triangle
  const float4* mats;    // 2 float4 per material
  const float4* lights;  // 2 float4 per light, light_count + 1 records
  const srt_bvh_record* bvhs;
  const float2* noise_xy;
  const float* noise_u;
  float4* accum;
  uint32_t* out;
  unsigned long long* stats;
  unsigned long long* batch_ctr;  // next unclaimed 64-item batch of the launch (zeroed before it)
  int W, H, WH;
  int light_count;   // lightCount uniform (loop count)
  int light_records; // records in the light SSBO; index >= light_records reads zeros
  uint32_t bvh_count;
  int show_model;
  int max_depth;
  int frame_first, nframes, write_output, reset;
  int rank, nranks, band_rows, local_rows;
  int ext_w, ext_h;
  int stack_entries;
  int nodes_f4, tris_f4;   // LDS-resident scene: sizes of the node / triangle arrays in float4
  float4* lbuf;            // sample buffer: nframes x local_pixels radiance samples
  int local_pixels;        // W * local_rows
  int trav_frac16;         // resume shading when fewer than trav_frac16/16 of working lanes traverse
  int stack_base_f4;       // first float4 of the per-lane stacks in dynamic LDS
  uint32_t* gstack;        // global-scene mode: per-lane stacks in HBM, entry field k of lane g at gstack[k * stride + g]
  int gstack_stride;       // lanes in the grid
  float cx, cy, cz, p00x, p00y, p00z, dux, duy, duz, dvx, dvy, dvz;
};

// Dynamic LDS of the path-tracing kernels: [scene copy (LDS mode)] [per-lane stacks].
extern __shared__ __attribute__((aligned(16))) float4 g_smem[];

enum { ST_RAYS = 0, ST_NODES, ST_TRIS, ST_RNGU, ST_RNGSQ, ST_LIGHTS, ST_MATS, ST_SAMPLES, ST_OVERFLOW, ST_MAXSTACK,
       ST_N, ST_CYC_REFILL = ST_N, ST_CYC_TRAV, ST_CYC_SHADE, ST_CYC_ITERS,
       // lane occupancy of the traversal loop (summed popcounts per iteration) and of shading
       ST_DBG_TITERS, ST_DBG_WORK, ST_DBG_TRAV, ST_DBG_LEAF, ST_DBG_INT, ST_DBG_SHADE,
       // per traversal sub-step k < 16: lanes taking it (summed), waves executing it, lanes popping after it
       ST_DBG_SUB, ST_TOTAL = ST_DBG_SUB + 48 };

// Diagnostic build only (-DSRT_SUBSTEP_STATS): per-sub-step lane counts (global atomics, slow).
#ifdef SRT_SUBSTEP_STATS
__device__ __forceinline__ void dbg_count(unsigned long long* stats, int idx, bool cond, bool waves) {
  const unsigned long long m = __ballot(cond);
  if (m && (threadIdx.x & 63) == 0) {
    atomicAdd(&stats[idx], (unsigned long long)__popcll(m));
    if (waves) atomicAdd(&stats[idx + 1], 1ull);
  }
}
#define DBG_COUNT(stats, idx, cond) dbg_count(stats, idx, cond, ((idx) - ST_DBG_SUB) % 3 == 0)
#else
#define DBG_COUNT(stats, idx, cond)
#endif

// Diagnostic build only (-DSRT_PHASE_TIMING): per-wave shader-clock stamps at the
// phase boundaries of sample_kernel, summed into stats[ST_CYC_*].
#ifdef SRT_PHASE_TIMING
#define PHASE_STAMP(var) unsigned long long var = __builtin_amdgcn_s_memtime()
#else
#define PHASE_STAMP(var)
#endif

struct Counters {
  uint32_t v[ST_N];
};

template <bool COUNT>
__device__ __forceinline__ void bump(Counters& c, int k, uint32_t n = 1) {
  if constexpr (COUNT) c.v[k] += n;
}

struct Mat {
  f3 albedo, specular;
  float roughness, metalness;
  bool useSpec;
};

struct Hit {
  bool hit;
  f3 p, normal;
  Mat mat;
};

struct LightRec {
  f3 pos;
  float intensity;
  f3 color;
};

// raytrace_compute.glsl:299-364: five hard-coded spheres and their materials
__device__ __forceinline__ void sphere_data(int i, f3& pos, float& radius, Mat& m) {
  switch (i) {
    case 0: pos = mk(1.8f, 0.0f, -2.0f); radius = 0.5f;   // blue (material4)
      m = Mat{mk(0.2f, 0.4f, 1.0f), mk(0.8f, 0.8f, 0.9f), 0.01f, 0.9f, false}; break;
    case 1: pos = mk(0.0f, -100.5f, -1.0f); radius = 100.0f;  // ground (material1)
      m = Mat{mk(0.2f, 0.8f, 0.8f), mk(0.2f, 0.4f, 0.4f), 0.01f, 0.99f, false}; break;
    case 2: pos = mk(0.55f, 0.0f, -2.0f); radius = 0.5f;  // green (material3)
      m = Mat{mk(0.2f, 0.9f, 0.3f), mk(0.2f, 0.9f, 0.9f), 0.3f, 0.95f, true}; break;
    case 3: pos = mk(-0.55f, 0.0f, -2.0f); radius = 0.5f;  // red (material2)
      m = Mat{mk(0.8f, 0.3f, 0.3f), mk(0.9f, 0.7f, 0.7f), 0.1f, 0.5f, true}; break;
    default: pos = mk(-1.8f, 0.0f, -2.0f); radius = 0.5f;  // yellow (material5)
      m = Mat{mk(0.9f, 0.8f, 0.1f), mk(0.3f, 0.3f, 0.1f), 0.7f, 0.3f, false}; break;
  }
}

// ---------------------------------------------------------------------------
// per-lane context
// ---------------------------------------------------------------------------
struct Lane {
  int base;             // (y * Height) + x  (raytrace_utils.glsl:11-12,45-46)
  uint32_t* stk;        // LDS stack: entry k field f at stk[(Fk+f) * stride] (global-scene mode: a ring of kShortStack)
  int stride;
  uint32_t* gstk;       // global-scene mode: the whole stack in HBM, same layout
  int gstride;
};

// (a % m) for 0 <= a, 0 < m, with the common case a < 2m handled by one compare
__device__ __forceinline__ int wrap_index(int a, int m) {
  if (a >= m) a -= m;
  if (a >= m) a %= m;  // only when Width < Height (index base y*Height + x can exceed W*H)
  return a;
}

// raytrace_utils.glsl:28-30
__device__ __forceinline__ float rand_float(float sx, float sy) {
  const float d = sx * 12.9898f + sy * 78.233f;
  return fractf(sin_f(d) * 43758.5453f);
}

// raytrace_utils.glsl:44-54 randFloatSampleUniform, split into the index and
// the fetch so one bounce's independent draws are all in flight together.
__device__ __forceinline__ int randU_index(const KParams& kp, const Lane& ln, float sx, float sy) {
  const float r = rand_float(sx, sy) * (float)kp.W * (float)kp.H;
  return wrap_index(ln.base + f2i(r), kp.WH);
}
template <bool COUNT>
__device__ __forceinline__ float randU(const KParams& kp, const Lane& ln, Counters& c, float sx, float sy) {
  bump<COUNT>(c, ST_RNGU);
  return kp.noise_u[randU_index(kp, ln, sx, sy)];
}

__device__ __forceinline__ float luminance(f3 c) { return c.x * 0.2126f + c.y * 0.7152f + c.z * 0.0722f; }
__device__ __forceinline__ f3 specularF0(f3 b, float m) {
  const float om = 1.0f - m;
  return mk(0.04f * om + b.x * m, 0.04f * om + b.y * m, 0.04f * om + b.z * m);
}
__device__ __forceinline__ f3 perpendicular(f3 u) {
  const f3 a = mk(__builtin_fabsf(u.x), __builtin_fabsf(u.y), __builtin_fabsf(u.z));
  const unsigned xm = ((a.x - a.y) < 0.0f && (a.x - a.z) < 0.0f) ? 1u : 0u;
  const unsigned ym = (a.y - a.z) < 0.0f ? (1u ^ xm) : 0u;
  const unsigned zm = 1u ^ (xm | ym);
  return cross(u, mk((float)xm, (float)ym, (float)zm));
}
__device__ __forceinline__ float shadowedF90(f3 F0) { return fmn(1.0f, (1.0f / 0.04f) * luminance(F0)); }
__device__ __forceinline__ f3 fresnelSchlickNew(f3 f0, float f90, float NdotS) {
  const float p = pow5_f(1.0f - NdotS);
  return f0 + mk(f90 - f0.x, f90 - f0.y, f90 - f0.z) * p;
}
__device__ __forceinline__ f3 schlickFresnel(f3 f0, float u) {
  const float p = pow5_f(fmx(0.001f, 1.0f - u));
  return f0 + (mk(1.0f, 1.0f, 1.0f) - f0) * p;
}
__device__ __forceinline__ float linearToSrgb(float c) {
  if (c < 0.0031308f) return c * 12.92f;
  return 1.055f * pow_f(c, 1.0f / 2.4f) - 0.055f;
}
__device__ __forceinline__ uint32_t to_unorm8(float x) {
  if (x != x) return 0u;
  return (uint32_t)__builtin_rintf(clampf(x, 0.0f, 1.0f) * 255.0f);
}

// ---------------------------------------------------------------------------
// BVH traversal (ray_intersects.glsl:49-133), order-exact
// ---------------------------------------------------------------------------
// IntersectsBox.  Hardware v_min/v_max (IEEE minNum/maxNum) give the same
// value as GLSL min/max up to the sign of a zero result, and the result is
// only ever compared (< dist, isinf), so every decision is unchanged.
__device__ __forceinline__ float box_t(f3 o, f3 inv, float4 lo, float4 hi) {
  const float t0x = (lo.x - o.x) * inv.x, t0y = (lo.y - o.y) * inv.y, t0z = (lo.z - o.z) * inv.z;
  const float t1x = (hi.x - o.x) * inv.x, t1y = (hi.y - o.y) * inv.y, t1z = (hi.z - o.z) * inv.z;
  const float tn = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(t0x, t1x), __builtin_fminf(t0y, t1y)),
                                   __builtin_fminf(t0z, t1z));
  const float tf = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(t0x, t1x), __builtin_fmaxf(t0y, t1y)),
                                   __builtin_fmaxf(t0z, t1z));
  return tn <= tf ? ((tn >= 0.0f) ? tn : tf) : __builtin_inff();
}

__device__ __forceinline__ bool box_ok(float b, float dist) { return b < dist && !isinf_f(b); }

// LDS byte offsets are 32-bit: keep the address arithmetic in 32 bits.
__device__ __forceinline__ float4 lds4(uint32_t byte_off) {
  return *reinterpret_cast<const float4*>(reinterpret_cast<const char*>(g_smem) + byte_off);
}
template <bool LDSM>
__device__ __forceinline__ float4 node4(const KParams& kp, uint32_t i) {
  if constexpr (LDSM) return lds4(i << 4);
  else return kp.nodes[i];
}
// the records of triangle `i` onwards (3 float4 per triangle)
template <bool LDSM>
__device__ __forceinline__ const float4* tri_ptr(const KParams& kp, uint32_t i) {
  if constexpr (LDSM)
    return reinterpret_cast<const float4*>(reinterpret_cast<const char*>(g_smem) + (((uint32_t)kp.nodes_f4 + 3 * i) << 4));
  else return kp.tris + 3 * (size_t)i;
}
template <bool LDSM>
__device__ __forceinline__ float4 tri4(const KParams& kp, uint32_t i) {
  if constexpr (LDSM) return lds4(((uint32_t)kp.nodes_f4 + i) << 4);
  else return kp.tris[i];
}

// Traversal stack entry: global mode 3 dwords (ref, count, t); LDS mode 2
// dwords (ref | count << 24, t) -- LDS mode is only used for scenes whose
// triangle / node indices fit 24 bits and leaves hold < 256 triangles.
template <bool LDSM>
__device__ __forceinline__ void stk_push(const Lane& ln, int sp, uint32_t ref, uint32_t cnt, float t) {
  if constexpr (LDSM) {
    ln.stk[(2 * sp + 0) * ln.stride] = ref | (cnt << 24);
    ln.stk[(2 * sp + 1) * ln.stride] = __float_as_uint(t);
  } else {
    ln.stk[(3 * sp + 0) * ln.stride] = ref;
    ln.stk[(3 * sp + 1) * ln.stride] = cnt;
    ln.stk[(3 * sp + 2) * ln.stride] = __float_as_uint(t);
  }
}
template <bool LDSM>
__device__ __forceinline__ float stk_t(const Lane& ln, int sp) {
  return __uint_as_float(ln.stk[((LDSM ? 2 : 3) * sp + (LDSM ? 1 : 2)) * ln.stride]);
}
template <bool LDSM>
__device__ __forceinline__ void stk_ref(const Lane& ln, int sp, uint32_t& ref, uint32_t& cnt) {
  if constexpr (LDSM) {
    const uint32_t w = ln.stk[(2 * sp) * ln.stride];
    ref = w & 0xFFFFFFu;
    cnt = w >> 24;
  } else {
    ref = ln.stk[(3 * sp + 0) * ln.stride];
    cnt = ln.stk[(3 * sp + 1) * ln.stride];
  }
}
// Entry `slot` of a lane-interleaved stack area (LDS or HBM): field k of the
// entry at base[(F * slot + k) * stride], F = 2 (PACK: ref | count << 24, t) or 3.
template <bool PACK>
__device__ __forceinline__ void slot_write(uint32_t* base, int stride, int slot, uint32_t ref, uint32_t cnt, float t) {
  if constexpr (PACK) {
    base[(2 * slot + 0) * stride] = ref | (cnt << 24);
    base[(2 * slot + 1) * stride] = __float_as_uint(t);
  } else {
    base[(3 * slot + 0) * stride] = ref;
    base[(3 * slot + 1) * stride] = cnt;
    base[(3 * slot + 2) * stride] = __float_as_uint(t);
  }
}
template <bool PACK>
__device__ __forceinline__ void slot_read(const uint32_t* base, int stride, int slot, uint32_t& ref, uint32_t& cnt,
                                          float& t) {
  if constexpr (PACK) {
    const uint32_t w = base[(2 * slot + 0) * stride];
    ref = w & 0xFFFFFFu;
    cnt = w >> 24;
    t = __uint_as_float(base[(2 * slot + 1) * stride]);
  } else {
    ref = base[(3 * slot + 0) * stride];
    cnt = base[(3 * slot + 1) * stride];
    t = __uint_as_float(base[(3 * slot + 2) * stride]);
  }
}

// 1.0f / a, correctly rounded, for every a that is not denormal.  v_rcp_f32
// plus one FMA Newton step equals the correctly rounded quotient for every
// 2^-126 <= |a| < 2^126 (all 2^32 inputs checked on gfx950:
// tools/rcp_exhaustive.hip, tests/test_gpu_rcp.py); |a| >= 2^126, inf and NaN
// take the full division on a branch that is skipped unless some lane of the
// wave needs it.  Callers must not use the result for denormal a (the
// triangle test rejects |a| < 1e-4 before f matters).
__device__ __forceinline__ float recip_normal(float a) {
  float f = recip_newton(a);
  if (__builtin_expect(!(__builtin_fabsf(a) < 0x1p126f), 0)) f = 1.0f / a;
  return f;
}

// IntersectsTriangle (ray_intersects.glsl:61-96, Moller-Trumbore with edges
// precomputed at upload) evaluated without branches: every quantity the reference
// computes on its way to each early return is computed, and the accept
// predicate is their conjunction -- the same decision and the same t
// (f = 1 / a is the correctly rounded division of the reference).
__device__ __forceinline__ bool tri_accept(f3 o, f3 d, float4 A, float4 B, float4 C, float dist, float& tout) {
  const f3 v0 = mk(A.x, A.y, A.z), e1 = mk(A.w, B.x, B.y), e2 = mk(B.z, B.w, C.x);
  const f3 h = cross(d, e2);
  const float a = dot(e1, h);
  const bool parallel = (a > -0.0001f) & (a < 0.0001f);
  const float f = recip_normal(a);  // |a| < 1e-4 is rejected (parallel)
  const f3 s = o - v0;
  const float u = f * dot(s, h);
  const f3 q = cross(s, e1);
  const float v = f * dot(d, q);
  const float t = f * dot(e2, q);
  tout = t;
  return !parallel & !((u < 0.0f) | (u > 1.0f)) & !((v < 0.0f) | (u + v > 1.0f)) & (t > 0.00001f) & (t < dist);
}

// tri_accept split in two for the leaf step: the part up to the reciprocal
// (true when |a| needs the division: recip_normal's fallback range), then the rest.
struct TriPrep {
  f3 v0, e1, e2, h;
  float a, f;
};
__device__ __forceinline__ bool tri_prep(f3 d, float4 A, float4 B, float4 C, TriPrep& p) {
  p.v0 = mk(A.x, A.y, A.z);
  p.e1 = mk(A.w, B.x, B.y);
  p.e2 = mk(B.z, B.w, C.x);
  p.h = cross(d, p.e2);
  p.a = dot(p.e1, p.h);
  p.f = recip_newton(p.a);
  return !(__builtin_fabsf(p.a) < 0x1p126f);
}
__device__ __forceinline__ bool tri_finish(f3 o, f3 d, const TriPrep& p, float dist, float& tout) {
  const bool parallel = (p.a > -0.0001f) & (p.a < 0.0001f);
  const f3 s = o - p.v0;
  const float u = p.f * dot(s, p.h);
  const f3 q = cross(s, p.e1);
  const float v = p.f * dot(d, q);
  const float t = p.f * dot(p.e2, q);
  tout = t;
  return !parallel & !((u < 0.0f) | (u > 1.0f)) & !((v < 0.0f) | (u + v > 1.0f)) & (t > 0.00001f) & (t < dist);
}

// Depth-first traversal in the reference's pop order (right child first).
// Each child's box is tested once, when its parent is expanded; a child that
// fails is never pushed (the running distance only shrinks, so it would fail
// at its pop too); a pushed child is re-checked against the distance at pop
// time with its stored entry distance (the same value IntersectsBox returns).
// `any`: stop at the first accepted triangle (shadow rays, CheckHit(...).hit).
template <bool COUNT, bool LDSM>
__device__ uint32_t traverse(const KParams& kp, const Lane& ln, Counters& c, uint32_t root, f3 o, f3 d,
                             float& dist, bool any) {
  // Flat loop: each iteration performs ONE step for the lane -- test one
  // triangle of the current leaf, expand the current internal node, or pop --
  // so lanes at leaves and lanes at internal nodes advance together.
  // `ref`/`cnt` describe the current node as the reference's node record does
  // (leaf: first triangle + remaining count; internal: index of its first
  // child, cnt == 0); kNone = nothing current, pop next.
  constexpr uint32_t kNone = 0xFFFFFFFFu;
  const f3 inv = mk(recip_exact(d.x), recip_exact(d.y), recip_exact(d.z));
  uint32_t hit = kNone;
  const float4 rlo = node4<LDSM>(kp, 2 * root + 2), rhi = node4<LDSM>(kp, 2 * root + 3);
  bump<COUNT>(c, ST_NODES);
  if (!box_ok(box_t(o, inv, rlo, rhi), dist)) return hit;
  uint32_t ref = __float_as_uint(rlo.w), cnt = __float_as_uint(rhi.w);
  int sp = 0;
  for (;;) {
    if (cnt > 0) {
      // leaf: one triangle per step, in the reference's order
      bump<COUNT>(c, ST_TRIS);
      const uint32_t t3 = 3 * ref;
      float tt;
      if (tri_accept(o, d, tri4<LDSM>(kp, t3), tri4<LDSM>(kp, t3 + 1), tri4<LDSM>(kp, t3 + 2), dist, tt)) {
        dist = tt;
        hit = ref;
        if (any) break;
      }
      ++ref;
      if (--cnt == 0) ref = kNone;
    } else if (ref != kNone) {
      // internal: test both children now.  The reference pushes c0 then c1
      // and pops c1 first; a child whose box fails is never needed (the
      // distance only shrinks), a lone passing child is visited directly.
      const uint32_t pi = 2 * ref + 2;
      const float4 l0 = node4<LDSM>(kp, pi), h0 = node4<LDSM>(kp, pi + 1);
      const float4 l1 = node4<LDSM>(kp, pi + 2), h1 = node4<LDSM>(kp, pi + 3);
      bump<COUNT>(c, ST_NODES, 2);
      const float b0 = box_t(o, inv, l0, h0);
      const float b1 = box_t(o, inv, l1, h1);
      const bool v0 = box_ok(b0, dist), v1 = box_ok(b1, dist);
      const uint32_t r0 = __float_as_uint(l0.w), n0 = __float_as_uint(h0.w);
      if (v0 & v1) {
        if (sp >= kp.stack_entries) {  // cannot happen for a validated BVH
          bump<COUNT>(c, ST_OVERFLOW);
          break;
        }
        stk_push<LDSM>(ln, sp, r0, n0, b0);
        ++sp;
        if constexpr (COUNT) {
          if ((uint32_t)sp > c.v[ST_MAXSTACK]) c.v[ST_MAXSTACK] = (uint32_t)sp;
        }
      }
      ref = v1 ? __float_as_uint(l1.w) : (v0 ? r0 : kNone);
      cnt = v1 ? __float_as_uint(h1.w) : (v0 ? n0 : 0u);
    }
    if (cnt == 0 && ref == kNone) {
      // pop one entry; it is visited if it still beats the running distance
      if (sp == 0) break;
      --sp;
      if (stk_t<LDSM>(ln, sp) < dist) stk_ref<LDSM>(ln, sp, ref, cnt);
    }
  }
  return hit;
}

__device__ __forceinline__ f3 xform(const float* m, f3 v, float w) {
  return mk(((m[0] * v.x + m[4] * v.y) + m[8] * v.z) + m[12] * w,
            ((m[1] * v.x + m[5] * v.y) + m[9] * v.z) + m[13] * w,
            ((m[2] * v.x + m[6] * v.y) + m[10] * v.z) + m[14] * w);
}

// CheckHit over the model BVHs (raytrace_compute.glsl:143-162): closest hit
// triangle (dist updated), or with `any` the first accepted triangle.
template <bool COUNT, bool LDSM>
__device__ uint32_t trace_mesh(const KParams& kp, const Lane& ln, Counters& c, f3 ro, f3 rd, float& dist, bool any) {
  uint32_t hit_tri = 0xFFFFFFFFu;
  for (uint32_t i = 0; i < kp.bvh_count; ++i) {
    const srt_bvh_record& b = kp.bvhs[i];
    const f3 to = xform(b.frame, ro, 1.0f);
    const f3 td = xform(b.frame, rd, 0.0f);
    const uint32_t h = traverse<COUNT, LDSM>(kp, ln, c, b.first_index, to, td, dist, any);
    if (h != 0xFFFFFFFFu) {
      hit_tri = h;
      if (any) break;
    }
  }
  return hit_tri;
}

// raytrace_compute.glsl:93-120 SphereHit
__device__ __forceinline__ bool sphere_hit(f3 ro, f3 rd, f3 pos, float radius, float mn, float mx, float& t) {
  const f3 oc = pos - ro;
  const float ld = length(rd);
  const float a = ld * ld;
  const float h = dot(rd, oc);
  const float loc = length(oc);
  const float cc = loc * loc - (radius * radius);
  const float disc = h * h - a * cc;
  if (disc < 0.0f) return false;
  const float sq = __builtin_sqrtf(disc);
  float root = (h - sq) / a;
  if (!(mn < root && root < mx)) {
    root = (h + sq) / a;
    if (!(mn < root && root < mx)) return false;
  }
  t = root;
  return true;
}

// CheckHit over the five spheres (raytrace_compute.glsl:132-141): index of the
// closest sphere (dist updated) or, with `any`, of the first sphere hit; -1 if none.
__device__ __forceinline__ int trace_spheres(f3 ro, f3 rd, float mn, float& dist, bool any) {
  int best = -1;
  for (int i = 0; i < 5; ++i) {
    f3 pos; float radius; Mat m;
    sphere_data(i, pos, radius, m);
    float t;
    if (sphere_hit(ro, rd, pos, radius, mn, dist, t)) {
      best = i;
      dist = t;
      if (any) break;
    }
  }
  return best;
}

template <bool COUNT>
__device__ __forceinline__ LightRec load_light(const KParams& kp, Counters& c, int idx) {
  bump<COUNT>(c, ST_LIGHTS);
  const int i = (idx >= 0 && idx < kp.light_records) ? idx : kp.light_records;  // zero record
  const float4 a = kp.lights[2 * i], b = kp.lights[2 * i + 1];
  return LightRec{mk(a.x, a.y, a.z), a.w, mk(b.x, b.y, b.z)};
}

__device__ __forceinline__ float ggxD(float NdotH, float rough) {
  const float a2 = rough * rough;
  const float d = ((NdotH * a2 - NdotH) * NdotH + 1.0f);
  return a2 / fmx(0.001f, (d * d * 3.1415926535897f));
}
__device__ __forceinline__ float ggxDNew(float NdotH, float alphaSquared) {
  const float b = ((alphaSquared - 1.0f) * NdotH * NdotH + 1.0f);
  return alphaSquared / fmx(0.001f, (3.1415926535897f * b * b));
}
__device__ __forceinline__ float ggxSchlickMasking(float NdotL, float NdotV, float rough) {
  const float k = rough * rough / 2.0f;
  const float gv = NdotV / fmx(0.001f, (NdotV * (1.0f - k) + k));
  const float gl = NdotL / fmx(0.001f, (NdotL * (1.0f - k) + k));
  return __builtin_fabsf(gv * gl);
}
__device__ __forceinline__ float smithGAlpha(float alpha, float NdotS) {
  return NdotS / (fmx(0.0001f, alpha) * __builtin_sqrtf(1.0f - fmn(0.99999f, NdotS * NdotS)));
}
__device__ __forceinline__ float smithLambda(float a) {
  return (-1.0f + __builtin_sqrtf(1.0f + recip_exact(fmx(0.001f, a * a)))) * 0.5f;
}
__device__ __forceinline__ float smithG2(float alpha, float NdotL, float NdotV) {
  const float aL = smithGAlpha(alpha, NdotL);
  const float aV = smithGAlpha(alpha, NdotV);
  return recip_exact(1.0f + smithLambda(aL) + smithLambda(aV));
}

// brdf.glsl:200-224 SampleDirect up to the shadow factor: returns
// (ggxTerm + NdotL * albedo / pi) and the light term's unshadowed factors.
// Ld = getLightData's direction, H = its guarded half vector with V (computed
// by the caller, shared with the shadow ray; li = intensity * falloff there too)
__device__ f3 sample_direct_brdf(const Hit& hit, f3 Vv, f3 Ld, f3 H) {
  const f3 N = hit.normal;
  const float NdotL = sat(dot(N, Ld));
  const float NdotH = sat(dot(N, H));
  const float LdotH = sat(dot(Ld, H));
  const float NdotV = sat(dot(N, Vv));
  const float rough = hit.mat.roughness;
  const float D = ggxD(NdotH, rough);
  const float G = ggxSchlickMasking(NdotL, NdotV, rough);
  const f3 F = schlickFresnel(hit.mat.specular, LdotH);
  const f3 ggx = (F * (D * G)) / (4.0f * fmx(0.001f, NdotV));
  const f3 diff = (NdotL * hit.mat.albedo) / 3.1415926535897f;
  return ggx + diff;
}

// brdf.glsl:226-237 SampleDirectNew (GetAllBRDFValues :173-198, EvalSpecular :139-145
// with ggxNormalDistributionNew's arguments swapped as in the reference, EvalDiffuse :134-137)
// H = normalize(L + Vv) (computed by the caller as normalize(Vv + L))
__device__ f3 sample_direct_new(const Hit& hit, f3 Vv, f3 L, f3 H) {
  const f3 N = hit.normal;
  const float NdotL = sat(dot(N, L));
  const float NdotV = sat(dot(N, Vv));
  const float LdotH = sat(dot(L, H));
  const float NdotH = sat(dot(N, H));
  const f3 specF0 = specularF0(hit.mat.albedo, hit.mat.metalness);
  const f3 diffRefl = hit.mat.albedo * (1.0f - hit.mat.metalness);
  const float alpha = hit.mat.roughness * hit.mat.roughness;
  const float alphaSq = alpha * alpha;
  const f3 F = fresnelSchlickNew(specF0, shadowedF90(specF0), LdotH);
  const float D = ggxDNew(fmx(0.00001f, alphaSq), NdotH);
  const float G = smithG2(alpha, NdotL, NdotV);
  const float denom = 4.0f * fmx(NdotL, 0.001f) * fmx(NdotV, 0.001f);
  const f3 spec = (((F * G) * D) / fmx(denom, 0.001f)) * NdotL;
  const float oneOverPi = 1.0f / 3.1415926535897f;
  const f3 diff = diffRefl * (oneOverPi * NdotL);
  return ((mk(1.0f, 1.0f, 1.0f) - F) * diff) + spec;
}

// brdf.glsl:279-288
__device__ float brdf_probability(const Mat& m, f3 Vv, f3 N) {
  const float sF0 = luminance(specularF0(m.albedo, m.metalness));
  const float dR = luminance(m.albedo * (1.0f - m.metalness));
  const f3 f0 = mk(sF0, sF0, sF0);
  const float F = sat(luminance(fresnelSchlickNew(f0, shadowedF90(f0), fmx(0.0f, dot(Vv, N)))));
  const float diffuse = dR * (1.0f - F);
  const float p = (F / fmx(0.0001f, (F + diffuse)));
  return clampf(p, 0.1f, 0.9f);
}

// brdf.glsl:81-99 SampleSpecularHalfVec given its two uniform draws
__device__ __forceinline__ f3 specular_half(float rx, float ry, float rough, f3 N) {
  const f3 B = perpendicular(N);
  const f3 T = cross(B, N);
  const float a2 = rough * rough;
  const float cosT = __builtin_sqrtf(fmx(0.0f, (1.0f - rx) / ((a2 - 1.0f) * rx + 1.0f)));
  const float sinT = __builtin_sqrtf(fmx(0.0f, 1.0f - cosT * cosT));
  const float phi = ry * 3.1415926535897f * 2.0f;
  return ((T * (sinT * cos_f(phi))) + (B * (sinT * sin_f(phi)))) + (N * cosT);
}

__device__ __forceinline__ f3 reflect3(f3 I, f3 N) { return I - N * (2.0f * dot(N, I)); }

#define DIFFUSE_BRDF 1
#define SPECULAR_BRDF 2

// brdf.glsl:239-277 SampleIndirectNew with its uniform draws r1 = U(p.xy),
// r2 = U(p.yz) supplied (SampleDiffuse :60-74 and SampleSpecularHalfVec :81-99
// both draw exactly these two numbers).
// SampleIndirectNew (brdf.glsl:239-277).  The diffuse branch (SampleDiffuse +
// its Fresnel weight from SampleSpecularHalfVec) and the specular branch
// (SampleSpecularMicrofacet) share their basis, phi = 2*pi*r2 with its cos/sin
// ((2*pi)*r2 and (r2*pi)*2 round identically: the factor 2 is exact), the GGX
// half vector of (r1, r2) and one Fresnel evaluation, so lanes of a wave that
// took different branches compute those once; every value is the reference's.
__device__ bool sample_indirect(const Hit& hit, f3 Vv, int type, float r1, float r2, f3& dir, f3& weight) {
  const f3 N = hit.normal;
  if (dot(N, Vv) <= 0.0f) return false;
  const f3 specF0 = specularF0(hit.mat.albedo, hit.mat.metalness);
  const f3 B = perpendicular(N);
  const f3 T = cross(B, N);
  const float phi = 2.0f * 3.1415926535897f * r2;
  const float cphi = cos_f(phi), sphi = sin_f(phi);
  // SampleSpecularHalfVec(r1, r2, roughness, N) (brdf.glsl:81-99)
  const float a2 = hit.mat.roughness * hit.mat.roughness;
  const float cosT = __builtin_sqrtf(fmx(0.0f, (1.0f - r1) / ((a2 - 1.0f) * r1 + 1.0f)));
  const float sinT = __builtin_sqrtf(fmx(0.0f, 1.0f - cosT * cosT));
  const f3 Hs = ((T * (sinT * cphi)) + (B * (sinT * sphi))) + (N * cosT);
  f3 nd, w0;
  float fx;
  if (type == DIFFUSE_BRDF) {
    // SampleDiffuse (brdf.glsl:60-74)
    const float r = __builtin_sqrtf(__builtin_fabsf(r1));
    nd = ((T * (r * cphi)) + (B * (r * sphi))) + (N * __builtin_sqrtf(__builtin_fabsf(1.0f - r1)));
    w0 = hit.mat.albedo * (1.0f - hit.mat.metalness);
    fx = fmx(0.00001f, fmn(1.0f, dot(Vv, Hs)));  // VdotH
  } else {
    // brdf.glsl:102-132 SampleSpecularMicrofacet
    const float alpha = hit.mat.roughness * hit.mat.roughness;
    const float alphaSq = alpha * alpha;
    f3 H = Hs;
    if (alpha == 0.0f) {
      const f3 Lt = reflect3(-Vv, N);
      H = normalize(-Vv + Lt);
    }
    const f3 L = reflect3(-Vv, H);
    fx = fmx(0.00001f, fmn(1.0f, dot(H, L)));  // HdotL
    const float NdotL = fmx(0.00001f, fmn(1.0f, dot(N, L)));
    const float N2 = NdotL * NdotL;
    w0 = mk(2.0f / (__builtin_sqrtf(((alphaSq * (1.0f - N2)) + N2) / N2) + 1.0f), 0.0f, 0.0f);
    nd = L;
  }
  const f3 F = fresnelSchlickNew(specF0, shadowedF90(specF0), fx);
  if (type == DIFFUSE_BRDF) weight = w0 * (mk(1.0f, 1.0f, 1.0f) - F);
  else weight = F * w0.x;
  if (luminance(weight) == 0.0f) return false;
  dir = normalize(nd);
  if (dot(N, dir) <= 0.0f) return false;
  return true;
}

template <bool COUNT>
__device__ __forceinline__ void flush_counters(const KParams& kp, const Counters& c) {
  if constexpr (COUNT) {
    for (int k = 0; k < ST_N; ++k) {
      if (k == ST_MAXSTACK) {
        atomicMax(&kp.stats[k], (unsigned long long)c.v[k]);
      } else if (c.v[k]) {
        atomicAdd(&kp.stats[k], (unsigned long long)c.v[k]);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// the path-tracing kernels
// ---------------------------------------------------------------------------
// Work decomposition.  The reference accumulates one path sample per pixel
// per frame: accum = (((accum + L_f0) + L_f0+1) + ...) (raytrace_compute.glsl:
// 400-406).  Every sample L_k is independent (all randomness is a pure
// function of pixel, frame and hit position), only the SUM is ordered.  So
//   sample_kernel     computes samples (pixel, frame) in any order on any lane
//                     and stores each L_k (16 B) to an HBM sample buffer;
//   accumulate_kernel adds them per pixel in frame order (bit-identical sum)
//                     and writes the sRGB8 image.
// sample_kernel is persistent: each wave claims 64-item batches (an 8x8 tile
// of one frame) from a launch-wide counter; lanes whose path has ended take
// the next items of the wave's batch with a ballot + prefix count, so lanes
// stay busy regardless of per-pixel path cost.  Traversal is resumable: a
// wave steps all traversing lanes until fewer than a threshold remain, then
// shades the lanes whose ray has returned (and refills them) while the rest
// keep their traversal state (registers + LDS stack) for the next round.
// ---------------------------------------------------------------------------
struct Trav {
  f3 o, d, inv;       // ray in the current BVH's frame
  float dist;         // running intersection_distance
  uint32_t ref, cnt;  // current node (leaf: first triangle + remaining; internal: first child)
  uint32_t hit;       // best triangle so far (0xFFFFFFFF: none)
  uint32_t bi;        // current BVH
  int sp;
  int lo;             // global-scene mode: entries [lo, sp) are in the LDS ring, [0, lo) in HBM
  bool active;        // still traversing
  bool start;         // next step sets up BVH `bi`
};

constexpr uint32_t kNoneRef = 0xFFFFFFFFu;
#ifndef SRT_LEAF_TRIS
#define SRT_LEAF_TRIS 2
#endif
constexpr int kLeafTris = SRT_LEAF_TRIS;  // triangles tested per leaf step
// Sub-steps of one traversal iteration: 'I' expands an internal node, 'L'
// tests a leaf's next triangles; each is followed by a pop if nothing is current.
#ifndef SRT_STEP_PATTERN
#define SRT_STEP_PATTERN "ILILILIL"
#endif
constexpr char kStepPattern[] = SRT_STEP_PATTERN;
// global-scene mode: entries per lane kept in the LDS ring (power of two)
#ifndef SRT_SHORT_STACK
#define SRT_SHORT_STACK 16
#endif
constexpr int kShortStack = SRT_SHORT_STACK;
// consecutive 64-item batches a wave claims per atomic on the launch's batch counter
#ifndef SRT_CLAIM
#define SRT_CLAIM 4
#endif
constexpr int kClaim = SRT_CLAIM;
static_assert((kShortStack & (kShortStack - 1)) == 0, "kShortStack must be a power of two");
constexpr int kTriPad = 3;                // zero records past the triangle array (>= kLeafTris - 1)
static_assert(kLeafTris >= 1 && kLeafTris - 1 <= kTriPad, "kLeafTris");

// Sets up BVH `t.bi` for the world ray (the reference's per-model transform,
// raytrace_compute.glsl:146-147) and tests its root box.
template <bool COUNT, bool LDSM>
__device__ __forceinline__ void trav_begin_bvh(const KParams& kp, Counters& c, Trav& t, f3 ro, f3 rd) {
  const srt_bvh_record& b = kp.bvhs[t.bi];
  t.o = xform(b.frame, ro, 1.0f);
  t.d = xform(b.frame, rd, 0.0f);
  t.inv = mk(recip_exact(t.d.x), recip_exact(t.d.y), recip_exact(t.d.z));
  const uint32_t root = b.first_index;
  const float4 rlo = node4<LDSM>(kp, 2 * root + 2), rhi = node4<LDSM>(kp, 2 * root + 3);
  bump<COUNT>(c, ST_NODES);
  const bool ok = box_ok(box_t(t.o, t.inv, rlo, rhi), t.dist);
  t.ref = ok ? __float_as_uint(rlo.w) : kNoneRef;
  t.cnt = ok ? __float_as_uint(rhi.w) : 0u;
  t.sp = 0;
  t.lo = 0;
  t.start = false;
}

// Leaf sub-step: up to kLeafTris triangles of the current leaf, in order: each
// is tested against the distance the previous one left; a shadow ray stops at
// its first accept (the triangle array is padded with kTriPad zero records).
template <bool COUNT, bool LDSM>
__device__ __forceinline__ void trav_leaf(const KParams& kp, Counters& c, Trav& t, bool any) {
  const uint32_t n = t.cnt < (uint32_t)kLeafTris ? t.cnt : (uint32_t)kLeafTris;
  bump<COUNT>(c, ST_TRIS, n);
  float dist = t.dist;
  uint32_t hit = t.hit;
  bool stop = false;
  const float4* tp = tri_ptr<LDSM>(kp, t.ref);
  // all triangles' loads and reciprocals first (one shared fallback branch),
  // so the triangles' arithmetic overlaps; then the tests in order
  TriPrep pr[kLeafTris];
  bool slow = false;
#pragma unroll
  for (int k = 0; k < kLeafTris; ++k) slow |= tri_prep(t.d, tp[3 * k], tp[3 * k + 1], tp[3 * k + 2], pr[k]);
  if (__builtin_expect(slow, 0)) {
#pragma unroll
    for (int k = 0; k < kLeafTris; ++k) pr[k].f = 1.0f / pr[k].a;
  }
#pragma unroll
  for (int k = 0; k < kLeafTris; ++k) {
    float tk;
    const bool tk_ok = tri_finish(t.o, t.d, pr[k], dist, tk);
    const bool ak = k == 0 ? tk_ok : (((uint32_t)k < n) & !stop & tk_ok);  // a leaf holds >= 1 triangle
    dist = ak ? tk : dist;
    hit = ak ? t.ref + k : hit;
    stop = stop | (ak & any);
  }
  t.dist = dist;
  t.hit = hit;
  t.ref += n;
  t.cnt -= n;
  t.active = !stop;
  t.ref = (t.cnt == 0 || stop) ? kNoneRef : t.ref;
  t.cnt = stop ? 0u : t.cnt;
}

// Internal sub-step: test both children's boxes; push c0 when both pass, go to
// c1 if it passes, else to c0 if it passes.
template <bool COUNT, bool LDSM, bool PACK>
__device__ __forceinline__ void trav_internal(const KParams& kp, const Lane& ln, Counters& c, Trav& t) {
  const uint32_t pi = 2 * t.ref + 2;
  const float4 l0 = node4<LDSM>(kp, pi), h0 = node4<LDSM>(kp, pi + 1);
  const float4 l1 = node4<LDSM>(kp, pi + 2), h1 = node4<LDSM>(kp, pi + 3);
  bump<COUNT>(c, ST_NODES, 2);
  const float b0 = box_t(t.o, t.inv, l0, h0);
  const float b1 = box_t(t.o, t.inv, l1, h1);
  const bool v0 = box_ok(b0, t.dist), v1 = box_ok(b1, t.dist);
  const uint32_t r0 = __float_as_uint(l0.w), n0 = __float_as_uint(h0.w);
  // the c0 slot is written unconditionally (it is free either way; the stack
  // holds depth + 1 entries, validated at upload)
  if constexpr (LDSM) {
    slot_write<true>(ln.stk, ln.stride, t.sp, r0, n0, b0);
  } else {
    if (t.sp - t.lo == kShortStack) {  // ring full: its oldest entry moves to HBM (rare)
      uint32_t r, n;
      float bt;
      slot_read<PACK>(ln.stk, ln.stride, t.lo & (kShortStack - 1), r, n, bt);
      slot_write<PACK>(ln.gstk, ln.gstride, t.lo, r, n, bt);
      ++t.lo;
    }
    slot_write<PACK>(ln.stk, ln.stride, t.sp & (kShortStack - 1), r0, n0, b0);
  }
  t.sp += (v0 & v1) ? 1 : 0;
  if constexpr (COUNT) {
    if ((uint32_t)t.sp > c.v[ST_MAXSTACK]) c.v[ST_MAXSTACK] = (uint32_t)t.sp;
  }
  t.ref = v1 ? __float_as_uint(l1.w) : (v0 ? r0 : kNoneRef);
  t.cnt = v1 ? __float_as_uint(h1.w) : (v0 ? n0 : 0u);
}

// Nothing current: pop one entry (visited if it still beats the running
// distance), or finish this BVH.  A lane whose next BVH is pending (`start`,
// set up at the next iteration) does nothing.
template <bool LDSM, bool PACK>
__device__ __forceinline__ void trav_pop(const KParams& kp, const Lane& ln, Trav& t, bool any) {
  if (t.active & !t.start & (t.cnt == 0) & (t.ref == kNoneRef)) {
    if (t.sp > 0) {
      --t.sp;
      uint32_t r, n;
      float et;
      if constexpr (LDSM) {
        slot_read<true>(ln.stk, ln.stride, t.sp, r, n, et);
      } else if (t.sp < t.lo) {  // below the LDS ring: from HBM (rare)
        slot_read<PACK>(ln.gstk, ln.gstride, t.sp, r, n, et);
        t.lo = t.sp;
      } else {
        slot_read<PACK>(ln.stk, ln.stride, t.sp & (kShortStack - 1), r, n, et);
      }
      const bool take = et < t.dist;
      t.ref = take ? r : kNoneRef;
      t.cnt = take ? n : 0u;
    } else if ((any && t.hit != kNoneRef) || t.bi + 1 >= kp.bvh_count) {
      t.active = false;  // CheckHit's loop over bvh_count is complete
    } else {
      ++t.bi;
      t.start = true;
    }
  }
}

template <bool COUNT, bool LDSM, bool PACK, int K>
__device__ __forceinline__ void trav_substeps(const KParams& kp, const Lane& ln, Counters& c, Trav& t, bool any) {
  if constexpr (kStepPattern[K] != 0) {
    if constexpr (kStepPattern[K] == 'I') {
      DBG_COUNT(kp.stats, ST_DBG_SUB + 3 * K, t.cnt == 0 && t.ref != kNoneRef);
      if (t.cnt == 0 && t.ref != kNoneRef) trav_internal<COUNT, LDSM, PACK>(kp, ln, c, t);
    } else {
      DBG_COUNT(kp.stats, ST_DBG_SUB + 3 * K, t.cnt > 0);
      if (t.cnt > 0) trav_leaf<COUNT, LDSM>(kp, c, t, any);
    }
    DBG_COUNT(kp.stats, ST_DBG_SUB + 3 * K + 2, t.active & !t.start & (t.cnt == 0) & (t.ref == kNoneRef));
    trav_pop<LDSM, PACK>(kp, ln, t, any);
    trav_substeps<COUNT, LDSM, PACK, K + 1>(kp, ln, c, t, any);
  }
}

// One traversal iteration (see traverse() for the order argument): the
// sub-steps of kStepPattern in turn, each taken by the lanes whose current
// node is of its kind, so a lane makes up to strlen(kStepPattern) steps of
// its own sequence per iteration, in order.  `any` selects the shadow-ray
// (first hit) variant.
template <bool COUNT, bool LDSM, bool PACK>
__device__ __forceinline__ void trav_step(const KParams& kp, const Lane& ln, Counters& c, Trav& t, f3 ro, f3 rd,
                                          bool any) {
  if (t.start) trav_begin_bvh<COUNT, LDSM>(kp, c, t, ro, rd);  // only for BVHs after the first
  trav_substeps<COUNT, LDSM, PACK, 0>(kp, ln, c, t, any);
}

__device__ __forceinline__ int lane_rank(unsigned long long mask, int lane) {
  return __popcll(mask & ((1ull << lane) - 1ull));
}

template <bool COUNT, bool LDSM, bool PACK, int BLOCK>
#ifndef SRT_GLOBAL_WAVES
#define SRT_GLOBAL_WAVES 4
#endif
// waves per SIMD the register allocation must allow: 4 (<= 128 VGPRs) in LDS
// mode, where the 1024-thread block's LDS caps residency at 4 anyway;
// SRT_GLOBAL_WAVES in global-scene mode, whose HBM latency wants more waves
__global__ __launch_bounds__(BLOCK, LDSM ? 4 : SRT_GLOBAL_WAVES) void sample_kernel(KParams kp) {
  const int tid = threadIdx.x;
  if constexpr (LDSM) {  // the block copies the scene (nodes + triangles) into LDS once
    const int total = kp.nodes_f4 + kp.tris_f4;
    for (int i = tid; i < total; i += blockDim.x)
      g_smem[i] = (i < kp.nodes_f4) ? kp.nodes[i] : kp.tris[i - kp.nodes_f4];
    __syncthreads();
  }
  const int lane = tid & 63;
  Lane ln;
  if constexpr (LDSM) {
    ln.stk = reinterpret_cast<uint32_t*>(g_smem + kp.stack_base_f4) + tid;
    ln.stride = blockDim.x;
  } else {  // the top kShortStack entries in an LDS ring, the rest in HBM (lane-interleaved, coalesced)
    ln.stk = reinterpret_cast<uint32_t*>(g_smem) + tid;
    ln.stride = BLOCK;
    ln.gstk = kp.gstack + (size_t)blockIdx.x * BLOCK + tid;
    ln.gstride = kp.gstack_stride;
  }
  ln.base = 0;
  Counters c;
  for (int k = 0; k < ST_N; ++k) c.v[k] = 0;

  const f3 center = mk(kp.cx, kp.cy, kp.cz);
  const int tiles_x = (kp.W + 7) >> 3;
  const int n_tiles = tiles_x * ((kp.local_rows + 7) >> 3);
  const int n_batches = n_tiles * kp.nframes;  // < 2^31: the host bounds the frames per launch
  // batches are claimed one at a time from a launch-wide counter, so waves
  // that drew cheap tiles take more of them (no static-share tail).  The
  // next batch is claimed one ahead: lane 0's atomic returns while the
  // current batch is consumed, and is only read (broadcast) when needed.
  // kClaim consecutive batches per claim.
  // `batch` and everything derived from it are wave-uniform (scalar registers).
  unsigned long long claimed = 0;
  if (lane == 0) claimed = atomicAdd(kp.batch_ctr, 1ull);
  int batch = __builtin_amdgcn_readfirstlane((int)__shfl(claimed, 0)) * kClaim;
  int claim_left = kClaim - 1;  // batches of the current claim after `batch`
  if (lane == 0) claimed = atomicAdd(kp.batch_ctr, 1ull);
  int batch_next = 0;         // items of `batch` already handed out

  // per-lane sample / path / traversal state
  bool has_work = false;
  int x = 0, gy = 0, li = 0, fidx = 0;
  f3 ro = mk(0.f, 0.f, 0.f), rd = mk(0.f, 0.f, 1.f), T, color, q0, q1, nd;
  float tmax = 0.0f;
  int depth = 0, randIndex = 0, hit_sphere = -1, bounces = 0;
  bool shadow_phase = false, term = false;
  Trav tr;
  tr.active = false;
  tr.start = false;
  tr.hit = kNoneRef;

  auto start_ray = [&]() {
    tr.dist = tmax;
    tr.hit = kNoneRef;
    tr.bi = 0;
    tr.active = true;
    tr.start = false;
    bump<COUNT>(c, ST_RAYS);
    if (kp.show_model) {
      trav_begin_bvh<COUNT, LDSM>(kp, c, tr, ro, rd);
      if (tr.cnt == 0 && tr.ref == kNoneRef) {  // root box missed: next BVH, or done
        if (kp.bvh_count > 1) tr.start = true, tr.bi = 1;
        else tr.active = false;
      }
    } else {  // the five spheres are "traversed" in one go
      float dist = tmax;
      hit_sphere = trace_spheres(ro, rd, 0.001f, dist, shadow_phase);
      tr.dist = dist;
      tr.active = false;
    }
  };
  auto finish_sample = [&]() {
    color = color + T * mk(0.05f, 0.05f, 0.05f);  // skyColor, raytrace_compute.glsl:219,292
    kp.lbuf[(size_t)fidx * (size_t)kp.local_pixels + (size_t)li] = make_float4(color.x, color.y, color.z, 0.0f);
    has_work = false;
  };

#ifdef SRT_PHASE_TIMING
  unsigned long long cyc_refill = 0, cyc_trav = 0, cyc_shade = 0, iters = 0;
  unsigned long long d_titers = 0, d_work = 0, d_trav = 0, d_leaf = 0, d_int = 0, d_shade = 0;
#endif
  for (;;) {
    PHASE_STAMP(t_a);
    // ---- (A) idle lanes take the next items of the wave's batches ----
    for (;;) {
      const unsigned long long idle = __ballot(!has_work);
      if (idle == 0ull || batch >= n_batches) break;
      const int avail = 64 - batch_next;
      const int r = lane_rank(idle, lane);
      // the batch's frame and 8x8 tile (wave-uniform integer divisions, once per batch)
      const int frame_i = batch / n_tiles;
      const int tile = batch - frame_i * n_tiles;
      const int ty = tile / tiles_x, tx = tile - ty * tiles_x;
      const int samp = (kp.frame_first + frame_i) % kp.WH;
      // row band of the tile when bands are whole tiles (the default 8 rows)
      const int band_u = (kp.band_rows & 7) == 0 ? ty / (kp.band_rows >> 3) : -1;
      if (!has_work && r < avail) {
        const int item = batch_next + r;
        const int px = tx * 8 + (item & 7), ly = ty * 8 + (item >> 3);
        if (px < kp.ext_w && ly < kp.local_rows) {
          int band;
          if (band_u >= 0) band = band_u;
          else band = ly / kp.band_rows;
          const int yy = (band * kp.nranks + kp.rank) * kp.band_rows + (ly - band * kp.band_rows);
          if (yy < kp.ext_h) {
            has_work = true;
            x = px;
            gy = yy;
            li = ly * kp.W + px;
            fidx = frame_i;
            ln.base = gy * kp.H + x;
            // GetRay (raytrace_compute.glsl:78-90) with SampleSquare (raytrace_utils.glsl:10-17)
            const float2 nz = kp.noise_xy[wrap_index(ln.base + samp, kp.WH)];
            bump<COUNT>(c, ST_RNGSQ);
            bump<COUNT>(c, ST_SAMPLES);
            const f3 p00 = mk(kp.p00x, kp.p00y, kp.p00z);
            const f3 du = mk(kp.dux, kp.duy, kp.duz);
            const f3 dv = mk(kp.dvx, kp.dvy, kp.dvz);
            const f3 ps = (p00 + du * ((float)x + (nz.x - 0.5f))) + dv * ((float)gy + (nz.y - 0.5f));
            ro = center;
            rd = ps - center;
            tmax = __builtin_inff();
            T = mk(1.0f, 1.0f, 1.0f);
            color = mk(0.0f, 0.0f, 0.0f);
            depth = kp.max_depth;
            randIndex = 0;
            bounces = 0;
            shadow_phase = false;
            term = false;
            start_ray();
          }
        }
      }
      const int taken = __popcll(idle) < avail ? __popcll(idle) : avail;
      batch_next += taken;
      if (batch_next == 64) {
        if (claim_left > 0) {
          ++batch;
          --claim_left;
        } else {
          batch = __builtin_amdgcn_readfirstlane((int)__shfl(claimed, 0)) * kClaim;
          claim_left = kClaim - 1;
          if (lane == 0) claimed = atomicAdd(kp.batch_ctr, 1ull);
        }
        batch_next = 0;
      }
    }
    if (__ballot(has_work) == 0ull) break;
    PHASE_STAMP(t_b);

    // ---- (B) traverse until too few lanes are still traversing ----
    if (kp.show_model) {
      // has_work is fixed during traversal; trav_frac16 <= 16 makes
      // n_trav * 16 < n_work * trav_frac16 imply n_trav < n_work
      const int work_lim = __popcll(__ballot(has_work)) * kp.trav_frac16;
      for (;;) {
        const unsigned long long trav = __ballot(tr.active);
        if (trav == 0ull) break;
        if (__popcll(trav) * 16 < work_lim) break;
#ifdef SRT_PHASE_TIMING
        ++d_titers;
        d_work += __popcll(__ballot(has_work));
        d_trav += __popcll(trav);
        d_leaf += __popcll(__ballot(tr.active && tr.cnt > 0));
        d_int += __popcll(__ballot(tr.active && tr.cnt == 0 && tr.ref != kNoneRef));
#endif
        if (tr.active) trav_step<COUNT, LDSM, PACK>(kp, ln, c, tr, ro, rd, shadow_phase);
      }
    }

    PHASE_STAMP(t_c);
#ifdef SRT_PHASE_TIMING
    d_shade += __popcll(__ballot(has_work && !tr.active));
#endif
    // ---- (C) lanes whose ray returned: shade (GetRayColor's loop body) ----
    if (has_work && !tr.active) {
      const bool hit = kp.show_model ? (tr.hit != kNoneRef) : (hit_sphere >= 0);
      const float dist = tr.dist;
      if (shadow_phase) {  // CheckLightOccluded returned: this bounce's direct light
        color = color + (hit ? q0 : q1);
        if (term) {
          finish_sample();
        } else {
          rd = nd;  // the bounce ray starts at the same hit point as the shadow ray
          tmax = __builtin_inff();
          shadow_phase = false;
          start_ray();
        }
      } else if (!hit) {
        finish_sample();
      } else {
        // ---- hit record (CheckHit) ----
        Hit rec;
        rec.hit = true;
        if (kp.show_model) {
          rec.p = (dist * rd) + ro;
          const uint32_t ht = tr.hit;
          const float4 A = tri4<LDSM>(kp, 3 * ht), B = tri4<LDSM>(kp, 3 * ht + 1), C = tri4<LDSM>(kp, 3 * ht + 2);
          rec.normal = normalize(cross(mk(A.w, B.x, B.y), mk(B.z, B.w, C.x)));
          const uint32_t mi = __float_as_uint(C.y);
          const float4 m0 = kp.mats[2 * mi], m1 = kp.mats[2 * mi + 1];
          bump<COUNT>(c, ST_MATS);
          rec.mat.albedo = mk(m0.x, m0.y, m0.z);
          rec.mat.roughness = m0.w;
          rec.mat.specular = mk(m1.x, m1.y, m1.z);
          rec.mat.metalness = 0.1f;
          rec.mat.useSpec = true;
        } else {
          f3 pos; float radius;
          sphere_data(hit_sphere, pos, radius, rec.mat);
          rec.p = ro + rd * dist;
          const f3 outward = (rec.p - pos) / radius;   // SetFaceNormal (raytrace_utils.glsl:23-26)
          rec.normal = (dot(rd, outward) < 0.0f) ? outward : -outward;
        }
        const f3 p = rec.p;
        const f3 Vv = -rd;

        // ---- this bounce's independent uniform draws, fetched together ----
        const int n = kp.light_count;
        const bool fixed_spec = (rec.mat.metalness == 1.0f && rec.mat.roughness == 0.0f);
        const int i_r1 = randU_index(kp, ln, p.x, p.y);             // light index; SampleDiffuse r1
        const int i_r2 = randU_index(kp, ln, p.y, p.z);             // SampleDiffuse r2
        const int i_sel = randU_index(kp, ln, p.y + 0.0f, p.z + 0.0f);
        const int i_bp = randU_index(kp, ln, p.x + (float)depth, p.y + (float)depth);
        const bool rr = depth <= 0;
        const int i_rr = rr ? randU_index(kp, ln, p.x + (float)randIndex, p.y + (float)randIndex) : 0;
        const float r1 = kp.noise_u[i_r1];
        const float r2 = kp.noise_u[i_r2];
        const float u_sel0 = kp.noise_u[i_sel];
        const float u_bp = kp.noise_u[i_bp];
        const float u_rr = rr ? kp.noise_u[i_rr] : 1.0f;
        if constexpr (COUNT) c.v[ST_RNGU] += 4 + (rr ? 1 : 0);

        // ---- SampleLights (raytrace_compute.glsl:179-206) ----
        // randLightIndex uses the same seed every iteration, so the light and its
        // pdf are loop-invariant; after the first selection later iterations only
        // re-select it, so their draws are skipped (the result is unchanged).
        bool selected = false;
        float lw = 0.0f;
        LightRec L;
        f3 toL = mk(0.f, 0.f, 0.f);
        float fo = 0.0f, d2L = 0.0f;
        if (n > 0) {
          L = load_light<COUNT>(kp, c, f2i(__builtin_rintf(r1 * (float)n)));
          toL = L.pos - p;
          d2L = dot(toL, toL);
          fo = recip_exact((0.01f * 0.01f) + d2L);  // GetLightFalloff(p, L) (brdf.glsl:147-152)
          const float inten = L.intensity * fo;
          const float lpdf = luminance(mk(inten, inten, inten));
          const float ris = lpdf * (float)n;
          float total = 0.0f, pdf = 0.0f;
          for (int i = 0; i < n; ++i) {
            total += ris;
            if (!selected) {
              const float r = (i == 0) ? u_sel0 : randU<COUNT>(kp, ln, c, p.y + (float)i, p.z + (float)i);
              if (r < (ris / total)) {
                pdf = lpdf;
                selected = true;
              }
            }
          }
          lw = (total / (float)n) / fmx(0.001f, pdf);
        }

        // ---- direct light, both shadow outcomes (raytrace_compute.glsl:233-246) ----
        f3 sdir = mk(0.f, 0.f, 0.f);
        float smax = 0.0f;
        if (selected) {
          // shared by the shadow ray, getLightData and both direct-light BRDFs:
          // length(toL), normalize(toL) = toL * (1 / length), light_dir = the
          // normalized vector (toL itself when zero), the half vector of it and V
          smax = __builtin_sqrtf(d2L);
          sdir = toL * recip_exact(smax);
          const f3 Ld = smax > 0.0f ? sdir : toL;
          const f3 vl = Vv + Ld;
          const float lvl = length(vl);
          const f3 Hn = vl * recip_exact(lvl);  // normalize(vl)
          if (rec.mat.useSpec) {
            const float li_ = L.intensity * fo;
            const f3 bd = sample_direct_brdf(rec, Vv, Ld, lvl > 0.0f ? Hn : vl);
            q1 = (T * (((1.0f * L.color) * li_) * bd)) * lw;
            q0 = (T * (((0.0f * L.color) * li_) * bd)) * lw;
          } else {
            const f3 lint = ((L.color * fo) * L.intensity) * lw;
            const f3 tx = T * sample_direct_new(rec, Vv, Ld, Hn);
            q1 = (tx * 1.0f) * lint;
            q0 = (tx * 0.0f) * lint;
          }
        }

        // ---- BRDF choice, Russian roulette, next direction (:248-285) ----
        int type;
        if (fixed_spec) {
          type = SPECULAR_BRDF;
        } else {
          const float bp = brdf_probability(rec.mat, Vv, rec.normal);
          // T / bp (specular) or T / (1 - bp) (diffuse): one division by the chosen divisor
          const bool spec = u_bp < bp;
          type = spec ? SPECULAR_BRDF : DIFFUSE_BRDF;
          T = T / (spec ? bp : (1.0f - bp));
        }
        term = false;
        if (rr) {
          const float surv = clampf(luminance(T), 0.1f, 1.0f);
          if (u_rr > surv) {
            term = true;
          } else {
            T = T / surv;
            randIndex++;
          }
        } else {
          depth--;
        }
        if (!term) {
          f3 dir, bw;
          if (!sample_indirect(rec, Vv, type, r1, r2, dir, bw)) {
            term = true;
          } else {
            T = T * bw;
            nd = dir;
          }
        }

        // The reference's loop has no depth cap (Russian roulette clamps the
        // survival probability to >= 0.1).  A path still alive after 2^20
        // bounces is cut (and counted) so a pathological scene cannot hang the GPU.
        if (++bounces >= (1 << 20) && !term) {
          term = true;
          bump<COUNT>(c, ST_OVERFLOW);
        }
        ro = p;
        if (selected) {  // trace CheckLightOccluded's ray next (t in (0.001, |light - p|))
          rd = sdir;
          tmax = smax;
          shadow_phase = true;
          start_ray();
        } else if (term) {
          finish_sample();
        } else {
          rd = nd;
          tmax = __builtin_inff();
          start_ray();
        }
      }
    }
#ifdef SRT_PHASE_TIMING
    PHASE_STAMP(t_d);
    cyc_refill += t_b - t_a;
    cyc_trav += t_c - t_b;
    cyc_shade += t_d - t_c;
    ++iters;
#endif
  }
#ifdef SRT_PHASE_TIMING
  if (lane == 0) {
    atomicAdd(&kp.stats[ST_CYC_REFILL], cyc_refill);
    atomicAdd(&kp.stats[ST_CYC_TRAV], cyc_trav);
    atomicAdd(&kp.stats[ST_CYC_SHADE], cyc_shade);
    atomicAdd(&kp.stats[ST_CYC_ITERS], iters);
    atomicAdd(&kp.stats[ST_DBG_TITERS], d_titers);
    atomicAdd(&kp.stats[ST_DBG_WORK], d_work);
    atomicAdd(&kp.stats[ST_DBG_TRAV], d_trav);
    atomicAdd(&kp.stats[ST_DBG_LEAF], d_leaf);
    atomicAdd(&kp.stats[ST_DBG_INT], d_int);
    atomicAdd(&kp.stats[ST_DBG_SHADE], d_shade);
  }
#endif
  flush_counters<COUNT>(kp, c);
}

// Ordered sum of the sample buffer into the accumulation image (raytrace_compute.glsl:
// 404-406 for frames frame_first .. frame_first + nframes - 1) and the sRGB8
// image for accumFrames = out_frames (:412-413).
__global__ __launch_bounds__(256) void accumulate_kernel(KParams kp, int out_frames) {
  const int li = blockIdx.x * blockDim.x + threadIdx.x;
  if (li >= kp.local_pixels) return;
  const int ly = li / kp.W, x = li - ly * kp.W;
  const int band = ly / kp.band_rows;
  const int gy = (band * kp.nranks + kp.rank) * kp.band_rows + (ly - band * kp.band_rows);
  if (x >= kp.ext_w || gy >= kp.ext_h) return;
  const float4 a0 = kp.accum[li];
  f3 acc = mk(a0.x, a0.y, a0.z);
  const float4* L = kp.lbuf + li;
  for (int k = 0; k < kp.nframes; ++k) {
    const float4 s = L[(size_t)k * (size_t)kp.local_pixels];
    acc = acc + mk(s.x, s.y, s.z);
  }
  kp.accum[li] = make_float4(acc.x, acc.y, acc.z, 1.0f);
  if (kp.write_output) {
    const f3 o = acc / (float)out_frames;
    const uint32_t r = to_unorm8(linearToSrgb(o.x)), g = to_unorm8(linearToSrgb(o.y)),
                   b = to_unorm8(linearToSrgb(o.z));
    kp.out[li] = r | (g << 8) | (b << 16) | (255u << 24);
  }
}

// resetAccumBuffer (raytrace_compute.glsl:390-393)
__global__ __launch_bounds__(256) void reset_kernel(KParams kp) {
  const int li = blockIdx.x * blockDim.x + threadIdx.x;
  if (li >= kp.local_pixels) return;
  const int ly = li / kp.W, x = li - ly * kp.W;
  const int band = ly / kp.band_rows;
  const int gy = (band * kp.nranks + kp.rank) * kp.band_rows + (ly - band * kp.band_rows);
  if (x >= kp.ext_w || gy >= kp.ext_h) return;
  kp.accum[li] = make_float4(0.0f, 0.0f, 0.0f, 1.0f);
}

// The closest-hit test kernel of ray_intersects.glsl:135-161.
__global__ __launch_bounds__(256) void closest_kernel(KParams kp, const srt_ray* rays, uint32_t n, uint32_t* hits,
                                                      float* tout) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Lane ln;
  ln.base = 0;
  ln.stk = reinterpret_cast<uint32_t*>(g_smem) + threadIdx.x;
  ln.stride = blockDim.x;
  Counters c;
  for (int k = 0; k < ST_N; ++k) c.v[k] = 0;
  const srt_ray r = rays[i];
  const f3 o = mk(r.origin[0], r.origin[1], r.origin[2]);
  const f3 d = mk(r.direction[0], r.direction[1], r.direction[2]);
  float dist = r.intersection_distance;
  uint32_t hit = 0xFFFFFFFFu;
  for (uint32_t b = 0; b < kp.bvh_count; ++b) {
    const srt_bvh_record& rec = kp.bvhs[b];
    const uint32_t h = traverse<true, false>(kp, ln, c, rec.first_index, xform(rec.frame, o, 1.0f),
                                      xform(rec.frame, d, 0.0f), dist, false);
    if (h != 0xFFFFFFFFu) hit = h;
  }
  hits[i] = hit;
  tout[i] = dist;
  flush_counters<true>(kp, c);
}

// Root-side assembly after the multi-GPU gather: gathered[r] holds rank r's
// packed local rows (bands b with b % nranks == r, `rows_pad` rows each);
// writes the full-frame accumulation image and its sRGB8 display image
// (raytrace_compute.glsl:412-413 with accumFrames = `frames`).
__global__ __launch_bounds__(256) void assemble_kernel(const float4* gathered, int nranks, int rows_pad, int W, int H,
                                                       int band_rows, int frames, float4* accum, uint32_t* out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)W * (size_t)H) return;
  const int y = (int)(i / (size_t)W), x = (int)(i - (size_t)y * W);
  const int band = y / band_rows;
  const int r = band % nranks;
  const int lband = band / nranks;
  const int ly = lband * band_rows + (y - band * band_rows);
  const float4 a = gathered[((size_t)r * rows_pad + ly) * W + x];
  if (accum) accum[i] = a;
  if (out) {
    const float inv = (float)frames;
    const f3 o = mk(a.x, a.y, a.z) / inv;
    const uint32_t rr = to_unorm8(linearToSrgb(o.x)), g = to_unorm8(linearToSrgb(o.y)), b = to_unorm8(linearToSrgb(o.z));
    out[i] = rr | (g << 8) | (b << 16) | (255u << 24);
  }
}

}  // namespace srt

// ===========================================================================
// host side: the device context behind the C ABI
// ===========================================================================
namespace srt {

static std::mutex g_err_mu;
static std::string g_err;
void SetError(const std::string& msg) {
  std::lock_guard<std::mutex> lk(g_err_mu);
  g_err = msg;
}
const char* LastError() {
  std::lock_guard<std::mutex> lk(g_err_mu);
  return g_err.c_str();
}

}  // namespace srt

#define HIP_OK(expr)                                                                          \
  do {                                                                                        \
    hipError_t e_ = (expr);                                                                   \
    if (e_ != hipSuccess) {                                                                   \
      srt::SetError(std::string(#expr) + ": " + hipGetErrorString(e_));                     \
      return SRT_ERR_HIP;                                                                     \
    }                                                                                         \
  } while (0)

struct srt_context {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  // uniforms
  int W = 0, H = 0, accum_frames = 0, reset = 0, show_model = 0, light_count = 0, max_depth = 5;
  uint32_t bvh_count = 0;
  float cam_origin[3] = {0, 0, 0}, cam_dir[3] = {0, 0, -1}, cam_up[3] = {0, 1, 0}, cam_right[3] = {1, 0, 0};
  // tiling
  int rank = 0, nranks = 1, band_rows = 16;
  // scene
  float4* d_nodes = nullptr;
  float4* d_tris = nullptr;
  float4* d_mats = nullptr;
  srt_bvh_record* d_bvhs = nullptr;
  uint32_t bvh_capacity = 0;
  uint32_t bvh_uploaded = 0;   // records on the device (valid while !bvhs_dirty)
  bool bvhs_dirty = true;
  std::vector<srt_bvh_record> h_bvhs;
  uint32_t n_nodes = 0, n_tris = 0, n_mats = 0;
  int stack_entries = 1;
  bool scene_ok = false;
  bool lds_ok = false;        // scene indices fit the packed LDS stack entry
  bool force_global = false;  // SRT_FORCE_GLOBAL_SCENE=1 disables LDS mode
  // lights
  std::vector<srt_light> h_lights;
  float4* d_lights = nullptr;
  uint32_t light_capacity = 0;
  bool lights_dirty = true;
  // noise
  float2* d_noise_xy = nullptr;
  float* d_noise_u = nullptr;
  size_t noise_texels = 0;
  // images
  float4* d_accum = nullptr;
  uint32_t* d_out = nullptr;
  bool images_external = false;
  int img_w = 0, img_rows = 0;
  // sample buffer (nframes x local pixels float4)
  float4* d_lbuf = nullptr;
  uint32_t* d_gstack = nullptr;  // global-scene mode traversal stacks
  size_t gstack_bytes = 0;
  unsigned long long* d_batch_ctr = nullptr;  // one batch counter per chunk launch
  int batch_ctr_cap = 0;
  size_t lbuf_bytes = 0;
  size_t lbuf_cap = (size_t)16 << 30;  // SRT_SAMPLE_BUFFER_MB
  int trav_frac16 = 8;                 // SRT_TRAV_FRAC16 (measured best on Rubik 1080p with 2-triangle leaf steps)
  int lds_block = 1024;                // SRT_LDS_BLOCK (512 or 1024 threads per block in LDS mode)
  int num_cus = 256;
  // stats
  unsigned long long* d_stats = nullptr;
  srt_stats stats{};
  // per-chunk HIP events around the sample kernel of the last render call
  std::vector<hipEvent_t> ev;
  int ev_used = 0;
};

namespace {

void FreeDev(void* p) {
  if (p) (void)hipFree(p);
}

int LocalRows(const srt_context* c, int H) {
  int rows = 0;
  const int nb = (H + c->band_rows - 1) / c->band_rows;
  for (int b = c->rank; b < nb; b += c->nranks) rows += std::min(c->band_rows, H - b * c->band_rows);
  return rows;
}

int EnsureBvhs(srt_context* c) {
  const uint32_t need = std::max<uint32_t>(c->bvh_count, 1);
  if (!c->bvhs_dirty && c->bvh_uploaded >= need) return SRT_OK;
  std::vector<srt_bvh_record> recs(need);
  std::memset(recs.data(), 0, sizeof(srt_bvh_record) * need);   // bvhs[i >= n] read as zeros
  for (uint32_t i = 0; i < need && i < c->h_bvhs.size(); ++i) recs[i] = c->h_bvhs[i];
  if (need > c->bvh_capacity) {
    FreeDev(c->d_bvhs);
    c->d_bvhs = nullptr;
    HIP_OK(hipMalloc(&c->d_bvhs, sizeof(srt_bvh_record) * need));
    c->bvh_capacity = need;
  }
  HIP_OK(hipMemcpyAsync(c->d_bvhs, recs.data(), sizeof(srt_bvh_record) * need, hipMemcpyHostToDevice, c->stream));
  HIP_OK(hipStreamSynchronize(c->stream));
  c->bvh_uploaded = need;
  c->bvhs_dirty = false;
  return SRT_OK;
}

int EnsureLights(srt_context* c) {
  if (!c->lights_dirty) return SRT_OK;
  // the uploaded records plus one zero record that out-of-range indices map
  // to (lights[lightCount] is an out-of-bounds SSBO read, src/main.cpp:690)
  const size_t n = c->h_lights.size() + 1;
  std::vector<float4> rec(2 * n, make_float4(0, 0, 0, 0));
  for (size_t i = 0; i < c->h_lights.size(); ++i) {
    const srt_light& l = c->h_lights[i];
    rec[2 * i] = make_float4(l.position[0], l.position[1], l.position[2], l.intensity);
    rec[2 * i + 1] = make_float4(l.color[0], l.color[1], l.color[2], 0.0f);
  }
  if (n > c->light_capacity) {
    FreeDev(c->d_lights);
    c->d_lights = nullptr;
    HIP_OK(hipMalloc(&c->d_lights, sizeof(float4) * 2 * n));
    c->light_capacity = (uint32_t)n;
  }
  HIP_OK(hipMemcpyAsync(c->d_lights, rec.data(), sizeof(float4) * 2 * n, hipMemcpyHostToDevice, c->stream));
  HIP_OK(hipStreamSynchronize(c->stream));
  c->lights_dirty = false;
  return SRT_OK;
}

// GetCamera (raytrace_compute.glsl:47-76) with focusDist = 1 (:384)
void CameraParams(const srt_context* c, srt::KParams* kp) {
  const float aspect = (float)c->W / (float)c->H;
  const float hf = (float)c->W / aspect;
  int height = (hf != hf) ? 0 : (int)hf;
  height = (height < 1) ? 1 : height;
  const float focus = 1.0f;
  const float w[3] = {-c->cam_dir[0], -c->cam_dir[1], -c->cam_dir[2]};
  float du[3], dv[3], p00[3];
  for (int i = 0; i < 3; ++i) {
    const float viewU = c->cam_right[i] * focus;
    const float viewV = c->cam_up[i] * focus;
    du[i] = viewU / (float)c->W;
    dv[i] = viewV / (float)height;
    const float ll = ((c->cam_origin[i] - focus * w[i]) - viewU / 2.0f) - viewV / 2.0f;
    p00[i] = ll + 0.5f * (du[i] + dv[i]);
  }
  kp->cx = c->cam_origin[0]; kp->cy = c->cam_origin[1]; kp->cz = c->cam_origin[2];
  kp->p00x = p00[0]; kp->p00y = p00[1]; kp->p00z = p00[2];
  kp->dux = du[0]; kp->duy = du[1]; kp->duz = du[2];
  kp->dvx = dv[0]; kp->dvy = dv[1]; kp->dvz = dv[2];
}

int FillParams(srt_context* c, srt::KParams* kp, bool need_images) {
  if (c->W <= 0 || c->H <= 0) { srt::SetError("Width/Height not set"); return SRT_ERR_STATE; }
  if (c->show_model && !c->scene_ok) { srt::SetError("showModel set but no scene uploaded"); return SRT_ERR_STATE; }
  if (need_images) {
    if (c->noise_texels != (size_t)c->W * (size_t)c->H) {
      srt::SetError("noise buffers must hold Width*Height texels");
      return SRT_ERR_STATE;
    }
    if (!c->d_accum || c->img_w != c->W || c->img_rows != LocalRows(c, c->H)) {
      srt::SetError("images not allocated for the current Width/Height/tiling (srt_alloc_images)");
      return SRT_ERR_STATE;
    }
  }
  int rc = EnsureLights(c);
  if (rc) return rc;
  if (c->show_model) {
    rc = EnsureBvhs(c);
    if (rc) return rc;
  }
  std::memset(kp, 0, sizeof(*kp));
  kp->nodes = c->d_nodes;
  kp->tris = c->d_tris;
  kp->mats = c->d_mats;
  kp->lights = c->d_lights;
  kp->bvhs = c->d_bvhs;
  kp->noise_xy = c->d_noise_xy;
  kp->noise_u = c->d_noise_u;
  kp->accum = c->d_accum;
  kp->out = c->d_out;
  kp->stats = c->d_stats;
  kp->W = c->W;
  kp->H = c->H;
  kp->WH = c->W * c->H;
  kp->light_count = std::max(c->light_count, 0);
  kp->light_records = (int)c->h_lights.size();
  kp->bvh_count = c->bvh_count;
  kp->show_model = c->show_model;
  kp->max_depth = c->max_depth;
  kp->rank = c->rank;
  kp->nranks = c->nranks;
  kp->band_rows = c->band_rows;
  kp->local_rows = LocalRows(c, c->H);
  kp->local_pixels = kp->local_rows * c->W;
  kp->ext_w = c->W;
  kp->ext_h = c->H;
  kp->stack_entries = c->stack_entries;
  kp->nodes_f4 = (int)(2 * ((size_t)c->n_nodes + 1));
  kp->tris_f4 = (int)(3 * ((size_t)c->n_tris + srt::kTriPad));  // with the padding records
  CameraParams(c, kp);
  return SRT_OK;
}

// LDS budget per CU (gfx950: 160 KiB; one 1024-thread block per CU in LDS mode)
constexpr size_t kLdsBytes = 160 * 1024;

template <bool COUNT, bool LDSM, bool PACK, int BLOCK>
int LaunchSamples(srt_context* c, srt::KParams kp, size_t lds) {
  int per_cu = 0;
  HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, srt::sample_kernel<COUNT, LDSM, PACK, BLOCK>, BLOCK,
                                                        lds));
  per_cu = std::max(per_cu, 1);
  const int blocks = c->num_cus * per_cu;
  if constexpr (!LDSM) {  // global-scene mode: every lane's full stack in HBM (backing the LDS ring)
    const size_t lanes = (size_t)blocks * BLOCK;
    const size_t need = lanes * (PACK ? 2 : 3) * sizeof(uint32_t) * (size_t)kp.stack_entries;
    if (need > c->gstack_bytes) {
      FreeDev(c->d_gstack);
      c->d_gstack = nullptr;
      c->gstack_bytes = 0;
      HIP_OK(hipMalloc(&c->d_gstack, need));
      c->gstack_bytes = need;
    }
    kp.gstack = c->d_gstack;
    kp.gstack_stride = (int)lanes;
  }
  hipLaunchKernelGGL((srt::sample_kernel<COUNT, LDSM, PACK, BLOCK>), dim3(blocks), dim3(BLOCK), lds, c->stream, kp);
  HIP_OK(hipGetLastError());
  return SRT_OK;
}

// Runs frames kp.frame_first .. + kp.nframes - 1 (or the reset frame) through
// sample_kernel + accumulate_kernel, in chunks that fit the sample buffer.
int Launch(srt_context* c, srt::KParams& kp, bool count) {
  const int npx = kp.local_pixels;
  if (npx <= 0) return SRT_OK;
  const dim3 pgrid((unsigned)((npx + 255) / 256));
  if (kp.reset) {
    hipLaunchKernelGGL(srt::reset_kernel, pgrid, dim3(256), 0, c->stream, kp);
    HIP_OK(hipGetLastError());
    return SRT_OK;
  }
  if (kp.nframes <= 0) return SRT_OK;
  // LDS mode: the whole scene + 1024 lanes' 2-dword stacks fit in one CU's LDS
  const size_t scene_bytes = ((size_t)kp.nodes_f4 + (size_t)kp.tris_f4) * sizeof(float4);
  const int lds_block = c->lds_block;
  const size_t lds_mode_bytes = scene_bytes + (size_t)lds_block * 2 * sizeof(uint32_t) * (size_t)kp.stack_entries;
  const bool ldsm = kp.show_model && c->lds_ok && !c->force_global && lds_mode_bytes <= kLdsBytes;
  const int block = ldsm ? lds_block : 256;
  size_t lds;
  if (ldsm) {
    kp.stack_base_f4 = kp.nodes_f4 + kp.tris_f4;
    lds = lds_mode_bytes;
  } else {  // LDS rings of kShortStack entries per lane, backed by HBM stacks (LaunchSamples)
    kp.stack_base_f4 = 0;
    lds = (size_t)block * (c->lds_ok ? 2 : 3) * sizeof(uint32_t) * (size_t)srt::kShortStack;
  }
  // sample buffer: as many frames per chunk as the buffer cap allows
  const size_t per_frame = (size_t)npx * sizeof(float4);
  // frames per launch: what the sample buffer holds, and n_tiles * frames < 2^31 (the kernel's batch index)
  const size_t n_tiles = (size_t)((kp.W + 7) >> 3) * (size_t)((kp.local_rows + 7) >> 3);
  const size_t max_frames = std::max<size_t>(1, (size_t)0x7FFFFFFF / std::max<size_t>(1, n_tiles) - 1);
  const int chunk = (int)std::max<size_t>(
      1, std::min<size_t>(std::min<size_t>((size_t)kp.nframes, max_frames), c->lbuf_cap / per_frame));
  const size_t need = per_frame * (size_t)chunk;
  if (need > c->lbuf_bytes) {
    FreeDev(c->d_lbuf);
    c->d_lbuf = nullptr;
    c->lbuf_bytes = 0;
    HIP_OK(hipMalloc(&c->d_lbuf, need));
    c->lbuf_bytes = need;
  }
  kp.lbuf = c->d_lbuf;
  kp.trav_frac16 = c->trav_frac16;
  HIP_OK(hipMemsetAsync(c->d_stats, 0, sizeof(unsigned long long) * srt::ST_TOTAL, c->stream));
  const int out_frames = kp.frame_first + kp.nframes - 1;
  const int nchunks = (kp.nframes + chunk - 1) / chunk;
  if (nchunks > c->batch_ctr_cap) {
    FreeDev(c->d_batch_ctr);
    c->d_batch_ctr = nullptr;
    c->batch_ctr_cap = 0;
    HIP_OK(hipMalloc(&c->d_batch_ctr, sizeof(unsigned long long) * (size_t)nchunks));
    c->batch_ctr_cap = nchunks;
  }
  HIP_OK(hipMemsetAsync(c->d_batch_ctr, 0, sizeof(unsigned long long) * (size_t)nchunks, c->stream));
  while ((int)c->ev.size() < 2 * nchunks) {
    hipEvent_t e;
    HIP_OK(hipEventCreate(&e));
    c->ev.push_back(e);
  }
  c->ev_used = 0;
  for (int f0 = 0; f0 < kp.nframes; f0 += chunk) {
    srt::KParams kc = kp;
    kc.frame_first = kp.frame_first + f0;
    kc.nframes = std::min(chunk, kp.nframes - f0);
    kc.write_output = (f0 + chunk >= kp.nframes) ? kp.write_output : 0;
    kc.batch_ctr = c->d_batch_ctr + f0 / chunk;
    int rc;
    HIP_OK(hipEventRecord(c->ev[c->ev_used], c->stream));
    // LDS mode: packed entries (lds_ok); global-scene mode: packed when indices fit 24 bits
    const bool pack = c->lds_ok;
    if (count && ldsm) rc = block == 512 ? LaunchSamples<true, true, true, 512>(c, kc, lds)
                                         : LaunchSamples<true, true, true, 1024>(c, kc, lds);
    else if (count) rc = pack ? LaunchSamples<true, false, true, 256>(c, kc, lds)
                              : LaunchSamples<true, false, false, 256>(c, kc, lds);
    else if (ldsm) rc = block == 512 ? LaunchSamples<false, true, true, 512>(c, kc, lds)
                                     : LaunchSamples<false, true, true, 1024>(c, kc, lds);
    else rc = pack ? LaunchSamples<false, false, true, 256>(c, kc, lds) : LaunchSamples<false, false, false, 256>(c, kc, lds);
    if (rc) return rc;
    HIP_OK(hipEventRecord(c->ev[c->ev_used + 1], c->stream));
    c->ev_used += 2;
    hipLaunchKernelGGL(srt::accumulate_kernel, pgrid, dim3(256), 0, c->stream, kc, out_frames);
    HIP_OK(hipGetLastError());
  }
  if (count) {
    unsigned long long s[srt::ST_N];
    HIP_OK(hipMemcpyAsync(s, c->d_stats, sizeof(s), hipMemcpyDeviceToHost, c->stream));
    HIP_OK(hipStreamSynchronize(c->stream));
    c->stats.rays += s[srt::ST_RAYS];
    c->stats.nodes += s[srt::ST_NODES];
    c->stats.tris += s[srt::ST_TRIS];
    c->stats.rng_u += s[srt::ST_RNGU];
    c->stats.rng_sq += s[srt::ST_RNGSQ];
    c->stats.light_reads += s[srt::ST_LIGHTS];
    c->stats.mat_reads += s[srt::ST_MATS];
    c->stats.samples += s[srt::ST_SAMPLES];
    c->stats.stack_overflow += s[srt::ST_OVERFLOW];
    c->stats.max_stack = std::max<uint64_t>(c->stats.max_stack, s[srt::ST_MAXSTACK]);
  }
  return SRT_OK;
}

// Depth of each BVH (root depth 0) and index validation.
int ValidateNodes(const srt_bvh_node* nodes, uint32_t n_nodes, uint32_t n_tris, const srt_bvh_record* bvhs,
                  uint32_t n_bvhs, int* max_depth) {
  *max_depth = 0;
  std::vector<std::pair<uint32_t, int>> st;
  std::vector<uint8_t> seen(n_nodes, 0);
  for (uint32_t b = 0; b < n_bvhs; ++b) {
    if (bvhs[b].first_index >= n_nodes) {
      srt::SetError("BVH first_index out of range");
      return SRT_ERR_INVALID;
    }
    st.push_back({bvhs[b].first_index, 0});
    while (!st.empty()) {
      auto [i, d] = st.back();
      st.pop_back();
      *max_depth = std::max(*max_depth, d);
      const srt_bvh_node& n = nodes[i];
      if (n.prim_count > 0) {
        if ((uint64_t)n.first_child_or_prim_index + n.prim_count > n_tris) {
          srt::SetError("BVH leaf references triangles out of range");
          return SRT_ERR_INVALID;
        }
      } else {
        if ((uint64_t)n.first_child_or_prim_index + 1 >= n_nodes || seen[i]) {
          srt::SetError("BVH internal node references children out of range (or a cycle)");
          return SRT_ERR_INVALID;
        }
        seen[i] = 1;
        st.push_back({n.first_child_or_prim_index, d + 1});
        st.push_back({n.first_child_or_prim_index + 1, d + 1});
      }
    }
    std::fill(seen.begin(), seen.end(), 0);
  }
  return SRT_OK;
}

}  // namespace

// ===========================================================================
// C ABI (context part)
// ===========================================================================
extern "C" {

const char* srt_last_error(void) { return srt::LastError(); }
int srt_abi_version(void) { return SRT_ABI_VERSION; }

int srt_create(int device, void* stream, srt_context** out) {
  if (!out) return SRT_ERR_INVALID;
  HIP_OK(hipSetDevice(device));
  auto* c = new srt_context();
  c->device = device;
  if (const char* e = std::getenv("SRT_FORCE_GLOBAL_SCENE")) c->force_global = e[0] == '1';
  if (const char* e = std::getenv("SRT_SAMPLE_BUFFER_MB")) c->lbuf_cap = (size_t)std::max(1L, std::atol(e)) << 20;
  if (const char* e = std::getenv("SRT_SAMPLE_BUFFER_KB")) c->lbuf_cap = (size_t)std::max(1L, std::atol(e)) << 10;
  if (const char* e = std::getenv("SRT_LDS_BLOCK")) c->lds_block = std::atoi(e) == 512 ? 512 : 1024;
  if (const char* e = std::getenv("SRT_TRAV_FRAC16")) c->trav_frac16 = std::max(0, std::min(16, std::atoi(e)));
  {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
      c->num_cus = prop.multiProcessorCount;
  }
  if (stream) {
    c->stream = static_cast<hipStream_t>(stream);
  } else {
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
      delete c;
      srt::SetError(std::string("hipStreamCreate: ") + hipGetErrorString(e));
      return SRT_ERR_HIP;
    }
    c->own_stream = true;
  }
  if (hipMalloc(&c->d_stats, sizeof(unsigned long long) * srt::ST_TOTAL) != hipSuccess) {
    if (c->own_stream) (void)hipStreamDestroy(c->stream);
    delete c;
    srt::SetError("hipMalloc(stats) failed");
    return SRT_ERR_HIP;
  }
  *out = c;
  return SRT_OK;
}

int srt_destroy(srt_context* c) {
  if (!c) return SRT_ERR_INVALID;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  FreeDev(c->d_nodes); FreeDev(c->d_tris); FreeDev(c->d_mats); FreeDev(c->d_bvhs); FreeDev(c->d_lights);
  FreeDev(c->d_noise_xy); FreeDev(c->d_noise_u); FreeDev(c->d_stats); FreeDev(c->d_lbuf); FreeDev(c->d_gstack);
  FreeDev(c->d_batch_ctr);
  for (hipEvent_t e : c->ev) (void)hipEventDestroy(e);
  if (!c->images_external) { FreeDev(c->d_accum); FreeDev(c->d_out); }
  if (c->own_stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return SRT_OK;
}

void* srt_stream(srt_context* c) { return c ? static_cast<void*>(c->stream) : nullptr; }

int srt_set_bool(srt_context* c, const char* name, int v) {
  if (!c || !name) return SRT_ERR_INVALID;
  const std::string n(name);
  if (n == "resetAccumBuffer") c->reset = v ? 1 : 0;
  else if (n == "showModel") c->show_model = v ? 1 : 0;
  else return SRT_ERR_NOT_FOUND;
  return SRT_OK;
}

int srt_set_int(srt_context* c, const char* name, int v) {
  if (!c || !name) return SRT_ERR_INVALID;
  const std::string n(name);
  if (n == "Width") c->W = v;
  else if (n == "Height") c->H = v;
  else if (n == "accumFrames") c->accum_frames = v;
  else if (n == "lightCount") c->light_count = v;
  else if (n == "maxDepth") c->max_depth = v;
  else if (n == "resetAccumBuffer" || n == "showModel") return srt_set_bool(c, name, v);
  else if (n == "bvh_count") c->bvh_count = (uint32_t)v;
  else return SRT_ERR_NOT_FOUND;
  return SRT_OK;
}

int srt_set_uint(srt_context* c, const char* name, uint32_t v) {
  if (!c || !name) return SRT_ERR_INVALID;
  if (std::string(name) == "bvh_count") {
    c->bvh_count = v;
    return SRT_OK;
  }
  return srt_set_int(c, name, (int)v);
}

int srt_set_float(srt_context* c, const char* name, float v) {
  if (!c || !name) return SRT_ERR_INVALID;
  (void)v;
  return SRT_ERR_NOT_FOUND;  // the kernel declares no float uniforms
}

int srt_set_vec3(srt_context* c, const char* name, float x, float y, float z) {
  if (!c || !name) return SRT_ERR_INVALID;
  const std::string n(name);
  float* dst = nullptr;
  if (n == "cameraOrigin") dst = c->cam_origin;
  else if (n == "cameraDirection") dst = c->cam_dir;
  else if (n == "cameraUp") dst = c->cam_up;
  else if (n == "cameraRight") dst = c->cam_right;
  else return SRT_ERR_NOT_FOUND;
  dst[0] = x; dst[1] = y; dst[2] = z;
  return SRT_OK;
}

int srt_set_tiling(srt_context* c, int rank, int nranks, int band_rows) {
  if (!c || nranks < 1 || rank < 0 || rank >= nranks || band_rows < 1) return SRT_ERR_INVALID;
  c->rank = rank;
  c->nranks = nranks;
  c->band_rows = band_rows;
  return SRT_OK;
}

int srt_local_rows(srt_context* c) { return c ? LocalRows(c, c->H) : -1; }

int srt_dispatch(srt_context* c, uint32_t gx, uint32_t gy) {
  if (!c) return SRT_ERR_INVALID;
  HIP_OK(hipSetDevice(c->device));
  srt::KParams kp;
  int rc = FillParams(c, &kp, true);
  if (rc) return rc;
  kp.ext_w = (int)std::min<uint64_t>((uint64_t)gx * 8, (uint64_t)c->W);
  kp.ext_h = (int)std::min<uint64_t>((uint64_t)gy * 8, (uint64_t)c->H);
  kp.frame_first = c->accum_frames;
  kp.nframes = 1;
  kp.write_output = 1;
  kp.reset = c->reset;
  if (!kp.reset && c->accum_frames == 0) {
    srt::SetError("accumFrames must be >= 1 for a sampling dispatch (the reference increments it first)");
    return SRT_ERR_STATE;
  }
  return Launch(c, kp, false);
}

int srt_render_frames(srt_context* c, int frame_first, int nframes, int write_output, int count) {
  if (!c || nframes < 0 || frame_first < 1) return SRT_ERR_INVALID;
  HIP_OK(hipSetDevice(c->device));
  srt::KParams kp;
  int rc = FillParams(c, &kp, true);
  if (rc) return rc;
  if (nframes == 0) return SRT_OK;
  kp.frame_first = frame_first;
  kp.nframes = nframes;
  kp.write_output = write_output ? 1 : 0;
  kp.reset = 0;
  return Launch(c, kp, count != 0);
}

int srt_finish(srt_context* c) {
  if (!c) return SRT_ERR_INVALID;
  HIP_OK(hipStreamSynchronize(c->stream));
  return SRT_OK;
}

// Diagnostic: shader-clock cycles per phase of the last render (SRT_PHASE_TIMING builds only; zeros otherwise).
// out[0..3]: refill / traversal / shading cycles, outer iterations; out[4..9]: traversal
// iterations and summed lane counts (working, traversing, at a leaf, at an internal node),
// lanes shading (summed over outer iterations).
// out[10..57]: per sub-step k (3 values): lanes taking it, waves executing it, lanes popping after it.
extern "C" int srt_debug_phase_cycles(srt_context* c, unsigned long long out[58]) {
  if (!c || !out) return SRT_ERR_INVALID;
  HIP_OK(hipMemcpyAsync(out, c->d_stats + srt::ST_CYC_REFILL, 58 * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                        c->stream));
  HIP_OK(hipStreamSynchronize(c->stream));
  return SRT_OK;
}

int srt_last_kernel_ms(srt_context* c, float* ms) {
  if (!c || !ms) return SRT_ERR_INVALID;
  *ms = 0.0f;
  for (int i = 0; i + 1 < c->ev_used; i += 2) {
    HIP_OK(hipEventSynchronize(c->ev[i + 1]));
    float t = 0.0f;
    HIP_OK(hipEventElapsedTime(&t, c->ev[i], c->ev[i + 1]));
    *ms += t;
  }
  return SRT_OK;
}

int srt_get_stats(srt_context* c, srt_stats* out) {
  if (!c || !out) return SRT_ERR_INVALID;
  *out = c->stats;
  return SRT_OK;
}

int srt_reset_stats(srt_context* c) {
  if (!c) return SRT_ERR_INVALID;
  c->stats = srt_stats{};
  return SRT_OK;
}

int srt_upload_scene(srt_context* c, const srt_bvh_record* bvhs, uint32_t n_bvhs, const srt_bvh_node* nodes,
                     uint32_t n_nodes, const srt_material_obj* mats, const float* tex_albedo, uint32_t n_mats,
                     const srt_triangle* tris, uint32_t n_tris, const srt_vertex* verts, uint32_t n_verts) {
  if (!c || (n_bvhs && !bvhs) || (n_nodes && !nodes) || (n_mats && !mats) || (n_tris && !tris) ||
      (n_verts && !verts))
    return SRT_ERR_INVALID;
  if (n_nodes == 0 || n_bvhs == 0) {
    srt::SetError("scene needs at least one BVH and one node");
    return SRT_ERR_INVALID;
  }
  int depth = 0;
  int rc = ValidateNodes(nodes, n_nodes, n_tris, bvhs, n_bvhs, &depth);
  if (rc) return rc;
  HIP_OK(hipSetDevice(c->device));
  // nodes: 32-B records behind a 32-B pad so sibling pairs are 64-B aligned
  std::vector<float4> hn(2 * ((size_t)n_nodes + 1));
  hn[0] = hn[1] = make_float4(0, 0, 0, 0);
  for (uint32_t i = 0; i < n_nodes; ++i) {
    const srt_bvh_node& n = nodes[i];
    float w0, w1;
    std::memcpy(&w0, &n.first_child_or_prim_index, 4);
    std::memcpy(&w1, &n.prim_count, 4);
    hn[2 * (size_t)i + 2] = make_float4(n.min_bounds[0], n.min_bounds[1], n.min_bounds[2], w0);
    hn[2 * (size_t)i + 3] = make_float4(n.max_bounds[0], n.max_bounds[1], n.max_bounds[2], w1);
  }
  // materials -> shading materials (raytrace_utils.glsl:140-175); one zero
  // record appended for out-of-range material indices (OOB SSBO reads = 0)
  std::vector<float4> hm(2 * ((size_t)n_mats + 1), make_float4(0, 0, 0, 0));
  for (uint32_t i = 0; i <= n_mats; ++i) {
    srt_material_obj m{};
    if (i < n_mats) m = mats[i];
    float alb[3] = {m.diffuse[0], m.diffuse[1], m.diffuse[2]};
    if (m.use_texture) {
      for (int k = 0; k < 3; ++k) alb[k] = tex_albedo ? tex_albedo[3 * (size_t)i + k] : 0.0f;
    }
    const float rough = 1.0f / (m.specular_ex + 0.0000001f);
    hm[2 * (size_t)i] = make_float4(alb[0], alb[1], alb[2], rough);
    hm[2 * (size_t)i + 1] = make_float4(m.specular[0], m.specular[1], m.specular[2], 0.0f);
  }
  // triangles: v0, e1 = v1 - v0, e2 = v2 - v0, material
  // kTriPad zero records past the end: a multi-triangle leaf step may read (and discard) them
  std::vector<float4> ht(3 * ((size_t)n_tris + srt::kTriPad), make_float4(0, 0, 0, 0));
  auto vert = [&](uint32_t i, int k) -> float { return i < n_verts ? verts[i].vertex[k] : 0.0f; };
  for (uint32_t t = 0; t < n_tris; ++t) {
    const srt_triangle& tr = tris[t];
    float v0[3], e1[3], e2[3];
    for (int k = 0; k < 3; ++k) {
      v0[k] = vert(tr.v0_idx, k);
      e1[k] = vert(tr.v1_idx, k) - v0[k];
      e2[k] = vert(tr.v2_idx, k) - v0[k];
    }
    const uint32_t mi = tr.material_idx < n_mats ? tr.material_idx : n_mats;
    float mf;
    std::memcpy(&mf, &mi, 4);
    ht[3 * (size_t)t + 0] = make_float4(v0[0], v0[1], v0[2], e1[0]);
    ht[3 * (size_t)t + 1] = make_float4(e1[1], e1[2], e2[0], e2[1]);
    ht[3 * (size_t)t + 2] = make_float4(e2[2], mf, 0.0f, 0.0f);
  }
  FreeDev(c->d_nodes); FreeDev(c->d_mats); FreeDev(c->d_tris);
  c->d_nodes = nullptr; c->d_mats = nullptr; c->d_tris = nullptr;
  c->scene_ok = false;
  HIP_OK(hipMalloc(&c->d_nodes, hn.size() * sizeof(float4)));
  HIP_OK(hipMalloc(&c->d_mats, hm.size() * sizeof(float4)));
  HIP_OK(hipMalloc(&c->d_tris, ht.size() * sizeof(float4)));
  HIP_OK(hipMemcpyAsync(c->d_nodes, hn.data(), hn.size() * sizeof(float4), hipMemcpyHostToDevice, c->stream));
  HIP_OK(hipMemcpyAsync(c->d_mats, hm.data(), hm.size() * sizeof(float4), hipMemcpyHostToDevice, c->stream));
  HIP_OK(hipMemcpyAsync(c->d_tris, ht.data(), ht.size() * sizeof(float4), hipMemcpyHostToDevice, c->stream));
  HIP_OK(hipStreamSynchronize(c->stream));
  c->h_bvhs.assign(bvhs, bvhs + n_bvhs);
  c->bvhs_dirty = true;
  c->n_nodes = n_nodes;
  c->n_tris = n_tris;
  c->n_mats = n_mats;
  c->stack_entries = depth + 1;
  uint32_t max_leaf = 0;
  for (uint32_t i = 0; i < n_nodes; ++i) max_leaf = std::max(max_leaf, nodes[i].prim_count);
  c->lds_ok = n_tris < (1u << 24) && n_nodes < (1u << 24) && max_leaf < 256;
  c->scene_ok = true;
  if (c->bvh_count == 0) c->bvh_count = n_bvhs;
  // the zero records beyond n_bvhs traverse from node 0 with a zero ray
  // (raytrace_compute.glsl:144-147 reading bvhs[i] out of bounds)
  return SRT_OK;
}

int srt_update_model_matrix(srt_context* c, uint32_t index, const float frame[16]) {
  if (!c || !frame) return SRT_ERR_INVALID;
  if (index >= c->h_bvhs.size()) {
    srt::SetError("UpdateModelMatrix: index out of range");  // std::vector::at throws
    return SRT_ERR_INVALID;
  }
  std::memcpy(c->h_bvhs[index].frame, frame, sizeof(float) * 16);
  c->bvhs_dirty = true;
  return SRT_OK;  // pushed to the device at the next launch (EnsureBvhs)
}

int srt_set_lights(srt_context* c, const srt_light* lights, uint32_t n) {
  if (!c || (n && !lights)) return SRT_ERR_INVALID;
  c->h_lights.assign(lights, lights + n);
  c->lights_dirty = true;
  return SRT_OK;
}

int srt_set_noise(srt_context* c, const float* noise_rgb, const float* noise_u_rgb, size_t texels) {
  if (!c || !noise_rgb || !noise_u_rgb || texels == 0) return SRT_ERR_INVALID;
  HIP_OK(hipSetDevice(c->device));
  std::vector<float2> xy(texels);
  std::vector<float> u(texels);
  for (size_t i = 0; i < texels; ++i) {
    xy[i] = make_float2(noise_rgb[3 * i], noise_rgb[3 * i + 1]);
    u[i] = noise_u_rgb[3 * i];
  }
  if (texels != c->noise_texels) {
    FreeDev(c->d_noise_xy); FreeDev(c->d_noise_u);
    c->d_noise_xy = nullptr; c->d_noise_u = nullptr; c->noise_texels = 0;
    HIP_OK(hipMalloc(&c->d_noise_xy, texels * sizeof(float2)));
    HIP_OK(hipMalloc(&c->d_noise_u, texels * sizeof(float)));
  }
  HIP_OK(hipMemcpyAsync(c->d_noise_xy, xy.data(), texels * sizeof(float2), hipMemcpyHostToDevice, c->stream));
  HIP_OK(hipMemcpyAsync(c->d_noise_u, u.data(), texels * sizeof(float), hipMemcpyHostToDevice, c->stream));
  HIP_OK(hipStreamSynchronize(c->stream));
  c->noise_texels = texels;
  return SRT_OK;
}

int srt_alloc_images(srt_context* c) {
  if (!c || c->W <= 0 || c->H <= 0) return SRT_ERR_STATE;
  HIP_OK(hipSetDevice(c->device));
  const int rows = LocalRows(c, c->H);
  const size_t px = (size_t)c->W * (size_t)std::max(rows, 1);
  if (!c->images_external) { FreeDev(c->d_accum); FreeDev(c->d_out); }
  c->images_external = false;
  c->d_accum = nullptr; c->d_out = nullptr;
  HIP_OK(hipMalloc(&c->d_accum, px * sizeof(float4)));
  HIP_OK(hipMalloc(&c->d_out, px * sizeof(uint32_t)));
  HIP_OK(hipMemsetAsync(c->d_accum, 0, px * sizeof(float4), c->stream));
  HIP_OK(hipMemsetAsync(c->d_out, 0, px * sizeof(uint32_t), c->stream));
  HIP_OK(hipStreamSynchronize(c->stream));
  c->img_w = c->W;
  c->img_rows = rows;
  return SRT_OK;
}

int srt_read_accum(srt_context* c, float* host, size_t bytes) {
  if (!c || !host || !c->d_accum) return SRT_ERR_INVALID;
  const size_t need = (size_t)c->img_w * c->img_rows * sizeof(float4);
  if (bytes < need) return SRT_ERR_INVALID;
  HIP_OK(hipMemcpyAsync(host, c->d_accum, need, hipMemcpyDeviceToHost, c->stream));
  HIP_OK(hipStreamSynchronize(c->stream));
  return SRT_OK;
}

int srt_write_accum(srt_context* c, const float* host, size_t bytes) {
  if (!c || !host || !c->d_accum) return SRT_ERR_INVALID;
  const size_t need = (size_t)c->img_w * c->img_rows * sizeof(float4);
  if (bytes < need) return SRT_ERR_INVALID;
  HIP_OK(hipMemcpyAsync(c->d_accum, host, need, hipMemcpyHostToDevice, c->stream));
  HIP_OK(hipStreamSynchronize(c->stream));
  return SRT_OK;
}

int srt_read_output(srt_context* c, uint8_t* host, size_t bytes) {
  if (!c || !host || !c->d_out) return SRT_ERR_INVALID;
  const size_t need = (size_t)c->img_w * c->img_rows * sizeof(uint32_t);
  if (bytes < need) return SRT_ERR_INVALID;
  HIP_OK(hipMemcpyAsync(host, c->d_out, need, hipMemcpyDeviceToHost, c->stream));
  HIP_OK(hipStreamSynchronize(c->stream));
  return SRT_OK;
}

int srt_write_output(srt_context* c, const char* path, int flip_y) {
  if (!c || !path || !c->d_out || c->img_w <= 0 || c->img_rows <= 0) return SRT_ERR_INVALID;
  std::vector<uint8_t> px((size_t)c->img_w * c->img_rows * 4);
  const int rc = srt_read_output(c, px.data(), px.size());
  if (rc) return rc;
  return srt_image_write(path, px.data(), c->img_w, c->img_rows, flip_y);
}

int srt_set_image_buffers(srt_context* c, void* accum_dev, void* out_dev) {
  if (!c || !accum_dev || !out_dev || c->W <= 0 || c->H <= 0) return SRT_ERR_INVALID;
  if (!c->images_external) { FreeDev(c->d_accum); FreeDev(c->d_out); }
  c->d_accum = static_cast<float4*>(accum_dev);
  c->d_out = static_cast<uint32_t*>(out_dev);
  c->images_external = true;
  c->img_w = c->W;
  c->img_rows = LocalRows(c, c->H);
  return SRT_OK;
}

int srt_assemble_bands(srt_context* c, const void* gathered, int nranks, int rows_pad, int band_rows, int frames,
                       void* accum_full, void* out_full) {
  if (!c || !gathered || nranks < 1 || rows_pad < 1 || band_rows < 1 || frames < 1 || c->W <= 0 || c->H <= 0)
    return SRT_ERR_INVALID;
  HIP_OK(hipSetDevice(c->device));
  const size_t n = (size_t)c->W * (size_t)c->H;
  hipLaunchKernelGGL(srt::assemble_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c->stream,
                     static_cast<const float4*>(gathered), nranks, rows_pad, c->W, c->H, band_rows, frames,
                     static_cast<float4*>(accum_full), static_cast<uint32_t*>(out_full));
  HIP_OK(hipGetLastError());
  return SRT_OK;
}

int srt_image_pointers(srt_context* c, void** accum_dev, void** out_dev) {
  if (!c) return SRT_ERR_INVALID;
  if (accum_dev) *accum_dev = c->d_accum;
  if (out_dev) *out_dev = c->d_out;
  return SRT_OK;
}

int srt_trace_closest(srt_context* c, const srt_ray* rays, uint32_t n, uint32_t* hits, float* t_out) {
  if (!c || (n && (!rays || !hits || !t_out))) return SRT_ERR_INVALID;
  if (!c->scene_ok) { srt::SetError("no scene uploaded"); return SRT_ERR_STATE; }
  if (n == 0) return SRT_OK;
  HIP_OK(hipSetDevice(c->device));
  srt::KParams kp;
  std::memset(&kp, 0, sizeof kp);
  int rc = EnsureBvhs(c);
  if (rc) return rc;
  kp.nodes = c->d_nodes;
  kp.tris = c->d_tris;
  kp.bvhs = c->d_bvhs;
  kp.bvh_count = c->bvh_count;
  kp.stack_entries = c->stack_entries;
  kp.stats = c->d_stats;
  srt_ray* d_rays = nullptr;
  uint32_t* d_hits = nullptr;
  float* d_t = nullptr;
  HIP_OK(hipMalloc(&d_rays, sizeof(srt_ray) * n));
  HIP_OK(hipMalloc(&d_hits, sizeof(uint32_t) * n));
  HIP_OK(hipMalloc(&d_t, sizeof(float) * n));
  HIP_OK(hipMemcpyAsync(d_rays, rays, sizeof(srt_ray) * n, hipMemcpyHostToDevice, c->stream));
  HIP_OK(hipMemsetAsync(c->d_stats, 0, sizeof(unsigned long long) * srt::ST_N, c->stream));
  const int block = 256;
  const size_t lds = (size_t)block * 3 * sizeof(uint32_t) * (size_t)kp.stack_entries;
  hipLaunchKernelGGL(srt::closest_kernel, dim3((n + block - 1) / block), dim3(block), lds, c->stream, kp, d_rays, n,
                     d_hits, d_t);
  HIP_OK(hipGetLastError());
  unsigned long long s[srt::ST_N];
  HIP_OK(hipMemcpyAsync(hits, d_hits, sizeof(uint32_t) * n, hipMemcpyDeviceToHost, c->stream));
  HIP_OK(hipMemcpyAsync(t_out, d_t, sizeof(float) * n, hipMemcpyDeviceToHost, c->stream));
  HIP_OK(hipMemcpyAsync(s, c->d_stats, sizeof(s), hipMemcpyDeviceToHost, c->stream));
  HIP_OK(hipStreamSynchronize(c->stream));
  c->stats.rays += n;
  c->stats.nodes += s[srt::ST_NODES];
  c->stats.tris += s[srt::ST_TRIS];
  (void)hipFree(d_rays);
  (void)hipFree(d_hits);
  (void)hipFree(d_t);
  return SRT_OK;
}

}  // extern "C"
