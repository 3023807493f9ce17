// traversal.hpp -- BVH traversal, order-exact: slab and Moller-Trumbore tests, scene
// access (LDS copy or HBM), traversal stacks, the flat closest-hit walk and the
// resumable step machine of sample_kernel.
#pragma once

#include "device_common.hpp"

namespace srt {
using namespace dev;

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

// box_ok(box_t(...), dist) with one compare fewer: `b` receives the entry
// distance IntersectsBox returns whenever the result is true.  Equivalence:
// for tn <= tf, b = sel and `sel < dist` already rejects sel = +inf, so only
// -inf needs its own test; otherwise (tn > tf, or a NaN bound) IntersectsBox
// returns +inf, which no `< dist` accepts.
__device__ __forceinline__ bool box_test(f3 o, f3 inv, float4 lo, float4 hi, float dist, float& b) {
  const float t0x = (lo.x - o.x) * inv.x, t0y = (lo.y - o.y) * inv.y, t0z = (lo.z - o.z) * inv.z;
  const float t1x = (hi.x - o.x) * inv.x, t1y = (hi.y - o.y) * inv.y, t1z = (hi.z - o.z) * inv.z;
  const float tn = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(t0x, t1x), __builtin_fminf(t0y, t1y)),
                                   __builtin_fminf(t0z, t1z));
  const float tf = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(t0x, t1x), __builtin_fmaxf(t0y, t1y)),
                                   __builtin_fmaxf(t0z, t1z));
  b = (tn >= 0.0f) ? tn : tf;
  return (tn <= tf) & (b < dist) & (b != -__builtin_inff());
}

// LDS byte offsets are 32-bit: keep the address arithmetic in 32 bits.
__device__ __forceinline__ float4 lds4(uint32_t byte_off) {
  return *reinterpret_cast<const float4*>(reinterpret_cast<const char*>(g_smem) + byte_off);
}
// LDS mode stores the node array's 64-B sibling-pair blocks (float4 4b .. 4b + 3)
// at a stride of kNodeBlkF4 float4.  A ds_read_b128 serves 16 lanes per LDS
// cycle from a 256-B bank row (16 slots of 16 B); with 64-B blocks every lane
// reading field k of some pair lands on one of only 4 slots, (4 * pair + k) mod 16,
// so random pairs collide ~4 ways.  An 80-B stride spreads them over all 16.
#ifndef SRT_NODE_PAD
#define SRT_NODE_PAD 1
#endif
constexpr uint32_t kNodeBlkF4 = SRT_NODE_PAD ? 5u : 4u;
__device__ __forceinline__ uint32_t node_lds_f4(uint32_t i) { return (i >> 2) * kNodeBlkF4 + (i & 3u); }
template <bool LDSM>
__device__ __forceinline__ float4 node4(const KParams& kp, uint32_t i) {
  if constexpr (LDSM) return lds4(node_lds_f4(i) << 4);
  else return kp.nodes[i];
}
// The child pair whose first slot is `ref0` (odd: the pair's block is 64-B
// aligned; LDS mode is only chosen for node arrays where every pair is).
template <bool LDSM>
__device__ __forceinline__ void node_pair(const KParams& kp, uint32_t ref0, float4& l0, float4& h0, float4& l1,
                                          float4& h1) {
  if constexpr (LDSM) {
    // block (ref0 + 1) / 2 = ref0 / 2 + 1 (ref0 is odd), of 16 * kNodeBlkF4 bytes; ref0 < 2^24 in LDS
    // mode, so a v_mad_u32_u24 (a 32-bit multiply is a quarter-rate v_mul_lo_u32), and the
    // compiler sees the 16-B alignment that lets it use ds_read_b128
    const uint32_t b = __umul24(ref0 >> 1, kNodeBlkF4 * 16u) + kNodeBlkF4 * 16u;
    l0 = lds4(b);
    h0 = lds4(b + 16u);
    l1 = lds4(b + 32u);
    h1 = lds4(b + 48u);
  } else {
    const uint32_t pi = 2 * ref0 + 2;
    l0 = kp.nodes[pi];
    h0 = kp.nodes[pi + 1];
    l1 = kp.nodes[pi + 2];
    h1 = kp.nodes[pi + 3];
  }
}
// the records of triangle `i` onwards (3 float4 per triangle)
template <bool LDSM>
__device__ __forceinline__ const float4* tri_ptr(const KParams& kp, uint32_t i) {
  if constexpr (LDSM)  // i < 2^24 in LDS mode: one v_mad_u32_u24 (a 32-bit mul + add becomes a slow v_mad_u64_u32)
    return reinterpret_cast<const float4*>(reinterpret_cast<const char*>(g_smem) + ((uint32_t)kp.nodes_lds_f4 * 16u +
                                                                                  __umul24(i, 48u)));
  else return kp.tris + 3 * (size_t)i;
}
template <bool LDSM>
__device__ __forceinline__ float4 tri4(const KParams& kp, uint32_t i) {
  if constexpr (LDSM) return lds4(((uint32_t)kp.nodes_lds_f4 + i) << 4);
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
// tools/rcp_exhaustive.hip, tests/test_gpu_exhaustive_math.py); |a| >= 2^126, inf and NaN
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
      const uint32_t pi = 2 * (ref | kp.ref_or) + 2;
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

struct Trav {
  f3 o, d, inv;       // ray in the current BVH's frame
  float dist;         // running intersection_distance
  uint32_t ref, cnt;  // current node: leaf (cnt > 0): first triangle + remaining; internal (cnt == 0):
                      // first child; nothing current: cnt == kNoneCnt (ref is then unused)
  uint32_t hit;       // best triangle so far (0xFFFFFFFF: none)
  uint32_t bi;        // current BVH
  int sp;
  int lo;             // global-scene mode: entries [lo, sp) are in the LDS ring, [0, lo) in HBM
  bool active;        // still traversing
  bool start;         // next step sets up BVH `bi`
};

constexpr uint32_t kNoneRef = 0xFFFFFFFFu;
// Trav::cnt of "nothing current, pop next": one compare tells the three states
// apart (leaf: (int)cnt > 0; internal: cnt == 0; none: cnt == kNoneCnt), and
// ref needs no update when a lane runs out of nodes.  Leaf counts are < 2^31
// (srt_upload_scene validates it).
constexpr uint32_t kNoneCnt = 0xFFFFFFFFu;
// Wavefront mode's flagged node copy: the count of a treelet root (an internal node at the treelet
// depth), whose child index holds the treelet's id instead (wavefront.hpp; leaves then hold < 255).
constexpr uint32_t kTreeletCnt = 255u;
__device__ __forceinline__ bool trav_at_leaf(uint32_t cnt) { return (int)cnt > 0; }
#ifndef SRT_LEAF_TRIS
#define SRT_LEAF_TRIS 2
#endif
constexpr int kLeafTris = SRT_LEAF_TRIS;  // triangles tested per leaf step (global-scene mode)
// LDS mode tests three triangles per leaf step, over 11 sub-steps per iteration
// that start with two internal steps (Rubik 1080p: 5,976 -> 6,106 Mrays/s with
// ILIL..., 6,150-6,157 with IIL...; 4 per step 5,451-5,493)
#ifndef SRT_LEAF_TRIS_LDS
#define SRT_LEAF_TRIS_LDS 3
#endif
template <bool LDSM>
constexpr int kLeafTrisM = LDSM ? SRT_LEAF_TRIS_LDS : kLeafTris;
// Sub-steps of one traversal iteration: 'I' expands an internal node, 'L'
// tests a leaf's next triangles; each is followed by a pop if nothing is current.
// (global-scene mode's IL schedule, the one trees past 600 MB take: internal
// steps first, as in LDS mode; C5 582 -> 592 Mrays/s with two, 594 -> 601 with
// three)
#ifndef SRT_STEP_PATTERN
#define SRT_STEP_PATTERN "IIILILILILILIL"
#endif
#ifndef SRT_STEP_PATTERN_LDS
#define SRT_STEP_PATTERN_LDS "IILILILILIL"
#endif
constexpr char kStepPattern[] = SRT_STEP_PATTERN;         // global-scene mode, IL schedule
constexpr char kStepPatternLds[] = SRT_STEP_PATTERN_LDS;  // LDS mode
template <bool LDSM>
constexpr char step_kind(int k) { return LDSM ? kStepPatternLds[k] : kStepPattern[k]; }
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
// sphere_kernel: batches per claim (its batches are cheap: the launch counter's atomic rate, ~88 M claims/s,
// not the tail, limits it; C2 on one box, kernel ms, with a tail window of 1 claim per wave: 4 per claim
// 3.45, 8 3.17, 16 3.47; profiles/r04_experiments/claim_contention.txt)
#ifndef SRT_CLAIM_SPH
#define SRT_CLAIM_SPH 8
#endif
constexpr int kClaimSph = SRT_CLAIM_SPH;
static_assert((kShortStack & (kShortStack - 1)) == 0, "kShortStack must be a power of two");
constexpr int kTriPad = 3;                // zero records past the triangle array (>= kLeafTris - 1)
constexpr uint32_t kNodePad = 2;          // zero node records past the array: the speculative next-pair read
// Internal steps expand the right child in the same step when its child pair
// is the next pair of the array (trav_internal; pathtrace.hip LayoutNodes).
#ifndef SRT_SPINE
#define SRT_SPINE 1
#endif
// Global-scene mode only: it waits on memory; the LDS-resident kernel is bound by
// VALU issue, and the second level's box tests cost it more than the LDS latency
// they hide (5,676 -> 5,239 Mrays/s on Rubik 1080p).
template <bool LDSM>
constexpr bool kSpine = SRT_SPINE && !LDSM;
#ifndef SRT_MASK_LEAF2
#define SRT_MASK_LEAF2 0
#endif
// Global-scene mode, fused schedule (trav_fused): sub-steps per traversal iteration
#ifndef SRT_GLOBAL_FUSED
#define SRT_GLOBAL_FUSED 8
#endif
constexpr int kFusedSteps = SRT_GLOBAL_FUSED;
static_assert(kLeafTris >= 1 && kLeafTris - 1 <= kTriPad, "kLeafTris");
static_assert(SRT_LEAF_TRIS_LDS >= 1 && SRT_LEAF_TRIS_LDS - 1 <= kTriPad, "SRT_LEAF_TRIS_LDS");

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
  t.ref = __float_as_uint(rlo.w);
  t.cnt = ok ? __float_as_uint(rhi.w) : kNoneCnt;
  t.sp = 0;
  t.lo = 0;
  t.start = false;
}

// Leaf sub-step: up to kLeafTris triangles of the current leaf, in order: each
// is tested against the distance the previous one left; a shadow ray stops at
// its first accept (the triangle array is padded with kTriPad zero records).
// `tp`: the kLeafTris triangle records from t.ref on, already loaded (3 float4 each).
template <bool COUNT, bool LDSM>
__device__ __forceinline__ void trav_leaf_x(const KParams& kp, Counters& c, Trav& t, bool any, const float4* tp) {
  constexpr int kLT = kLeafTrisM<LDSM>;
  const uint32_t n = t.cnt < (uint32_t)kLT ? t.cnt : (uint32_t)kLT;
  bump<COUNT>(c, ST_TRIS, n);
  float dist = t.dist;
  uint32_t hit = t.hit;
  bool stop = false;
  // all triangles' loads and reciprocals first (one shared fallback branch),
  // so the triangles' arithmetic overlaps; then the tests in order
  TriPrep pr[kLT];
  bool slow = false;
#pragma unroll
  for (int k = 0; k < kLT; ++k) slow |= tri_prep(t.d, tp[3 * k], tp[3 * k + 1], tp[3 * k + 2], pr[k]);
  if (__builtin_expect(slow, 0)) {
#pragma unroll
    for (int k = 0; k < kLT; ++k) pr[k].f = 1.0f / pr[k].a;
  }
#pragma unroll
  for (int k = 0; k < kLT; ++k) {
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
  const uint32_t rest = t.cnt - n;
  t.active = !stop;
  t.cnt = (rest == 0 || stop) ? kNoneCnt : rest;
  t.sp = stop ? 0 : t.sp;  // a stopped shadow ray pops nothing (trav_pop tests no `active`)
  if constexpr (!LDSM) t.lo = stop ? 0 : t.lo;
}
template <bool COUNT, bool LDSM>
__device__ __forceinline__ void trav_leaf(const KParams& kp, Counters& c, Trav& t, bool any) {
  if constexpr (LDSM) {
    trav_leaf_x<COUNT, LDSM>(kp, c, t, any, tri_ptr<LDSM>(kp, t.ref));
  } else {
    // Global-scene mode reads only the current leaf's records: a record past the leaf's last
    // triangle (tested, then discarded) is read from the leaf's first record instead, so a step
    // touches only the lines its leaf lies in (LayoutTris keeps a one- or two-triangle leaf in one).
    const float4* p = tri_ptr<false>(kp, t.ref);
    float4 x[3 * kLeafTris];
#pragma unroll
    for (int k = 0; k < kLeafTris; ++k) {
      const float4* q = (k == 0 || (uint32_t)k < t.cnt) ? p + 3 * k : p;
      x[3 * k] = q[0];
      x[3 * k + 1] = q[1];
      x[3 * k + 2] = q[2];
    }
    trav_leaf_x<COUNT, false>(kp, c, t, any, x);
  }
}

// Internal sub-step: test both children's boxes; push c0 when both pass, go to
// c1 if it passes, else to c0 if it passes.
// (l0, h0, l1, h1): the child pair; (m0, g0, m1, g1): c1's child pair when `spine`.
template <bool COUNT, bool LDSM, bool PACK, int RING = kShortStack>
__device__ __forceinline__ void trav_internal_x(const KParams& kp, const Lane& ln, Counters& c, Trav& t,
                                                const float4 l0, const float4 h0, const float4 l1, const float4 h1,
                                                const float4 m0, const float4 g0, const float4 m1, const float4 g1,
                                                const bool spine) {
  bump<COUNT>(c, ST_NODES, 2);
  float b0, b1;
  const bool v0 = box_test(t.o, t.inv, l0, h0, t.dist, b0);
  const bool v1 = box_test(t.o, t.inv, l1, h1, t.dist, b1);
  const uint32_t r0 = __float_as_uint(l0.w), n0 = __float_as_uint(h0.w);
  // the c0 slot is written unconditionally (it is free either way; the stack
  // holds depth + 1 entries, validated at upload)
  auto push_entry = [&](uint32_t r_, uint32_t n_, float b_) {
    if constexpr (LDSM) {
      slot_write<true>(ln.stk, ln.stride, t.sp, r_, n_, b_);
    } else {
      if (t.sp - t.lo == RING) {  // ring full: its oldest entry moves to HBM (rare)
        uint32_t r, n;
        float bt;
        slot_read<PACK>(ln.stk, ln.stride, t.lo & (RING - 1), r, n, bt);
        slot_write<PACK>(ln.gstk, ln.gstride, t.lo, r, n, bt);
        ++t.lo;
      }
      slot_write<PACK>(ln.stk, ln.stride, t.sp & (RING - 1), r_, n_, b_);
    }
  };
  push_entry(r0, n0, b0);
  t.sp += (v0 & v1) ? 1 : 0;
  if constexpr (COUNT) {
    if ((uint32_t)t.sp > c.v[ST_MAXSTACK]) c.v[ST_MAXSTACK] = (uint32_t)t.sp;
  }
  t.ref = v1 ? __float_as_uint(l1.w) : r0;
  t.cnt = v1 ? __float_as_uint(h1.w) : (v0 ? n0 : kNoneCnt);
  if constexpr (kSpine<LDSM>) {
    // The reference pops c1 right after pushing it and re-tests its box with
    // the unchanged distance (it passes), so when c1 is internal its expansion
    // is the lane's next step.  Its child pair was read with this node's (the
    // layout puts it next): expand it now -- one memory round trip for two levels.
    if (v1 & spine) {
      bump<COUNT>(c, ST_NODES, 2);
      float e0, e1;
      const bool w0 = box_test(t.o, t.inv, m0, g0, t.dist, e0);
      const bool w1 = box_test(t.o, t.inv, m1, g1, t.dist, e1);
      const uint32_t s0 = __float_as_uint(m0.w), k0 = __float_as_uint(g0.w);
      push_entry(s0, k0, e0);
      t.sp += (w0 & w1) ? 1 : 0;
      if constexpr (COUNT) {
        if ((uint32_t)t.sp > c.v[ST_MAXSTACK]) c.v[ST_MAXSTACK] = (uint32_t)t.sp;
      }
      t.ref = w1 ? __float_as_uint(m1.w) : s0;
      t.cnt = w1 ? __float_as_uint(g1.w) : (w0 ? k0 : kNoneCnt);
    }
  }
}
template <bool COUNT, bool LDSM, bool PACK, int RING = kShortStack>
__device__ __forceinline__ void trav_internal(const KParams& kp, const Lane& ln, Counters& c, Trav& t) {
  const uint32_t ref0 = t.ref | kp.ref_or;  // the child pair's first slot
  const bool spine = kSpine<LDSM> && (ref0 != t.ref);  // c1 is internal and its pair follows
  const uint32_t pi = 2 * ref0 + 2;
  float4 l0, h0, l1, h1;
  node_pair<LDSM>(kp, ref0, l0, h0, l1, h1);
  float4 m0, g0, m1, g1;  // c1's child pair
  if (spine) {
    m0 = node4<LDSM>(kp, pi + 4);
    g0 = node4<LDSM>(kp, pi + 5);
    m1 = node4<LDSM>(kp, pi + 6);
    g1 = node4<LDSM>(kp, pi + 7);
  }
  trav_internal_x<COUNT, LDSM, PACK, RING>(kp, ln, c, t, l0, h0, l1, h1, m0, g0, m1, g1, spine);
}

template <bool LDSM, bool PACK, int RING = kShortStack>
__device__ __forceinline__ void trav_pop(const KParams& kp, const Lane& ln, Trav& t);

// Cooperative line loads (global-scene mode, SRT_COOP).  The fused sub-step's loads are divergent
// gathers: each lane reads its own 64-128 B with 4-8 dwordx4 instructions, and the vector-memory
// pipeline (TA/TD) spends about one cycle per distinct cache line per instruction -- ~30 per
// instruction, busy 0.93-0.97 of the kernel's time (profiles/r05_experiments/vmem_pipeline.json).
// Instead, 8 lanes fetch one lane's request together: one instruction moves 8 requests' whole lines
// (1 KB, 8 lines) by LDS-DMA into a per-wave stage, and each lane reads its own row back.  The active
// lanes are ranked (mbcnt of the wave's ballot) and publish their request word in a rank table; a round
// stages kCoopRows ranks (three groups of 8), so a sub-step with more active lanes takes a second
// round.  Row r holds slot k at 16-B position (k + (r >> 1)) & 7, so 16 lanes reading the same slot
// of consecutive rows hit 16 different 16-B bank slots.
#ifndef SRT_COOP
#define SRT_COOP 0
#endif
constexpr int kCoopRows = 24;
constexpr uint32_t kCoopRowBytes = 128;                                          // 8 float4
constexpr uint32_t kCoopWaveBytes = kCoopRows * kCoopRowBytes + 64 * 4;          // rows + rank table
constexpr uint32_t kCoopIdxBits = 29;  // request word: float4 index | (nf4 / 2 - 2) << 29 | leaf << 31

template <bool COUNT, bool PACK, int RING>
__device__ __forceinline__ void trav_fused_coop(const KParams& kp, const Lane& ln, Counters& c, Trav& t, bool any) {
  const bool at_int = t.cnt == 0u, at_leaf = trav_at_leaf(t.cnt);
  const bool act = at_int | at_leaf;
  const uint32_t ref0 = t.ref | kp.ref_or;
  const bool spine = kSpine<false> && at_int && (ref0 != t.ref);
  static_assert(kLeafTris == 2, "trav_fused_coop stages two triangle records");
  const uint64_t M = __ballot(act);
  const uint32_t n = (uint32_t)__popcll(M);  // wave-uniform
  float4 x[8];
  if (n != 0u) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t stage = (uint32_t)kp.coop_off + (threadIdx.x >> 6) * kCoopWaveBytes;  // wave-uniform
    uint32_t* table = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(g_smem) + stage + kCoopRows * kCoopRowBytes);
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(M >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)M, 0u));
    if (act) {
      const uint32_t idx = at_leaf ? 3u * t.ref : 2u * ref0 + 2u;
      const uint32_t cls = at_leaf ? 1u : (spine ? 2u : 0u);  // nf4 = 4 + 2 cls
      table[rank] = idx | (cls << kCoopIdxBits) | ((at_leaf ? 1u : 0u) << 31);
    }
    for (uint32_t base = 0; base < n; base += (uint32_t)kCoopRows) {  // rounds (wave-uniform)
      if (base != 0u) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the last round's rows are read
#pragma unroll
      for (int j = 0; j < kCoopRows / 8; ++j) {
        if (base + 8u * j < n) {  // wave-uniform
          const uint32_t row = 8u * j + (lane >> 3), r = base + row;
          if (r < n) {
            const uint32_t w = table[r];
            const uint32_t k = ((lane & 7u) - (row >> 1)) & 7u;  // the slot this lane's position holds
            const uint32_t nf4 = 4u + 2u * ((w >> kCoopIdxBits) & 3u);
            const float4* src = ((w >> 31) ? kp.tris : kp.nodes) + (w & ((1u << kCoopIdxBits) - 1u)) + k;
            if (k < nf4)
              __builtin_amdgcn_global_load_lds(
                  (__attribute__((address_space(1))) void*)src,
                  (__attribute__((address_space(3))) void*)((__attribute__((address_space(3))) char*)g_smem + stage +
                                                            (uint32_t)j * 8u * kCoopRowBytes),
                  16, 0, 0);
          }
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (act && rank - base < (uint32_t)kCoopRows) {  // (unsigned: rank >= base)
        const uint32_t row = rank - base, rot = row >> 1;
        const uint32_t rb = stage + row * kCoopRowBytes;
#pragma unroll
        for (int k = 0; k < 4; ++k) x[k] = lds4(rb + (((uint32_t)k + rot) & 7u) * 16u);
        if (at_leaf | spine) {
          x[4] = lds4(rb + ((4u + rot) & 7u) * 16u);
          x[5] = lds4(rb + ((5u + rot) & 7u) * 16u);
        }
        if (spine) {
          x[6] = lds4(rb + ((6u + rot) & 7u) * 16u);
          x[7] = lds4(rb + ((7u + rot) & 7u) * 16u);
        }
      }
    }
    if (at_int)
      trav_internal_x<COUNT, false, PACK, RING>(kp, ln, c, t, x[0], x[1], x[2], x[3], x[4], x[5], x[6], x[7], spine);
    else if (at_leaf)
      trav_leaf_x<COUNT, false>(kp, c, t, any, x);
  }
  trav_pop<false, PACK, RING>(kp, ln, t);
}

// Global-scene mode: one sub-step for both node kinds.  Lanes at an internal
// node and lanes at a leaf issue their loads (node pairs or triangle records)
// as one set of per-lane-addressed loads, so the wave waits for memory once
// for both; then each kind's tests run on their lanes.  The memory-latency-bound
// global mode trades the second kind's idle lanes for half the round trips;
// each lane's steps, and so its decisions, are unchanged.
template <bool COUNT, bool PACK, int RING = kShortStack, bool TL = false>
__device__ __forceinline__ void trav_fused(const KParams& kp, const Lane& ln, Counters& c, Trav& t, bool any) {
  const bool at_int = t.cnt == 0u, at_leaf = trav_at_leaf(t.cnt) && !(TL && t.cnt == kTreeletCnt);
  if (at_int | at_leaf) {
    const uint32_t ref0 = t.ref | kp.ref_or;
    const bool spine = kSpine<false> && at_int && (ref0 != t.ref);
    // leaf: kLeafTris = 2 records (6 float4; kTriPad zero records keep them in
    // bounds); internal: the pair (4 float4) and, on the spine, the next pair
    static_assert(kLeafTris == 2, "trav_fused loads two triangle records");
    const uint32_t pi = 2 * ref0 + 2;
    const float4* p = at_leaf ? kp.tris + 3 * (size_t)t.ref : kp.nodes + pi;
    float4 x[8];
    // an internal step whose pair (and spine pair) lie in the top levels' region reads them from the
    // block's LDS copy (padded pair blocks: the spine pair is the next block), off the vector-memory pipeline
    if (at_int && pi + (spine ? 8u : 4u) <= (uint32_t)kp.top_f4) {
      const uint32_t b = (uint32_t)kp.top_lds_f4 + (pi >> 2) * kNodeBlkF4;
      x[0] = g_smem[b];
      x[1] = g_smem[b + 1];
      x[2] = g_smem[b + 2];
      x[3] = g_smem[b + 3];
      if (spine) {
        x[4] = g_smem[b + kNodeBlkF4];
        x[5] = g_smem[b + kNodeBlkF4 + 1];
        x[6] = g_smem[b + kNodeBlkF4 + 2];
        x[7] = g_smem[b + kNodeBlkF4 + 3];
      }
    } else {
      // (a one-triangle leaf still reads two records here: reading its own record twice, as
      // trav_leaf does, measured 1% slower on the torus knot and within 0.5% elsewhere)
      x[0] = p[0];
      x[1] = p[1];
      x[2] = p[2];
#if SRT_MASK_LEAF2
      // experiment: a one-triangle leaf's lanes sit out its second record's three loads (a masked lane
      // costs the vector-memory pipeline nothing, tools/probes/vmem_cost.hip); the record's stand-in is a
      // zero record (a = 0: tested, then discarded by trav_leaf_x's k < n; a constant, so no load waits on it)
      const bool two = at_leaf && t.cnt >= 2u;
      x[3] = x[4] = x[5] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
      if (at_int | two) x[3] = p[3];
      if (spine | two) {
        x[4] = p[4];
        x[5] = p[5];
      }
#else
      x[3] = p[3];
      if (at_leaf | spine) {
        x[4] = p[4];
        x[5] = p[5];
      }
#endif
      if (spine) {
        x[6] = p[6];
        x[7] = p[7];
      }
    }
    if (at_int)
      trav_internal_x<COUNT, false, PACK, RING>(kp, ln, c, t, x[0], x[1], x[2], x[3], x[4], x[5], x[6], x[7], spine);
    else trav_leaf_x<COUNT, false>(kp, c, t, any, x);
  }
  trav_pop<false, PACK, RING>(kp, ln, t);
}

// Nothing current: pop one entry (visited if it still beats the running
// distance).  A lane whose stack is empty waits for trav_finish at the end of
// the iteration (its later sub-steps have nothing to do either), so the pop
// is one branch.  The test is two compares: a shadow ray that stopped has
// emptied its stack, and `start` is never set during the sub-steps
// (trav_finish sets it at the end of an iteration, trav_step clears it before
// the first sub-step).
template <bool LDSM, bool PACK, int RING>
__device__ __forceinline__ void trav_pop(const KParams& kp, const Lane& ln, Trav& t) {
  if ((t.cnt == kNoneCnt) & (t.sp > 0)) {
    --t.sp;
    uint32_t r, n;
    float et;
    if constexpr (LDSM) {
      slot_read<true>(ln.stk, ln.stride, t.sp, r, n, et);
    } else if (t.sp < t.lo) {  // below the LDS ring: from HBM (rare)
      slot_read<PACK>(ln.gstk, ln.gstride, t.sp, r, n, et);
      t.lo = t.sp;
    } else {
      slot_read<PACK>(ln.stk, ln.stride, t.sp & (RING - 1), r, n, et);
    }
    const bool take = et < t.dist;
    t.ref = r;
    t.cnt = take ? n : kNoneCnt;
  }
}

// End of an iteration: a lane with nothing current and an empty stack has
// finished this BVH -- CheckHit's loop over bvh_count is complete (or, for a
// shadow ray, a hit was found), or the next BVH is set up next iteration.
__device__ __forceinline__ void trav_finish(const KParams& kp, Trav& t, bool any) {
  if (t.active & (t.cnt == kNoneCnt) & (t.sp == 0)) {  // (see trav_pop for the short test)
    if ((any && t.hit != kNoneRef) || t.bi + 1 >= kp.bvh_count) {
      t.active = false;
    } else {
      ++t.bi;
      t.start = true;
    }
  }
}

template <bool COUNT, bool LDSM, bool PACK, bool FUSE, int K, int RING = kShortStack, bool TL = false,
          bool COOP = false>
__device__ __forceinline__ void trav_substeps(const KParams& kp, const Lane& ln, Counters& c, Trav& t, bool any) {
  if constexpr (FUSE) {
    static_assert(!LDSM, "fused sub-steps are a global-scene mode schedule");
    if constexpr (K < kFusedSteps) {
      if constexpr (COOP) trav_fused_coop<COUNT, PACK, RING>(kp, ln, c, t, any);
      else trav_fused<COUNT, PACK, RING, TL>(kp, ln, c, t, any);
      trav_substeps<COUNT, LDSM, PACK, FUSE, K + 1, RING, TL, COOP>(kp, ln, c, t, any);
    }
  } else if constexpr (step_kind<LDSM>(K) != 0) {
    if constexpr (step_kind<LDSM>(K) == 'I') {
      DBG_COUNT(kp.stats, ST_DBG_SUB + 3 * K, t.cnt == 0);
      if (t.cnt == 0) trav_internal<COUNT, LDSM, PACK, RING>(kp, ln, c, t);
    } else {
      DBG_COUNT(kp.stats, ST_DBG_SUB + 3 * K, trav_at_leaf(t.cnt));
      if (trav_at_leaf(t.cnt) && !(TL && t.cnt == kTreeletCnt)) trav_leaf<COUNT, LDSM>(kp, c, t, any);
    }
    DBG_COUNT(kp.stats, ST_DBG_SUB + 3 * K + 2, t.active & (t.cnt == kNoneCnt));
    trav_pop<LDSM, PACK, RING>(kp, ln, t);
    trav_substeps<COUNT, LDSM, PACK, FUSE, K + 1, RING, TL, COOP>(kp, ln, c, t, any);
  }
}

// One traversal iteration (see traverse() for the order argument): the
// sub-steps of the mode's pattern in turn, each taken by the lanes whose current
// node is of its kind, so a lane makes up to strlen(pattern) steps of
// its own sequence per iteration, in order.  `any` selects the shadow-ray
// (first hit) variant.
// RING: global-scene mode's LDS ring entries per lane (a power of two).
// TL (wavefront mode's top-level kernel): a current node whose count is kTreeletCnt is a treelet root of
// the flagged node copy; no sub-step takes it (the caller suspends the ray there, wavefront.hpp).
// COOP: the fused sub-steps' loads as cooperative line loads (trav_fused_coop; the caller stages them).
template <bool COUNT, bool LDSM, bool PACK, bool FUSE, int RING = kShortStack, bool TL = false, bool COOP = false>
__device__ __forceinline__ void trav_step(const KParams& kp, const Lane& ln, Counters& c, Trav& t, f3 ro, f3 rd,
                                          bool any) {
  static_assert((RING & (RING - 1)) == 0, "the LDS ring holds a power-of-two number of entries");
  if (t.start) trav_begin_bvh<COUNT, LDSM>(kp, c, t, ro, rd);  // only for BVHs after the first
  trav_substeps<COUNT, LDSM, PACK, FUSE, 0, RING, TL, COOP>(kp, ln, c, t, any);
  trav_finish(kp, t, any);
}

}  // namespace srt
