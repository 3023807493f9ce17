// device_common.hpp -- kernel parameters, launch statistics, per-lane context, RNG and small BRDF helpers
// of the path-tracing kernels (included once, by pathtrace.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "pt_math.hpp"
#include "srt_internal.hpp"

namespace srt {
using namespace dev;

// ---------------------------------------------------------------------------
// kernel parameters (kernarg segment -> scalar registers)
// ---------------------------------------------------------------------------
struct KParams {
  const float4* nodes;   // node i at nodes[2*i + 2], nodes[2*i + 3]
  const float4* tris;    // 3 float4 per triangle
  const float4* mats;    // 2 float4 per material (m1.w: sampled texture + 1, as bits)
  const float4* lights;  // 2 float4 per light, light_count + 1 records
  const srt_bvh_record* bvhs;
  const float2* noise_xy;
  const float* noise_u;
  float4* accum;
  uint32_t* out;
  unsigned long long* stats;
  unsigned long long* nan_ctr;  // path samples with a NaN component (accumulate_kernel; srt_nan_samples)
  uint32_t* batch_ctr;     // next unclaimed 64-item batch of the launch (zeroed before it)
  int tail_start;          // batches from which a claim takes one batch (LaunchSamples)
  int W, H, WH;
  int light_count;   // lightCount uniform (loop count)
  int light_records; // records in the light SSBO; index >= light_records reads zeros
  uint32_t bvh_count;
  int show_model;
  int max_depth;
  int frame_first, nframes, write_output, reset;
  int rank, nranks, band_rows, local_rows;
  int band_shift;          // log2(band_rows) when band_rows is a power of two, else -1
  int ext_w, ext_h;
  int stack_entries;
  int nodes_f4, tris_f4;   // LDS-resident scene: sizes of the node / triangle arrays in float4
  int nodes_lds_f4;        // LDS mode: float4 the node copy occupies (pair blocks padded, traversal.hpp node_lds_f4)
  // internal nodes' child index: pairs start at odd slots and an even index (the
  // pair's start - 1) flags a right child whose own pair follows (pathtrace.hip
  // LayoutNodes); ref_or = 1 decodes it, 0 for the identity layout (no flags)
  uint32_t ref_or;
  float4* lbuf;            // sample buffer: nframes x local_pixels radiance samples
  int local_pixels;        // W * local_rows
  int trav_frac16;         // resume shading when fewer than trav_frac16/16 of working lanes traverse
  int bounce_cap;          // bounces after which a path is cut (and counted in ST_BOUNCECAP)
  // pool_kernel (pool.hpp): LDS byte offsets of the control words, the 3 rings (pool_cap u32 each)
  // and the pool_slots 112-B records; the hits a shading wave waits for, and the level of the trace
  // + spare rings under which it shades fewer; the watchdog (s_memrealtime ticks)
  int pool_ctl_off, pool_ring_off, pool_rec_off, pool_cap, pool_slots, pool_batch, pool_tlow;
  unsigned long long pool_deadline;
  int stack_base_f4;       // first float4 of the per-lane stacks in dynamic LDS
  int coop_off;            // global-scene mode, SRT_COOP: LDS byte offset of the waves' load stages (traversal.hpp)
  // global-scene mode, fused instance: the node array's first top_f4 float4 (the top levels' pairs,
  // pathtrace.hip LayoutNodes) copied into each block's LDS at float4 top_lds_f4 (padded pair blocks,
  // node_lds_f4); 0: none
  int top_f4, top_lds_f4;
  uint32_t* gstack;        // global-scene mode: per-lane stacks in HBM, entry field k of lane g at gstack[k * stride + g]
  int gstack_stride;       // lanes in the grid
  float cx, cy, cz, p00x, p00y, p00z, dux, duy, duz, dvx, dvy, dvz;
  // texture sampling (the TEX kernel instances)
  const float4* tri_uv;      // 2 float4 per triangle: vertex uvs uv0 uv1 | uv2
  const float4* tex_texels;  // RGBA32F texels of all textures (SRT_TEX8=0 builds)
  const uint32_t* tex_texels8;  // RGBA8 texels of all textures, r | g << 8 | b << 16 (SRT_TEX8 builds)
  const uint4* tex_info;     // per texture: first texel, width, height
  uint32_t n_tex;
  // LDS copies of the light and material records (read per shading), when they fit
  int lights_lds, lights_base_f4;  // light_records + 1 records of 2 float4
  int mats_lds, mats_base_f4, mat_records;  // mat_records records of 2 float4
  const uint32_t* tile_order;  // the launch's tiles in schedule order (nullptr: natural order)
  uint32_t* tile_cost;         // per tile: first-frame bounces recorded for the next launch's order (or nullptr)
  unsigned long long* wave_trace;  // diagnostic build (SRT_WAVE_TRACE): 4 stamps per wave
  unsigned long long* span;        // {first wave's start, last wave's end} (s_memrealtime, 100 MHz), or nullptr
  const int* row_map;      // nranks > 1: the global row of each local row (row bands, pathtrace.hip FillParams)
};

// Dynamic LDS of the path-tracing kernels: [scene copy (LDS mode)] [per-lane stacks].
extern __shared__ __attribute__((aligned(16))) float4 g_smem[];

enum { ST_RAYS = 0, ST_NODES, ST_TRIS, ST_RNGU, ST_RNGSQ, ST_LIGHTS, ST_MATS, ST_SAMPLES, ST_OVERFLOW, ST_MAXSTACK,
       ST_BOUNCECAP,  // paths cut at the bounce cap (KParams::bounce_cap)
       ST_SHADOW,     // shadow rays among ST_RAYS (CheckLightOccluded, raytrace_compute.glsl:167-176)
       ST_N, ST_CYC_REFILL = ST_N, ST_CYC_TRAV, ST_CYC_SHADE, ST_CYC_ITERS,
       // lane occupancy of the traversal loop (summed popcounts per iteration) and of shading
       ST_DBG_TITERS, ST_DBG_WORK, ST_DBG_TRAV, ST_DBG_LEAF, ST_DBG_INT, ST_DBG_SHADE,
       // per traversal sub-step k < 16: lanes taking it (summed), waves executing it, lanes popping after it
       ST_DBG_SUB, ST_POOLERR = ST_DBG_SUB + 48,  // pool_kernel's watchdog fired (pool.hpp)
       ST_TOTAL };
// SRT_PHASE_TIMING builds, in the last two sub-steps' slots (no pattern has 15 sub-steps): traversing lanes
// summed per traversal iteration by ray kind (shadow, camera, bounce), and ray starts by kind (camera,
// shadow, bounce)
constexpr int ST_DBG_KIND = ST_DBG_SUB + 42;

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
  const float d = __builtin_fmaf(sy, 78.233f, sx * 12.9898f);  // dot(seed, vec2(12.9898, 78.233))
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

__device__ __forceinline__ float luminance(f3 c) { return dot(c, mk(0.2126f, 0.7152f, 0.0722f)); }
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

}  // namespace srt
