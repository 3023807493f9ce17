// kernels.hpp -- the kernels: persistent sample_kernel, accumulate_kernel, reset_kernel,
// closest_kernel (UpdateRays test path) and assemble_kernel (multi-GPU root).
#pragma once

#include "shading.hpp"
#include "traversal.hpp"

namespace srt {
using namespace dev;

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
__device__ __forceinline__ int lane_rank(unsigned long long mask, int lane) {
  return __popcll(mask & ((1ull << lane) - 1ull));
}

#ifndef SRT_TILE_SCHED
#define SRT_TILE_SCHED 1  // tiles of each frame in the last launch's cost order
#endif
// sphere_kernel: trace a bounce's shadow ray (1), and its next ray too (2), in the shading pass that
// set them up (each is one test of the five spheres)
#ifndef SRT_SPH_SHADOW_NOW
#define SRT_SPH_SHADOW_NOW 2
#endif
#ifndef SRT_NT_SAMPLES
#define SRT_NT_SAMPLES 0  // sample-buffer stores with the streaming (nontemporal) policy
#endif
#ifndef SRT_NT_JITTER
#define SRT_NT_JITTER 0   // camera-jitter (noiseTex) loads with the streaming policy (an experiment, round 5)
#endif
// sphere_kernel streams its camera-jitter loads and sample-buffer stores past the XCD's L2 (round 5): each
// is touched once per sample, and the L2 then holds the randomly gathered noiseUniformTex -- C2's L2 hit
// rate 0.68 -> 0.79 and its L2-miss lines per sample 84.6 -> 54.5 B (§8d: 52.6 B) at the same kernel time
// (profiles/r05_experiments/c2_streaming_policy.json); the mesh kernels lose 0.7-2% with it (their L2
// holds tree lines too), so they keep the default policy
#ifndef SRT_NT_SPH
#define SRT_NT_SPH 1
#endif
// The IL instance (trees past 600 MB) deals a tile's frames in a row (C5 783 -> 771 ms per launch,
// A/B on one box; 8 or 16 batches per claim instead of 4: 776 / 792 ms)
#ifndef SRT_TILE_MAJOR_IL
#define SRT_TILE_MAJOR_IL 1
#endif

// Global-scene mode's occupancy regimes (GW, waves per SIMD): 4 (<= 128 VGPRs, no
// spills; 16-entry LDS rings, 32 KiB per 256-lane block), or 5 (<= 96 VGPRs, ~10
// dwords spilled; 8-entry rings, 16 KiB per block) for trees small enough that
// more rays in flight beat the spills (srt_upload_scene picks it by scene size).
// (SRT_COOP builds keep 8-entry rings at either regime: the cooperative loads' stage takes the rest)
#ifndef SRT_RING_GW5
#define SRT_RING_GW5 8
#endif
__host__ __device__ constexpr int global_ring(int gw) { return (gw > 4 || SRT_COOP) ? SRT_RING_GW5 : kShortStack; }
// GetRayColor's loop body for a ray whose CheckHit hit (raytrace_compute.glsl:225-290): the
// hit record, this bounce's draws, SampleLights, both shadow outcomes of the direct light
// (q0: occluded, q1: visible), the BRDF choice, Russian roulette and the next direction.
// `ht`: the hit triangle (mesh scene) or `hit_sphere`; `dist`: the hit distance along (ro, rd).
// Returns what the path traces next: kShadeShadow (CheckLightOccluded's ray, ro/rd/tmax set,
// the bounce direction in nd), kShadeBounce (the next CheckHit ray) or kShadeDone.
enum { kShadeDone = 0, kShadeShadow = 1, kShadeBounce = 2 };
// SPH: the sphere scene's instance (sphere_kernel); every other caller is a mesh scene (showModel set).
template <bool COUNT, bool LDSM, bool TEX, bool SPH = false>
__device__ __forceinline__ int shade_hit(const KParams& kp, const Lane& ln, Counters& c, uint32_t ht, int hit_sphere,
                                         float dist, f3& ro, f3& rd, float& tmax, f3& T, int& depth, int& randIndex,
                                         int& bounces, bool& term, f3& q0, f3& q1, f3& nd) {
  // ---- hit record (CheckHit) ----
  Hit rec;
  rec.hit = true;
  if constexpr (!SPH) {
    rec.p = (dist * rd) + ro;
    const float4* tp = tri_ptr<LDSM>(kp, ht);
    const float4 A = tp[0], B = tp[1], C = tp[2];
    rec.normal = normalize(cross(mk(A.w, B.x, B.y), mk(B.z, B.w, C.x)));
    const uint32_t mi = __float_as_uint(C.y);
    float4 m0, m1;
    if (kp.mats_lds) {
      m0 = lds4((uint32_t)(kp.mats_base_f4 + 2 * mi) << 4);
      m1 = lds4((uint32_t)(kp.mats_base_f4 + 2 * mi + 1) << 4);
    } else {
      m0 = kp.mats[2 * mi];
      m1 = kp.mats[2 * mi + 1];
    }
    bump<COUNT>(c, ST_MATS);
    rec.mat.albedo = mk(m0.x, m0.y, m0.z);
    if constexpr (TEX) {  // the instance for scenes whose materials sample a texture
      const uint32_t tex = __float_as_uint(m1.w);  // sampled texture + 1
      if (tex != 0u) rec.mat.albedo = mesh_texture_albedo(kp, tex - 1, ht, A, B, C, dist, ro, rd);
    }
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
    // Iteration i selects when its draw r < ris / total_i with total_i =
    // (i + 1) * ris.  When ris / total is NaN (ris is 0 -- the zero record
    // past the lights -- or not finite) it is NaN at every i: no draw can
    // select and the draws are skipped: they never change a value (the
    // counters count the fetches the kernel makes).  This ~1-in-2n case
    // otherwise costs n - 1 dependent gathers, and with ~35 shading lanes
    // nearly every wave has such a lane.
    float total = ris, pdf = 0.0f;  // 0 + ris
    const float sel0 = div_rn(ris, total);
    if (u_sel0 < sel0) {
      pdf = lpdf;
      selected = true;
    }
    const bool draws = !selected && (sel0 == sel0);
    for (int i = 1; i < n; ++i) {
      total += ris;
      if (draws && !selected) {
        const float r = randU<COUNT>(kp, ln, c, p.y + (float)i, p.z + (float)i);
        if (r < div_rn(ris, total)) {
          pdf = lpdf;
          selected = true;
        }
      }
    }
    lw = div_rn(div_rn(total, (float)n), fmx(0.001f, pdf));
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
  // survival probability to >= 0.1).  A path still alive after
  // kp.bounce_cap bounces (2^20 unless SRT_BOUNCE_CAP says otherwise) is
  // cut and counted, so a pathological scene cannot hang the GPU.
  if (++bounces >= kp.bounce_cap && !term) {
    term = true;
    bump<COUNT>(c, ST_BOUNCECAP);
  }
  ro = p;
  if (selected) {  // trace CheckLightOccluded's ray next (t in (0.001, |light - p|))
    rd = sdir;
    tmax = smax;
    return kShadeShadow;
  }
  if (term) return kShadeDone;
  rd = nd;
  tmax = __builtin_inff();
  return kShadeBounce;
}

// waves per SIMD the register allocation must allow: 4 (<= 128 VGPRs) in LDS
// mode, where the 1024-thread block's LDS caps residency at 4 anyway; GW in
// global-scene mode (see global_ring), whose memory latency wants more waves
// FUSE: global-scene mode's fused sub-steps (trav_fused) instead of kStepPattern
// sample_kernel's body.  SPH: the sphere scene (showModel false: the five spheres, no BVH); otherwise a
// mesh scene (showModel set).  Each instance holds only its scene kind's code, so neither carries the
// other's registers beside its loop.
template <bool COUNT, bool LDSM, bool PACK, int BLOCK, bool TEX, bool FUSE, int GW, bool SPH>
__device__ __forceinline__ void sample_body(const KParams& kp) {
  const int tid = threadIdx.x;
  // the launch's span for its kernel time: pipelined launches overlap their neighbours, so HIP events
  // around them would time the wait for CUs too (pathtrace.hip Launch); vector atomics on two words
  if (kp.span && tid == 0) atomicMin(&kp.span[0], (unsigned long long)__builtin_amdgcn_s_memrealtime());
#ifdef SRT_WAVE_TRACE
  const unsigned long long tw0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long tw2 = 0;
#endif
  if constexpr (LDSM) {  // the block copies the scene (nodes + triangles) into LDS once
    // (node pair blocks at the padded stride, node_lds_f4; the pad slots are never read)
    for (int i = tid; i < kp.nodes_f4; i += blockDim.x) g_smem[node_lds_f4((uint32_t)i)] = kp.nodes[i];
    for (int i = tid; i < kp.tris_f4; i += blockDim.x) g_smem[kp.nodes_lds_f4 + i] = kp.tris[i];
  }
  if constexpr (FUSE && !LDSM) {  // global-scene mode: the top levels' pairs (kp.top_f4 float4, padded blocks)
    for (int i = tid; i < kp.top_f4; i += blockDim.x) g_smem[kp.top_lds_f4 + (int)node_lds_f4((uint32_t)i)] = kp.nodes[i];
  }
  {  // and the light and material records, when they fit (shading reads them from LDS)
    const int nl = kp.lights_lds ? 2 * (kp.light_records + 1) : 0, nm = kp.mats_lds ? 2 * kp.mat_records : 0;
    for (int i = tid; i < nl; i += blockDim.x) g_smem[kp.lights_base_f4 + i] = kp.lights[i];
    for (int i = tid; i < nm; i += blockDim.x) g_smem[kp.mats_base_f4 + i] = kp.mats[i];
  }
  __syncthreads();
  const int lane = tid & 63;
#ifdef SRT_WAVE_TRACE
  const unsigned long long tw1 = __builtin_amdgcn_s_memrealtime();
#endif
  Lane ln;
  if constexpr (LDSM) {
    ln.stk = reinterpret_cast<uint32_t*>(g_smem + kp.stack_base_f4) + tid;
    ln.stride = BLOCK;  // a compile-time stride: stack addressing by shifts, no v_mul_lo_u32
  } else {  // the top global_ring(GW) entries in an LDS ring, the rest in HBM (lane-interleaved, coalesced)
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
  // batches are claimed from a launch-wide counter of batches, so waves that
  // drew cheap tiles take more of them (no static-share tail).  A claim takes
  // kClaim consecutive batches and the next claim is issued one ahead (lane
  // 0's atomic returns while the current batch is consumed, and is only read,
  // broadcast, when needed).  From kp.tail_start on (16 claims per wave
  // before the end, pathtrace.hip) a claim takes one batch: a wave then holds
  // at most two batches, so the launch's tail is not set by slow waves still
  // draining several expensive batches each (tools/wave_trace.py).
  // `batch` and everything derived from it are wave-uniform (scalar
  // registers); the counter's overshoot past n_batches stays below 2^31.
  // The sphere scene's batches are cheap and take kClaimSph per claim.
  constexpr int kC = SPH ? kClaimSph : kClaim;
  uint32_t claimed = 0;
  int claim_sz = kp.tail_start > 0 ? kC : 1;  // size of the claim in flight
  if (lane == 0) claimed = atomicAdd(kp.batch_ctr, (uint32_t)claim_sz);
  int batch = __builtin_amdgcn_readfirstlane((int)__shfl(claimed, 0));
  int claim_left = claim_sz - 1;  // batches of the current claim after `batch`
  claim_sz = batch < kp.tail_start ? kC : 1;
  if (lane == 0) claimed = atomicAdd(kp.batch_ctr, (uint32_t)claim_sz);
  int batch_next = 0;         // items of `batch` already handed out

  // per-lane sample / path / traversal state
  bool has_work = false;
  int x = 0, gy = 0, li = 0, fidx = 0;
  f3 ro = mk(0.f, 0.f, 0.f), rd = mk(0.f, 0.f, 1.f), T, color, q0, q1, nd;
  float tmax = 0.0f;
  int depth = 0, randIndex = 0, hit_sphere = -1, bounces = 0;
  bool shadow_phase = false, term = false, pending = false;
  Trav tr;
  tr.active = false;
  tr.start = false;
  tr.hit = kNoneRef;
  tr.cnt = kNoneCnt;  // (idle: a wave-wide step leaves such a lane alone)
  tr.ref = 0;
  tr.sp = 0;
  tr.lo = 0;

#ifdef SRT_PHASE_TIMING
  unsigned long long d_kind[6] = {0, 0, 0, 0, 0, 0};  // (ST_DBG_KIND)
#endif
  auto start_ray = [&]() {
#ifdef SRT_PHASE_TIMING
    d_kind[shadow_phase ? 4 : (bounces == 0 ? 3 : 5)] += 1;  // per lane (ray starts by kind)
#endif
    tr.dist = tmax;
    tr.hit = kNoneRef;
    tr.bi = 0;
    tr.active = true;
    tr.start = false;
    bump<COUNT>(c, ST_RAYS);
    bump<COUNT>(c, ST_SHADOW, shadow_phase ? 1u : 0u);
    if constexpr (!SPH) {
      trav_begin_bvh<COUNT, LDSM>(kp, c, tr, ro, rd);
      if (tr.cnt == kNoneCnt) {  // root box missed: next BVH, or done
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
    if (SRT_TILE_SCHED && kp.tile_cost && fidx == 0) {  // this tile's cost for the next launch's order: its first frame's bounces
      const int ly = li / kp.W, px = li - ly * kp.W;
      atomicAdd(&kp.tile_cost[(ly >> 3) * tiles_x + (px >> 3)], (uint32_t)(bounces + 1));
    }
    color = color + T * mk(0.05f, 0.05f, 0.05f);  // skyColor, raytrace_compute.glsl:219,292
    if constexpr (SRT_NT_SAMPLES || (SPH && SRT_NT_SPH)) {
      // streaming store: the sample buffer passes through L2 once, and would evict the noise tables
      typedef float v4f __attribute__((ext_vector_type(4)));
      const v4f v = {color.x, color.y, color.z, 0.0f};
      __builtin_nontemporal_store(v, reinterpret_cast<v4f*>(kp.lbuf + ((size_t)fidx * (size_t)kp.local_pixels + (size_t)li)));
    } else {
      kp.lbuf[(size_t)fidx * (size_t)kp.local_pixels + (size_t)li] = make_float4(color.x, color.y, color.z, 0.0f);
    }
    has_work = false;
  };

#ifdef SRT_PHASE_TIMING
  unsigned long long cyc_refill = 0, cyc_trav = 0, cyc_shade = 0, iters = 0;
  unsigned long long d_titers = 0, d_work = 0, d_trav = 0, d_leaf = 0, d_int = 0, d_shade = 0;
#endif
  for (;;) {
    PHASE_STAMP(t_a);
    // ---- (A) idle lanes take the next items of the wave's batches ----
    // First every idle lane is assigned an item (a pass per batch the idle
    // lanes span: scalar batch decomposition, a few vector ops), then the
    // assigned lanes start their samples in one pass, so a refill that spans
    // two batches issues the camera-ray setup (and waits for its noise
    // fetch) once.
    bool fresh = false;          // assigned an item in this refill
    int a_pl = 0, a_gy = 0, a_f = 0, a_samp = 0;  // its pixel (x | local row << 16), global row, frame, sample index
    for (;;) {
      const unsigned long long idle = __ballot(!has_work & !fresh);
#ifdef SRT_WAVE_TRACE
      if (batch >= n_batches && tw2 == 0) tw2 = __builtin_amdgcn_s_memrealtime();
#endif
      if (idle == 0ull || batch >= n_batches) break;
      const int avail = 64 - batch_next;
      const int r = lane_rank(idle, lane);
      // the batch's frame and 8x8 tile (wave-uniform integer divisions, once per
      // batch): frame by frame, and within a frame the tiles in tile_order (the
      // last launch's tiles by decreasing cost, order_tiles_kernel), read by a
      // scalar load (constant address space: the order is read-only here)
      // the IL instance deals a tile's frames in a row (SRT_TILE_MAJOR_IL): a claim's batches then
      // trace the same pixels' camera rays, whose paths' lines are still in L2
      constexpr bool kTileMajor = SRT_TILE_MAJOR_IL && !LDSM && !FUSE && !SPH;
      const int frame_i = kTileMajor ? batch % kp.nframes : batch / n_tiles;
      const int trank = kTileMajor ? batch / kp.nframes : batch - frame_i * n_tiles;
#if SRT_TILE_SCHED
      const int tile = (int)((const __attribute__((address_space(4))) uint32_t*)(kp.tile_order))[trank];
#else
      const int tile = trank;
#endif
      const int ty = tile / tiles_x, tx = tile - ty * tiles_x;
      const int samp = (kp.frame_first + frame_i) % kp.WH;
      if (!has_work & !fresh & (r < avail)) {
        const int item = batch_next + r;
        const int px = tx * 8 + (item & 7), ly = ty * 8 + (item >> 3);
        if (px < kp.ext_w && ly < kp.local_rows) {
          // global row of local row ly: the identity on one rank; else the row
          // band's (kp.row_map, built by the host: a table read instead of the
          // band arithmetic keeps the refill's code small -- it is shared with
          // the traversal loop's registers, +0.7% on one rank)
          int yy = ly;
          if (kp.nranks > 1) yy = kp.row_map[ly];
          if (yy < kp.ext_h) {  // else the item is outside the dispatch extent: the lane tries the next one
            fresh = true;
            a_pl = px | (ly << 16);
            a_gy = yy;
            a_f = frame_i;
            a_samp = samp;
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
          batch = __builtin_amdgcn_readfirstlane((int)__shfl(claimed, 0));
          claim_left = claim_sz - 1;
          claim_sz = batch < kp.tail_start ? kC : 1;
          if (lane == 0) claimed = atomicAdd(kp.batch_ctr, (uint32_t)claim_sz);
        }
        batch_next = 0;
      }
    }
    if (fresh) {
      has_work = true;
      x = a_pl & 0xFFFF;
      gy = a_gy;
      li = (a_pl >> 16) * kp.W + x;
      fidx = a_f;
      ln.base = gy * kp.H + x;
      // GetRay (raytrace_compute.glsl:78-90) with SampleSquare (raytrace_utils.glsl:10-17)
      float2 nz;
      if constexpr (SRT_NT_JITTER || (SPH && SRT_NT_SPH)) {
        // the jitter texel streams past L2 (each is read once per sample), leaving the XCD's L2 to the
        // randomly gathered uniform-noise table
        typedef float v2f __attribute__((ext_vector_type(2)));
        const v2f nzv = __builtin_nontemporal_load(reinterpret_cast<const v2f*>(kp.noise_xy) + wrap_index(ln.base + a_samp, kp.WH));
        nz = make_float2(nzv.x, nzv.y);
      } else {
        nz = kp.noise_xy[wrap_index(ln.base + a_samp, kp.WH)];
      }
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
      pending = true;
    }
    // every lane with a ray to start (new samples, and the shadow / bounce
    // rays the last shading phase set up) starts it here, in one pass
    if (pending) {
      pending = false;
      start_ray();
    }
    if (__ballot(has_work) == 0ull) break;
    PHASE_STAMP(t_b);

    // ---- (B) traverse until too few lanes are still traversing ----
    if constexpr (!SPH) {
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
        d_kind[0] += __popcll(__ballot(tr.active && shadow_phase));
        d_kind[1] += __popcll(__ballot(tr.active && !shadow_phase && bounces == 0));
        d_kind[2] += __popcll(__ballot(tr.active && !shadow_phase && bounces > 0));
        d_leaf += __popcll(__ballot(tr.active && trav_at_leaf(tr.cnt)));
        d_int += __popcll(__ballot(tr.active && tr.cnt == 0));
#endif
        // (cooperative loads need every lane of the wave as a loader: the step runs wave-wide, and a lane
        // with no ray is idle in it -- nothing current, an empty stack, no BVH to set up)
        constexpr bool kCoopInst = (bool)SRT_COOP && FUSE && !LDSM;
        if (kCoopInst || tr.active)
          trav_step<COUNT, LDSM, PACK, FUSE, global_ring(GW), false, kCoopInst>(kp, ln, c, tr, ro, rd, shadow_phase);
      }
    }

    PHASE_STAMP(t_c);
#ifdef SRT_PHASE_TIMING
    d_shade += __popcll(__ballot(has_work && !tr.active));
#endif
    // ---- (C) lanes whose ray returned: shade (GetRayColor's loop body) ----
    if (has_work && !tr.active) {
      const bool hit = !SPH ? (tr.hit != kNoneRef) : (hit_sphere >= 0);
      const float dist = tr.dist;
      if (shadow_phase) {  // CheckLightOccluded returned: this bounce's direct light
        color = color + (hit ? q0 : q1);
        if (term) {
          finish_sample();
        } else {
          rd = nd;  // the bounce ray starts at the same hit point as the shadow ray
          tmax = __builtin_inff();
          shadow_phase = false;
          pending = true;  // started with the refill's new rays (one start_ray pass)
        }
      } else if (!hit) {
        finish_sample();
      } else {
        const int next = shade_hit<COUNT, LDSM, TEX, SPH>(kp, ln, c, tr.hit, hit_sphere, dist, ro, rd, tmax, T,
                                                          depth, randIndex, bounces, term, q0, q1, nd);
        if (next == kShadeDone) {
          finish_sample();
        } else {
          shadow_phase = next == kShadeShadow;
          pending = true;  // started with the refill's new rays (one start_ray pass)
          if constexpr (SPH && SRT_SPH_SHADOW_NOW >= 1) {
            // The sphere scene's rays are one test of the five spheres each: the shadow ray is traced
            // here, in the iteration that set it up, rather than in the next one -- the same test and
            // the same colour addition, in the path's order (as in the shadow_phase branch above) --
            // and (level 2) so is the bounce ray: a miss ends the sample now, a hit is shaded in the
            // next iteration.  So every lane with a hit shades in every iteration.
            if (shadow_phase) {
              pending = false;
              start_ray();
              color = color + ((hit_sphere >= 0) ? q0 : q1);
              if (term) {
                finish_sample();
              } else {
                rd = nd;
                tmax = __builtin_inff();
                shadow_phase = false;
                pending = true;
              }
            }
            if (SRT_SPH_SHADOW_NOW >= 2 && pending) {  // the bounce ray (kShadeBounce, or after the shadow ray)
              pending = false;
              start_ray();
              if (hit_sphere < 0) finish_sample();  // else its hit is shaded in the next iteration's pass
            }
          }
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
    for (int k = 0; k < 3; ++k) atomicAdd(&kp.stats[ST_DBG_KIND + k], d_kind[k]);
  }
  {  // ray starts were counted per lane
    for (int k = 3; k < 6; ++k) {
      unsigned long long v = d_kind[k];
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
      if (lane == 0) atomicAdd(&kp.stats[ST_DBG_KIND + k], v);
    }
  }
#endif
#ifdef SRT_WAVE_TRACE
  if (lane == 0 && kp.wave_trace) {
    unsigned long long* w = kp.wave_trace + 4 * ((size_t)blockIdx.x * (blockDim.x >> 6) + (tid >> 6));
    w[0] = tw0;
    w[1] = tw1;
    w[2] = tw2;
    w[3] = __builtin_amdgcn_s_memrealtime();
  }
#endif
  flush_counters<COUNT>(kp, c);
  if (kp.span && lane == 0) atomicMax(&kp.span[1], (unsigned long long)__builtin_amdgcn_s_memrealtime());
}

// A mesh scene (showModel set); FUSE/GW: global-scene mode's schedule and waves per SIMD.
template <bool COUNT, bool LDSM, bool PACK, int BLOCK, bool TEX, bool FUSE, int GW = 4>
__global__ __launch_bounds__(BLOCK, LDSM ? BLOCK / 256 : GW) void sample_kernel(KParams kp) {
  sample_body<COUNT, LDSM, PACK, BLOCK, TEX, FUSE, GW, false>(kp);
}

// The sphere scene (SHOW_MODEL 0, raytrace_compute.glsl:299-364): the same loop, each ray testing the
// five spheres in one go.
#ifndef SRT_SPH_WAVES
#define SRT_SPH_WAVES 4  // the register bound's waves per SIMD (it takes 87 VGPRs: 5 waves fit)
#endif
template <bool COUNT>
__global__ __launch_bounds__(256, SRT_SPH_WAVES) void sphere_kernel(KParams kp) {
  sample_body<COUNT, false, true, 256, false, false, 4, true>(kp);
}

// Schedule of the next sample_kernel launch: its n tiles by decreasing cost
// (the first-frame bounce counts the last launch recorded, bucketed on a
// quarter-octave log scale), so the launch's tail runs the cheapest tiles.
// Resets the costs for the next recording.  One block.  The order only
// decides which wave traces which samples, never a sample's value.
__device__ __forceinline__ int cost_bucket(uint32_t c) {
  const int b = (int)(__log2f((float)c + 1.0f) * 4.0f);
  return b < 63 ? b : 63;
}
__global__ __launch_bounds__(1024) void order_tiles_kernel(uint32_t* cost, uint32_t* order, int n) {
  __shared__ uint32_t hist[64];
  if (threadIdx.x < 64) hist[threadIdx.x] = 0;
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) atomicAdd(&hist[cost_bucket(cost[i])], 1u);
  __syncthreads();
  if (threadIdx.x == 0) {  // exclusive offsets, most expensive bucket first
    uint32_t s = 0;
    for (int b = 63; b >= 0; --b) {
      const uint32_t h = hist[b];
      hist[b] = s;
      s += h;
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    order[atomicAdd(&hist[cost_bucket(cost[i])], 1u)] = (uint32_t)i;
    cost[i] = 0u;
  }
}

// A launch's span record before the launch: {no start yet, no end yet}.
__global__ void span_init_kernel(unsigned long long* span) {
  if (threadIdx.x == 0) {
    span[0] = ~0ull;
    span[1] = 0ull;
  }
}

__global__ __launch_bounds__(256) void iota_kernel(uint32_t* order, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) order[i] = (uint32_t)i;
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
  uint32_t nan = 0;
  for (int k = 0; k < kp.nframes; ++k) {
    const float4 s = L[(size_t)k * (size_t)kp.local_pixels];
    acc = acc + mk(s.x, s.y, s.z);
    nan += ((s.x != s.x) | (s.y != s.y) | (s.z != s.z)) ? 1u : 0u;
  }
  kp.accum[li] = make_float4(acc.x, acc.y, acc.z, 1.0f);
  // failure detection: the reference tests a sample for NaN after accumulating it and
  // then discards the result (raytrace_compute.glsl:408-410); here it is counted
  if (nan) atomicAdd(kp.nan_ctr, (unsigned long long)nan);
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
// Stacks in LDS (stride = block), or in HBM when `gstk` is given (deep trees): each block
// has its own area of blockDim.x * 3 * stack_entries dwords, lane-interleaved within it, so
// the in-area index stays far below 2^31 for any ray count (the area's base is 64-bit).
__global__ __launch_bounds__(256) void closest_kernel(KParams kp, const srt_ray* rays, uint32_t n, uint32_t* hits,
                                                      float* tout, uint32_t* gstk) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Lane ln;
  ln.base = 0;
  ln.stk = gstk ? gstk + (size_t)blockIdx.x * blockDim.x * 3u * (uint32_t)kp.stack_entries + threadIdx.x
                : reinterpret_cast<uint32_t*>(g_smem) + threadIdx.x;
  ln.stride = (int)blockDim.x;
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
  // the hit record's input triangle index (its slot differs under LayoutTris)
  hits[i] = hit == 0xFFFFFFFFu ? hit : __float_as_uint(kp.tris[3 * (size_t)hit + 2].z);
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

// The multi-GPU root's per-frame step: every rank encoded its own rows' sRGB8 (accumFrames is one
// uniform for all), so the gather moves 4 B/px and the root only de-interleaves them.  Pixels outside
// the dispatch extent keep their old values, as a partial glDispatchCompute leaves them.
__global__ __launch_bounds__(256) void assemble_out_kernel(const uint32_t* gathered, int nranks, int rows_pad, int W,
                                                           int H, int band_rows, int ext_w, int ext_h, uint32_t* out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)W * (size_t)H) return;
  const int y = (int)(i / (size_t)W), x = (int)(i - (size_t)y * W);
  if (x >= ext_w || y >= ext_h) return;
  const int band = y / band_rows;
  const int r = band % nranks;
  const int ly = (band / nranks) * band_rows + (y - band * band_rows);
  out[i] = gathered[((size_t)r * rows_pad + ly) * W + x];
}

}  // namespace srt
