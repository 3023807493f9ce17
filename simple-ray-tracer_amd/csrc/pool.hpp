// pool.hpp -- the LDS-mode path-tracing kernel with cross-wave ray pools (DESIGN.md section 5,
// "Workgroup ray pools").
//
// sample_kernel keeps each path on one lane: a wave traverses until too few lanes still traverse,
// then shades the lanes whose ray returned.  In the metric frame only ~1 in 5 returned rays hit
// and need GetRayColor's full shading (the rest are sky, misses and shadow rays), so that shading
// code runs with ~7 of 64 lanes.  Here the 16 waves of the CU's block take two roles:
//   traversal waves (16 - kPoolShadeWaves) trace rays and start samples (batch claims, camera rays,
//     as sample_kernel's refill); shadow rays, misses and path ends are handled in the lane; a ray
//     that hits is deposited into a record in LDS and queued on the "shade" ring, and the lane takes
//     a shaded path's next ray from the "trace" ring (swapping it with the hit), or starts a sample;
//   shading waves run shade_hit on up to 64 queued hits at a time at full width, write each path's
//     next ray (shadow or bounce) into the same record and queue it on the trace ring; a record whose
//     path ended goes back to the "spare" ring.
// A record is a path's whole state between rays (28 dwords).  A hit that finds no traced ray to swap
// with deposits into a spare record.  Rings are lock-free (wave-aggregated LDS atomics, per-entry
// empty markers); no barrier is used after the setup.  Every path still runs the reference's
// arithmetic, one lane at a time, so the frame is bit-identical to sample_kernel's.  A watchdog ends
// every loop if the launch runs past kp.pool_deadline (s_memrealtime ticks) and flags ST_POOLERR.
#pragma once

#include "kernels.hpp"

namespace srt {
using namespace dev;

#ifndef SRT_POOL_SHADE
#define SRT_POOL_SHADE 2
#endif
constexpr int kPoolShadeWaves = SRT_POOL_SHADE;
constexpr int kPoolTravWaves = 16 - kPoolShadeWaves;
constexpr int kPoolTravLanes = 64 * kPoolTravWaves;
constexpr int kPoolRecF4 = 7;  // float4 per record
constexpr int kPollsMax = 16;  // idle polls (s_sleep 1 each) after which a shading wave takes a partial batch
constexpr uint32_t kRingEmpty = 0xFFFFFFFFu;
constexpr uint32_t kNoSlot = 0xFFFFFFFFu;
enum { kQShade = 0, kQTrace = 1, kQSpare = 2 };
// control words: head / tail / published count per ring, live paths, exhausted traversal waves, error
enum { PC_HEAD = 0, PC_TAIL = 3, PC_AVAIL = 6, PC_LIVE = 9, PC_EXH = 10, PC_ERR = 11, PC_WORDS = 12 };
// record flags: depth (bits 0-7), shadow ray, terminated after the shadow ray
constexpr uint32_t kFlagShadow = 1u << 8, kFlagTerm = 1u << 9;

// Diagnostic build (-DSRT_POOL_STATS): per-wave event counts and shader-clock cycles, summed into
// stats[ST_DBG_SUB + k] (tools/pool_check.py prints them).
enum { PD_T_OUTER = 0, PD_T_INNER, PD_T_ACTIVE, PD_T_IDLE, PD_T_SWAPPED, PD_T_HITS, PD_T_CYC_SWAP, PD_T_CYC_TRAV,
       PD_T_CYC_IDLE, PD_S_PASS, PD_S_POPPED, PD_S_DONE, PD_T_SPARE, PD_T_NEW, PD_S_IDLE, PD_S_CYC_BUSY, PD_S_CYC_IDLE,
       PD_T_WAIT, PD_T_C_RET, PD_T_C_POP, PD_T_C_SPARE, PD_T_C_REFILL, PD_T_C_START, PD_N };
#ifdef SRT_POOL_STATS
#define POOL_DBG(k, v) (dbg[k] += (unsigned long long)(v))
#define POOL_CLK() __builtin_amdgcn_s_memtime()
#else
#define POOL_DBG(k, v)
#define POOL_CLK() 0ull
#endif

struct Pool {
  uint32_t* ctl;
  uint32_t* ring;  // 3 rings of `cap` entries
  uint32_t mask;   // cap - 1
  uint32_t rec_off;  // byte offset of record 0 in LDS
  unsigned long long deadline;
#ifdef SRT_POOL_STATS
  unsigned long long dbg[PD_N];
#endif
};

// A path's state between rays (the registers sample_kernel keeps per lane), 7 float4 in LDS.
struct PathRec {
  f3 ro; float tmax;    // the ray to trace (a deposited hit: tmax holds the hit distance)
  f3 rd; uint32_t pix;  // pix = x | local row << 16
  f3 T; f3 color;
  int gy, fidx;         // global row, frame of the launch
  f3 q0; uint32_t flags;  // q0: direct light if occluded (a deposited hit: q0.x holds the triangle)
  f3 q1; int bounces;   // q1: direct light if visible
  f3 nd; int randIndex; // nd: the bounce direction after the shadow ray
};

__device__ __forceinline__ uint32_t vld(const uint32_t* p) { return *reinterpret_cast<const volatile uint32_t*>(p); }
__device__ __forceinline__ bool pool_expired(const Pool& P) {
  return __builtin_amdgcn_s_memrealtime() > P.deadline;
}
__device__ __forceinline__ void pool_fail(const KParams& kp, Pool& P) {
  if (atomicOr(&P.ctl[PC_ERR], 1u) == 0u &&
      atomicCAS(&kp.stats[ST_POOLERR], 0ull, 1ull + blockIdx.x) == 0ull) {  // the first block to fail:
    for (int k = 0; k < PC_WORDS; ++k)                                   // its control words, for diagnosis
      kp.stats[ST_DBG_SUB + 24 + k] = (unsigned long long)vld(&P.ctl[k]);
    kp.stats[ST_DBG_SUB + 24 + PC_WORDS] = threadIdx.x;
  }
}
__device__ __forceinline__ bool pool_error(const Pool& P) { return vld(&P.ctl[PC_ERR]) != 0u; }

__device__ __forceinline__ void rec_store(const Pool& P, uint32_t slot, const PathRec& r) {
  float4* q = reinterpret_cast<float4*>(reinterpret_cast<char*>(g_smem) + P.rec_off + __umul24(slot, 112u));
  q[0] = make_float4(r.ro.x, r.ro.y, r.ro.z, r.tmax);
  q[1] = make_float4(r.rd.x, r.rd.y, r.rd.z, __uint_as_float(r.pix));
  q[2] = make_float4(r.T.x, r.T.y, r.T.z, r.color.x);
  q[3] = make_float4(r.color.y, r.color.z, __int_as_float(r.gy), __int_as_float(r.fidx));
  q[4] = make_float4(r.q0.x, r.q0.y, r.q0.z, __uint_as_float(r.flags));
  q[5] = make_float4(r.q1.x, r.q1.y, r.q1.z, __int_as_float(r.bounces));
  q[6] = make_float4(r.nd.x, r.nd.y, r.nd.z, __int_as_float(r.randIndex));
}
__device__ __forceinline__ PathRec rec_load(const Pool& P, uint32_t slot) {
  const float4* q = reinterpret_cast<const float4*>(reinterpret_cast<const char*>(g_smem) + P.rec_off +
                                                    __umul24(slot, 112u));
  const float4 a = q[0], b = q[1], c = q[2], d = q[3], e = q[4], f = q[5], g = q[6];
  PathRec r;
  r.ro = mk(a.x, a.y, a.z); r.tmax = a.w;
  r.rd = mk(b.x, b.y, b.z); r.pix = __float_as_uint(b.w);
  r.T = mk(c.x, c.y, c.z); r.color = mk(c.w, d.x, d.y);
  r.gy = __float_as_int(d.z); r.fidx = __float_as_int(d.w);
  r.q0 = mk(e.x, e.y, e.z); r.flags = __float_as_uint(e.w);
  r.q1 = mk(f.x, f.y, f.z); r.bounces = __float_as_int(f.w);
  r.nd = mk(g.x, g.y, g.z); r.randIndex = __float_as_int(g.w);
  return r;
}
// Wave-level ring operations.  Every lane of the wave calls them (they ballot); `mine` / `want`
// select the lanes that push an id / ask for one.
__device__ __forceinline__ void ring_push(const KParams& kp, Pool& P, int q, bool mine, uint32_t id) {
  const unsigned long long m = __ballot(mine);
  if (m == 0ull) return;
  const int lane = threadIdx.x & 63;
  const int f = __ffsll((long long)m) - 1;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");  // the pushed records are written before their ids
  uint32_t t0 = 0;
  if (lane == f) t0 = atomicAdd(&P.ctl[PC_TAIL + q], (uint32_t)__popcll(m));
  t0 = __shfl(t0, f);
  if (mine) {
    // The entry may still hold an id of the previous lap that a consumer has claimed but not taken,
    // and a producer of a later lap may target it too: an atomic compare-and-swap from empty, so no
    // id is ever overwritten (whichever producer succeeds first, consumers of the entry take ids in
    // the order they are written; every claimed position has a producer, so each id is taken once).
    uint32_t* e = P.ring + (uint32_t)q * (P.mask + 1) + ((t0 + (uint32_t)lane_rank(m, lane)) & P.mask);
    while (atomicCAS(e, kRingEmpty, id) != kRingEmpty) {
      if (pool_expired(P)) { pool_fail(kp, P); break; }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if (lane == f) atomicAdd(&P.ctl[PC_AVAIL + q], (uint32_t)__popcll(m));
}

// Up to popcount(ballot(want)) published ids; the asking lane with rank r (0 .. k-1, distinct) gets
// the r-th if there are more than r, kNoSlot otherwise (and so do lanes that do not ask).  One lane
// reserves: a subtract from the published count (given back in part if it was short), then the
// positions from the head.
__device__ __forceinline__ uint32_t ring_pop_ranked(const KParams& kp, Pool& P, int q, bool want, uint32_t r) {
  const unsigned long long m = __ballot(want);
  if (m == 0ull) return kNoSlot;
  const int lane = threadIdx.x & 63;
  const int f = __ffsll((long long)m) - 1;
  uint32_t n = 0, h0 = 0;
  if (lane == f) {
    const uint32_t k = (uint32_t)__popcll(m);
    const int old = (int)atomicSub(&P.ctl[PC_AVAIL + q], k);  // may dip below zero for a moment
    n = old <= 0 ? 0u : ((uint32_t)old < k ? (uint32_t)old : k);
    if (n < k) atomicAdd(&P.ctl[PC_AVAIL + q], k - n);
    if (n) h0 = atomicAdd(&P.ctl[PC_HEAD + q], n);
  }
  n = __shfl(n, f);
  h0 = __shfl(h0, f);
  uint32_t id = kNoSlot;
  if (want && r < n) {
    // published, but the pusher of this position may not have written it yet: take the id with an
    // atomic exchange (never two consumers for one write)
    uint32_t* e = P.ring + (uint32_t)q * (P.mask + 1) + ((h0 + r) & P.mask);
    uint32_t v;
    while ((v = atomicExch(e, kRingEmpty)) == kRingEmpty) {
      if (pool_expired(P)) { pool_fail(kp, P); break; }
      __builtin_amdgcn_s_sleep(1);
    }
    id = v;
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  return id;
}
__device__ __forceinline__ uint32_t ring_pop(const KParams& kp, Pool& P, int q, bool want) {
  return ring_pop_ranked(kp, P, q, want, (uint32_t)lane_rank(__ballot(want), threadIdx.x & 63));
}

// wave-aggregated add to a control word
__device__ __forceinline__ void ctl_add(Pool& P, int w, bool mine, int sign) {
  const unsigned long long m = __ballot(mine);
  if (m == 0ull) return;
  if ((threadIdx.x & 63) == __ffsll((long long)m) - 1)
    atomicAdd(&P.ctl[w], (uint32_t)(sign * __popcll(m)));
}

__device__ __forceinline__ bool pool_done(const Pool& P) {
  return (vld(&P.ctl[PC_EXH]) == (uint32_t)kPoolTravWaves && vld(&P.ctl[PC_LIVE]) == 0u) || pool_error(P);
}

// The end of a path: color += T * skyColor (raytrace_compute.glsl:219,292) into the sample buffer,
// and the tile's cost for the next launch's order.
__device__ __forceinline__ void pool_finish(const KParams& kp, PathRec& r, int tiles_x) {
  const int x = (int)(r.pix & 0xFFFFu), ly = (int)(r.pix >> 16);
  if (SRT_TILE_SCHED && kp.tile_cost && r.fidx == 0)
    atomicAdd(&kp.tile_cost[(ly >> 3) * tiles_x + (x >> 3)], (uint32_t)(r.bounces + 1));
  r.color = r.color + r.T * mk(0.05f, 0.05f, 0.05f);
  kp.lbuf[(size_t)r.fidx * (size_t)kp.local_pixels + (size_t)(ly * kp.W + x)] =
      make_float4(r.color.x, r.color.y, r.color.z, 0.0f);
}

// ---------------------------------------------------------------------------
// traversal waves
// ---------------------------------------------------------------------------
template <bool COUNT>
__device__ __forceinline__ void pool_trace(const KParams& kp, Pool& P, Counters& c) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int tiles_x = (kp.W + 7) >> 3;
  const int n_tiles = tiles_x * ((kp.local_rows + 7) >> 3);
  const int n_batches = n_tiles * kp.nframes;  // < 2^31: the host bounds the frames per launch
  const f3 center = mk(kp.cx, kp.cy, kp.cz);
  Lane ln;
  ln.stk = reinterpret_cast<uint32_t*>(g_smem + kp.stack_base_f4) + tid;
  ln.stride = kPoolTravLanes;  // a compile-time stride (traversal lanes are threads 0 .. kPoolTravLanes - 1)
  ln.base = 0;
  // batch claims, as sample_kernel makes them (kClaim batches per atomic, one claim ahead)
  uint32_t claimed = 0;
  int claim_sz = kp.tail_start > 0 ? kClaim : 1;
  if (lane == 0) claimed = atomicAdd(kp.batch_ctr, (uint32_t)claim_sz);
  int batch = __builtin_amdgcn_readfirstlane((int)__shfl(claimed, 0));
  int claim_left = claim_sz - 1;
  claim_sz = batch < kp.tail_start ? kClaim : 1;
  if (lane == 0) claimed = atomicAdd(kp.batch_ctr, (uint32_t)claim_sz);
  int batch_next = 0;
  bool exhausted = false;
  PathRec pr;
  bool has = false, waiting = false;
  Trav tr;
  tr.active = false;
  tr.start = false;
  tr.hit = kNoneRef;
#ifdef SRT_POOL_STATS
  unsigned long long* dbg = P.dbg;
#endif
  for (;;) {
    [[maybe_unused]] const unsigned long long clk0 = POOL_CLK();
    POOL_DBG(PD_T_OUTER, 1);
    // ---- rays that returned: shadow rays and misses end here; hits wait for a record ----
    bool fin = false, restart = false;
    if (has && !tr.active && !waiting) {
      const bool hit = tr.hit != kNoneRef;
      if (pr.flags & kFlagShadow) {  // CheckLightOccluded returned: this bounce's direct light
        pr.color = pr.color + (hit ? pr.q0 : pr.q1);
        if (pr.flags & kFlagTerm) {
          fin = true;
        } else {  // the bounce ray starts at the same hit point
          pr.rd = pr.nd;
          pr.tmax = __builtin_inff();
          pr.flags &= ~kFlagShadow;
          restart = true;
        }
      } else if (!hit) {
        fin = true;
      } else {
        waiting = true;
        pr.q0.x = __uint_as_float(tr.hit);
        pr.tmax = tr.dist;
      }
    }
    if (fin) {
      pool_finish(kp, pr, tiles_x);
      has = false;
    }
    ctl_add(P, PC_LIVE, fin, -1);
    POOL_DBG(PD_T_HITS, __popcll(__ballot(waiting)));
    [[maybe_unused]] unsigned long long clk_s = POOL_CLK();
    POOL_DBG(PD_T_C_RET, clk_s - clk0);
    // ---- one pop from the trace ring: hits first (each swaps its record with a shaded path's next
    // ray), then empty lanes (the record they empty goes to the spare ring) ----
    {
      const unsigned long long wm = __ballot(waiting), em = __ballot(!has);
      const bool ask = waiting || !has;
      if ((wm | em) != 0ull &&
          (wm != 0ull || __builtin_amdgcn_readfirstlane(vld(&P.ctl[PC_AVAIL + kQTrace])) != 0u)) {
        const uint32_t rk = waiting ? (uint32_t)lane_rank(wm, lane) : (uint32_t)(__popcll(wm) + lane_rank(em, lane));
        const uint32_t id = ring_pop_ranked(kp, P, kQTrace, ask, rk);
        const bool got = id != kNoSlot, swapped = got && waiting;
        if (got) {
          const PathRec in = rec_load(P, id);
          if (waiting) rec_store(P, id, pr);
          pr = in;
          has = true;
          waiting = false;
          restart = true;
        }
        ring_push(kp, P, kQShade, swapped, id);
        ring_push(kp, P, kQSpare, got && !swapped, id);
        POOL_DBG(PD_T_SWAPPED, __popcll(__ballot(got)));
      }
    }
    POOL_DBG(PD_T_C_POP, POOL_CLK() - clk_s);
    clk_s = POOL_CLK();
    // ---- hits with no ray to swap with: a spare record ----
    if (__ballot(waiting) != 0ull) {
      const uint32_t sid = ring_pop(kp, P, kQSpare, waiting);
      const bool dep = sid != kNoSlot;
      if (dep) {
        rec_store(P, sid, pr);
        waiting = false;
        has = false;
      }
      ring_push(kp, P, kQShade, dep, sid);
      POOL_DBG(PD_T_SPARE, __popcll(__ballot(dep)));
    }
    POOL_DBG(PD_T_C_SPARE, POOL_CLK() - clk_s);
    clk_s = POOL_CLK();
    bool fresh = false;
    int a_pl = 0, a_gy = 0, a_f = 0, a_samp = 0;
    for (;;) {  // the refill of sample_kernel: idle lanes take the next items of the wave's batches
      const unsigned long long idle = __ballot(!has & !fresh);
      if (idle == 0ull || batch >= n_batches) break;
      const int avail = 64 - batch_next;
      const int r = lane_rank(idle, lane);
      const int frame_i = batch / n_tiles;
      const int trank = batch - frame_i * n_tiles;
#if SRT_TILE_SCHED
      const int tile = (int)((const __attribute__((address_space(4))) uint32_t*)(kp.tile_order))[trank];
#else
      const int tile = trank;
#endif
      const int ty = tile / tiles_x, tx = tile - ty * tiles_x;
      const int samp = (kp.frame_first + frame_i) % kp.WH;
      if (!has & !fresh & (r < avail)) {
        const int item = batch_next + r;
        const int px = tx * 8 + (item & 7), ly = ty * 8 + (item >> 3);
        if (px < kp.ext_w && ly < kp.local_rows) {
          int yy = ly;
          if (kp.nranks > 1) yy = kp.row_map[ly];  // the row band's global row (as sample_kernel)
          if (yy < kp.ext_h) {
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
          claim_sz = batch < kp.tail_start ? kClaim : 1;
          if (lane == 0) claimed = atomicAdd(kp.batch_ctr, (uint32_t)claim_sz);
        }
        batch_next = 0;
      }
    }
    ctl_add(P, PC_LIVE, fresh, +1);
    POOL_DBG(PD_T_NEW, __popcll(__ballot(fresh)));
    if (fresh) {
      const int x = a_pl & 0xFFFF;
      ln.base = a_gy * kp.H + x;
      // GetRay (raytrace_compute.glsl:78-90) with SampleSquare (raytrace_utils.glsl:10-17)
      const float2 nz = kp.noise_xy[wrap_index(ln.base + a_samp, kp.WH)];
      bump<COUNT>(c, ST_RNGSQ);
      bump<COUNT>(c, ST_SAMPLES);
      const f3 p00 = mk(kp.p00x, kp.p00y, kp.p00z);
      const f3 du = mk(kp.dux, kp.duy, kp.duz);
      const f3 dv = mk(kp.dvx, kp.dvy, kp.dvz);
      const f3 ps = (p00 + du * ((float)x + (nz.x - 0.5f))) + dv * ((float)a_gy + (nz.y - 0.5f));
      pr.ro = center;
      pr.rd = ps - center;
      pr.tmax = __builtin_inff();
      pr.pix = (uint32_t)a_pl;
      pr.T = mk(1.0f, 1.0f, 1.0f);
      pr.color = mk(0.0f, 0.0f, 0.0f);
      pr.gy = a_gy;
      pr.fidx = a_f;
      pr.flags = (uint32_t)kp.max_depth;
      pr.bounces = 0;
      pr.randIndex = 0;
      has = true;
      restart = true;
    }
    if (!exhausted && batch >= n_batches) {
      exhausted = true;
      if (lane == 0) atomicAdd(&P.ctl[PC_EXH], 1u);
    }
    POOL_DBG(PD_T_C_REFILL, POOL_CLK() - clk_s);
    clk_s = POOL_CLK();
    // ---- start the rays (new samples, shadow-to-bounce, rays taken from the trace ring) ----
    if (restart) {
      ln.base = pr.gy * kp.H + (int)(pr.pix & 0xFFFFu);
      tr.dist = pr.tmax;
      tr.hit = kNoneRef;
      tr.bi = 0;
      tr.active = true;
      tr.start = false;
      bump<COUNT>(c, ST_RAYS);
      bump<COUNT>(c, ST_SHADOW, (pr.flags & kFlagShadow) ? 1u : 0u);
      trav_begin_bvh<COUNT, true>(kp, c, tr, pr.ro, pr.rd);
      if (tr.cnt == kNoneCnt) {  // root box missed: next BVH, or done
        if (kp.bvh_count > 1) tr.start = true, tr.bi = 1;
        else tr.active = false;
      }
    }
    [[maybe_unused]] const unsigned long long clk1 = POOL_CLK();
    POOL_DBG(PD_T_C_START, clk1 - clk_s);
    POOL_DBG(PD_T_CYC_SWAP, clk1 - clk0);
    const unsigned long long trav0 = __ballot(tr.active);
    if (trav0 == 0ull) {
      if (__ballot(has) == 0ull) {  // nothing left in this wave's batches
        if (pool_done(P)) break;
      } else if (__ballot(has && !waiting) != 0ull) {
        continue;  // rays that ended at their root box: handled at once
      }
      if (pool_expired(P)) { pool_fail(kp, P); break; }
      __builtin_amdgcn_s_sleep(2);  // hits waiting for a record, or other waves' paths still live
      POOL_DBG(PD_T_IDLE, 1);
      POOL_DBG(PD_T_CYC_IDLE, POOL_CLK() - clk1);
      continue;
    }
    // ---- traverse until too few lanes are still traversing ----
    const int work_lim = __popcll(__ballot(has)) * kp.trav_frac16;
    for (;;) {
      const unsigned long long trav = __ballot(tr.active);
      if (trav == 0ull || __popcll(trav) * 16 < work_lim) break;
      POOL_DBG(PD_T_INNER, 1);
      POOL_DBG(PD_T_ACTIVE, __popcll(trav));
      if (tr.active) trav_step<COUNT, true, true, false>(kp, ln, c, tr, pr.ro, pr.rd, (pr.flags & kFlagShadow) != 0u);
    }
    POOL_DBG(PD_T_WAIT, __popcll(__ballot(waiting)));
    POOL_DBG(PD_T_CYC_TRAV, POOL_CLK() - clk1);
    if (pool_error(P)) break;
  }
}

// ---------------------------------------------------------------------------
// shading waves
// ---------------------------------------------------------------------------
template <bool COUNT>
__device__ __forceinline__ void pool_shade(const KParams& kp, Pool& P, Counters& c) {
  const int tiles_x = (kp.W + 7) >> 3;
  Lane ln;
  ln.stk = nullptr;
  ln.stride = 0;
  ln.base = 0;
#ifdef SRT_POOL_STATS
  unsigned long long* dbg = P.dbg;
#endif
  int polls = 0;  // idle polls since the last pass
  for (;;) {
    [[maybe_unused]] const unsigned long long clk0 = POOL_CLK();
    // a full batch of hits; or what there is when the traversal waves may run out of records, when
    // every live path is queued, or after kPollsMax idle polls (the batch is not filling up)
    const uint32_t sa = __builtin_amdgcn_readfirstlane(vld(&P.ctl[PC_AVAIL + kQShade]));
    const uint32_t ta = __builtin_amdgcn_readfirstlane(vld(&P.ctl[PC_AVAIL + kQTrace]));
    const uint32_t fa = __builtin_amdgcn_readfirstlane(vld(&P.ctl[PC_AVAIL + kQSpare]));
    const uint32_t live = __builtin_amdgcn_readfirstlane(vld(&P.ctl[PC_LIVE]));
    const bool go = sa >= (uint32_t)kp.pool_batch ||
                    (sa > 0u && (ta + fa < (uint32_t)kp.pool_tlow || sa + ta >= live || polls >= kPollsMax));
    ++polls;
    if (!go) {
      if (sa == 0u && pool_done(P)) break;
      if (pool_expired(P)) { pool_fail(kp, P); break; }
      __builtin_amdgcn_s_sleep(1);
      POOL_DBG(PD_S_IDLE, 1);
      POOL_DBG(PD_S_CYC_IDLE, POOL_CLK() - clk0);
      continue;
    }
    polls = 0;
    const uint32_t id = ring_pop(kp, P, kQShade, true);
    const bool mine = id != kNoSlot;
    POOL_DBG(PD_S_PASS, 1);
    POOL_DBG(PD_S_POPPED, __popcll(__ballot(mine)));
    bool done = false;
    if (mine) {  // GetRayColor's loop body for the hit
      PathRec pr = rec_load(P, id);
      ln.base = pr.gy * kp.H + (int)(pr.pix & 0xFFFFu);
      int depth = (int)(pr.flags & 0xFFu);
      bool term = false;
      const uint32_t ht = __float_as_uint(pr.q0.x);
      float tmax = 0.0f;
      const int next = shade_hit<COUNT, true, false>(kp, ln, c, ht, -1, pr.tmax, pr.ro, pr.rd, tmax, pr.T, depth,
                                                     pr.randIndex, pr.bounces, term, pr.q0, pr.q1, pr.nd);
      pr.tmax = tmax;
      if (next == kShadeDone) {
        pool_finish(kp, pr, tiles_x);
        done = true;
      } else {
        pr.flags = (uint32_t)depth | (next == kShadeShadow ? kFlagShadow : 0u) | (term ? kFlagTerm : 0u);
        rec_store(P, id, pr);
      }
    }
    ctl_add(P, PC_LIVE, done, -1);
    POOL_DBG(PD_S_DONE, __popcll(__ballot(done)));
    ring_push(kp, P, kQTrace, mine & !done, id);
    ring_push(kp, P, kQSpare, done, id);
    POOL_DBG(PD_S_CYC_BUSY, POOL_CLK() - clk0);
    if (pool_error(P)) break;
  }
}

template <bool COUNT>
__global__ __launch_bounds__(1024, 4) void pool_kernel(KParams kp) {
  const int tid = threadIdx.x;
  for (int i = tid; i < kp.nodes_f4; i += blockDim.x) g_smem[node_lds_f4((uint32_t)i)] = kp.nodes[i];
  for (int i = tid; i < kp.tris_f4; i += blockDim.x) g_smem[kp.nodes_lds_f4 + i] = kp.tris[i];
  {
    const int nl = kp.lights_lds ? 2 * (kp.light_records + 1) : 0, nm = kp.mats_lds ? 2 * kp.mat_records : 0;
    for (int i = tid; i < nl; i += blockDim.x) g_smem[kp.lights_base_f4 + i] = kp.lights[i];
    for (int i = tid; i < nm; i += blockDim.x) g_smem[kp.mats_base_f4 + i] = kp.mats[i];
  }
  Pool P;
  P.ctl = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(g_smem) + kp.pool_ctl_off);
  P.ring = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(g_smem) + kp.pool_ring_off);
  P.mask = (uint32_t)kp.pool_cap - 1u;
  P.rec_off = (uint32_t)kp.pool_rec_off;
  P.deadline = __builtin_amdgcn_s_memrealtime() + kp.pool_deadline;
  // every record starts in the spare ring
  for (int i = tid; i < PC_WORDS; i += blockDim.x) P.ctl[i] = 0u;
  for (int i = tid; i < 3 * kp.pool_cap; i += blockDim.x) {
    const int q = i / kp.pool_cap, k = i - q * kp.pool_cap;
    P.ring[i] = (q == kQSpare && k < kp.pool_slots) ? (uint32_t)k : kRingEmpty;
  }
  __syncthreads();
  if (tid == 0) {
    P.ctl[PC_TAIL + kQSpare] = (uint32_t)kp.pool_slots;
    P.ctl[PC_AVAIL + kQSpare] = (uint32_t)kp.pool_slots;
  }
  __syncthreads();
  Counters c;
  for (int k = 0; k < ST_N; ++k) c.v[k] = 0;
#ifdef SRT_POOL_STATS
  for (int k = 0; k < PD_N; ++k) P.dbg[k] = 0;
#endif
  if (tid < kPoolTravLanes) pool_trace<COUNT>(kp, P, c);
  else pool_shade<COUNT>(kp, P, c);
  flush_counters<COUNT>(kp, c);
#ifdef SRT_POOL_STATS
  if ((tid & 63) == 0)
    for (int k = 0; k < PD_N; ++k) atomicAdd(&kp.stats[ST_DBG_SUB + k], P.dbg[k]);
#endif
}

}  // namespace srt
