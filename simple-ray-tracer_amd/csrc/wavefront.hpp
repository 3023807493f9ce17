// wavefront.hpp -- global-scene mode as a wavefront of kernels ("Wavefront mode").
//
// sample_kernel keeps each path on one lane for its whole life: traversal, shading and the refill share
// one register allocation (the shading code sets it, ~111 VGPRs, 4-5 waves per SIMD), and hit shading
// runs with the few lanes whose ray hit.  Here a launch's samples flow through a pool of path slots in
// HBM, one iteration at a time, in three kernels:
//   wf_logic_kernel  one thread per slot: a ray that returned ends its shadow test (the direct light of
//                    the bounce, raytrace_compute.glsl:233-246), ends the path on a miss (:219,292), or
//                    queues the slot for shading on a hit; an empty slot takes the launch's next sample
//                    and sets up its camera ray (GetRay, :78-90).  Live rays are compacted into the ray
//                    queue and hits into the hit queue by a wave ballot + prefix count + one atomic;
//   wf_shade_kernel  one thread per queued hit: GetRayColor's loop body (shade_hit, :225-290) at full
//                    width; the path's next ray (shadow or bounce) joins the ray queue;
//   wf_trace_kernel  persistent: lanes take queued rays (ballot refill), run CheckHit (the resumable,
//                    order-exact traversal of traversal.hpp) and write (hit triangle, distance) back.
//                    It holds only traversal state, so it runs at more waves per SIMD than sample_kernel.
// Every path runs the reference's arithmetic on one thread at a time, so the samples -- stored to the
// sample buffer and summed per pixel in frame order by accumulate_kernel -- are bit-identical to
// sample_kernel's.
#pragma once

#include "kernels.hpp"

namespace srt {
using namespace dev;

// slot states
enum : uint32_t { WF_EMPTY = 0u, WF_TRACE = 1u, WF_RET = 2u, WF_HIT = 3u, WF_NONE = 0xFFu };
// control words of one iteration: ray queue length, hit queue length, the trace (or top) kernel's claim
// counter, slots live after the logic kernel; treelet scheduling: rays suspended at treelet roots, the
// bottom kernel's claim counter, rays it hands back to the next iteration's top kernel
enum { WQ_RAYS = 0, WQ_HITS = 1, WQ_CLAIM = 2, WQ_LIVE = 3, WQ_SUSP = 4, WQ_BCLAIM = 5, WQ_RES = 6, WQ_WORDS = 8 };
constexpr uint32_t kWfShadowBit = 0x80000000u;  // ray queue entry: slot | shadow ray
constexpr uint32_t kWfFlagShadow = 1u << 8, kWfFlagTerm = 1u << 9;  // record flags: depth (bits 0-7) | these

struct WfParams {
  float4* rec;      // path records, 7 float4 per slot, field-major: field k of slot s at rec[k * slots + s]
  uint2* res;       // the traced ray's result per slot: (hit triangle or kNoneRef, distance bits)
  uint32_t* state;  // per slot (WF_*)
  uint32_t* rayq;   // slots whose ray is traced this iteration (| kWfShadowBit for a shadow ray)
  uint32_t* hitq;   // slots whose ray hit, shaded this iteration
  uint32_t* ctl;    // WQ_WORDS per iteration
  uint32_t* items;  // the launch's next unclaimed sample item (64 per 8x8-tile batch)
  uint32_t slots;
  uint32_t n_items;
  int iter;
  // treelet scheduling (wf_top_kernel / wf_bottom_kernel)
  float4* tray;        // a suspended ray, 4 float4 per slot, field-major (wf_tray)
  uint32_t* tstk;      // its top-level stack entries, kTopStack x 3 dwords per slot
  uint32_t* slist;     // rays suspended this iteration (slots) and their treelets
  uint32_t* skey;
  uint32_t* blist;     // the same rays grouped by treelet (wf_scatter_kernel)
  uint32_t* rlist[2];  // rays the bottom kernel of iteration i hands to the top kernel of i + 1: rlist[i & 1]
  uint32_t* tcount;    // per treelet: rays suspended at it this iteration / scatter cursor
  uint32_t* tfill;
  const uint32_t* troot;  // per treelet: its root's child index in the real node array
  uint32_t n_treelets;
};

// The path state between rays (sample_kernel's per-lane registers), 7 float4:
//   0 (ro, tmax)  1 (rd, pix)  2 (T, color.x)  3 (color.y, color.z, gy, fidx)
//   4 (q0, flags) 5 (q1, bounces)  6 (nd, randIndex)
// q0/q1: the direct light if occluded / visible; a queued hit keeps its triangle in q0.x and its distance
// in tmax; pix = x | local row << 16.
struct WfPath {
  f3 ro; float tmax;
  f3 rd; uint32_t pix;
  f3 T, color;
  int gy, fidx;
  f3 q0; uint32_t flags;
  f3 q1; int bounces;
  f3 nd; int randIndex;
};

__device__ __forceinline__ float4* wf_field(const WfParams& w, int k, uint32_t s) {
  return w.rec + (size_t)k * w.slots + s;
}
__device__ __forceinline__ WfPath wf_load(const WfParams& w, uint32_t s) {
  const float4 a = *wf_field(w, 0, s), b = *wf_field(w, 1, s), c = *wf_field(w, 2, s), d = *wf_field(w, 3, s),
               e = *wf_field(w, 4, s), f = *wf_field(w, 5, s), g = *wf_field(w, 6, s);
  WfPath r;
  r.ro = mk(a.x, a.y, a.z); r.tmax = a.w;
  r.rd = mk(b.x, b.y, b.z); r.pix = __float_as_uint(b.w);
  r.T = mk(c.x, c.y, c.z); r.color = mk(c.w, d.x, d.y);
  r.gy = __float_as_int(d.z); r.fidx = __float_as_int(d.w);
  r.q0 = mk(e.x, e.y, e.z); r.flags = __float_as_uint(e.w);
  r.q1 = mk(f.x, f.y, f.z); r.bounces = __float_as_int(f.w);
  r.nd = mk(g.x, g.y, g.z); r.randIndex = __float_as_int(g.w);
  return r;
}
__device__ __forceinline__ void wf_store(const WfParams& w, uint32_t s, const WfPath& r) {
  *wf_field(w, 0, s) = make_float4(r.ro.x, r.ro.y, r.ro.z, r.tmax);
  *wf_field(w, 1, s) = make_float4(r.rd.x, r.rd.y, r.rd.z, __uint_as_float(r.pix));
  *wf_field(w, 2, s) = make_float4(r.T.x, r.T.y, r.T.z, r.color.x);
  *wf_field(w, 3, s) = make_float4(r.color.y, r.color.z, __int_as_float(r.gy), __int_as_float(r.fidx));
  *wf_field(w, 4, s) = make_float4(r.q0.x, r.q0.y, r.q0.z, __uint_as_float(r.flags));
  *wf_field(w, 5, s) = make_float4(r.q1.x, r.q1.y, r.q1.z, __int_as_float(r.bounces));
  *wf_field(w, 6, s) = make_float4(r.nd.x, r.nd.y, r.nd.z, __int_as_float(r.randIndex));
}

// Wave-aggregated append: the lanes with `mine` write `v` to consecutive entries of `q` (one atomic on
// the queue's length per wave: the ballot + prefix count that compacts the wave's live rays).
__device__ __forceinline__ void wf_append(uint32_t* len, uint32_t* q, bool mine, uint32_t v) {
  const unsigned long long m = __ballot(mine);
  if (m == 0ull) return;
  const int lane = threadIdx.x & 63;
  const int f = __ffsll((long long)m) - 1;
  uint32_t base = 0;
  if (lane == f) base = atomicAdd(len, (uint32_t)__popcll(m));
  base = __shfl(base, f);
  if (mine) q[base + (uint32_t)lane_rank(m, lane)] = v;
}

// The end of a path: color += T * skyColor (raytrace_compute.glsl:219,292) into the sample buffer, and
// the tile's cost for the next launch's order (as sample_kernel's finish_sample).
__device__ __forceinline__ void wf_finish(const KParams& kp, WfPath& r) {
  const int x = (int)(r.pix & 0xFFFFu), ly = (int)(r.pix >> 16);
  if (SRT_TILE_SCHED && kp.tile_cost && r.fidx == 0)
    atomicAdd(&kp.tile_cost[(ly >> 3) * ((kp.W + 7) >> 3) + (x >> 3)], (uint32_t)(r.bounces + 1));
  r.color = r.color + r.T * mk(0.05f, 0.05f, 0.05f);
  kp.lbuf[(size_t)r.fidx * (size_t)kp.local_pixels + (size_t)(ly * kp.W + x)] =
      make_float4(r.color.x, r.color.y, r.color.z, 0.0f);
}

// Sample item -> pixel, as sample_kernel's refill maps its batches: item = batch * 64 + k, batch =
// frame * n_tiles + rank of the tile in the launch's tile order, k the pixel within the 8x8 tile.
// False for an item outside the dispatch extent (the slot then takes none this iteration).
__device__ __forceinline__ bool wf_item_pixel(const KParams& kp, uint32_t item, int& pl, int& gy, int& f, int& samp) {
  const int tiles_x = (kp.W + 7) >> 3;
  const int n_tiles = tiles_x * ((kp.local_rows + 7) >> 3);
  const int batch = (int)(item >> 6), k = (int)(item & 63u);
  const int frame_i = batch / n_tiles;
  const int trank = batch - frame_i * n_tiles;
#if SRT_TILE_SCHED
  const int tile = (int)kp.tile_order[trank];
#else
  const int tile = trank;
#endif
  const int ty = tile / tiles_x, tx = tile - ty * tiles_x;
  const int px = tx * 8 + (k & 7), ly = ty * 8 + (k >> 3);
  if (px >= kp.ext_w || ly >= kp.local_rows) return false;
  int yy = ly;
  if (kp.nranks > 1) yy = kp.row_map[ly];  // the row band's global row
  if (yy >= kp.ext_h) return false;
  pl = px | (ly << 16);
  gy = yy;
  f = frame_i;
  samp = (kp.frame_first + frame_i) % kp.WH;
  return true;
}

// ---------------------------------------------------------------------------
// the logic kernel: one thread per slot
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void wf_logic_kernel(KParams kp, WfParams w) {
  const uint32_t s = blockIdx.x * 256u + threadIdx.x;
  const bool valid = s < w.slots;
  uint32_t* ctl = w.ctl + (size_t)WQ_WORDS * (size_t)w.iter;
  const int lane = threadIdx.x & 63;
  uint32_t st = valid ? w.state[s] : (uint32_t)WF_NONE;
  bool want = st == WF_EMPTY, trace = false, shade = false;  // (only wf_shade_kernel starts shadow rays)
  if (st == WF_RET) {
    WfPath r = wf_load(w, s);
    const uint2 res = w.res[s];
    const bool hit = res.x != kNoneRef;
    if (r.flags & kWfFlagShadow) {  // CheckLightOccluded returned: this bounce's direct light
      r.color = r.color + (hit ? r.q0 : r.q1);
      if (r.flags & kWfFlagTerm) {
        wf_finish(kp, r);
        want = true;
      } else {  // the bounce ray starts at the same hit point
        r.rd = r.nd;
        r.tmax = __builtin_inff();
        r.flags &= ~kWfFlagShadow;
        wf_store(w, s, r);
        trace = true;
      }
    } else if (!hit) {
      wf_finish(kp, r);
      want = true;
    } else {
      r.q0.x = __uint_as_float(res.x);
      r.tmax = __uint_as_float(res.y);
      wf_store(w, s, r);
      shade = true;
    }
  }
  // empty slots take the launch's next samples (consecutive items per wave, one atomic)
  {
    const unsigned long long m = __ballot(want);
    if (m != 0ull) {
      const int f = __ffsll((long long)m) - 1;
      uint32_t base = 0;
      if (lane == f) base = *reinterpret_cast<volatile uint32_t*>(w.items) < w.n_items
                                ? atomicAdd(w.items, (uint32_t)__popcll(m)) : w.n_items;
      base = __shfl(base, f);
      if (want) {
        const uint32_t item = base + (uint32_t)lane_rank(m, lane);
        int pl = 0, gy = 0, fi = 0, samp = 0;
        if (item < w.n_items && wf_item_pixel(kp, item, pl, gy, fi, samp)) {
          const int x = pl & 0xFFFF;
          // GetRay (raytrace_compute.glsl:78-90) with SampleSquare (raytrace_utils.glsl:10-17)
          const float2 nz = kp.noise_xy[wrap_index(gy * kp.H + x + samp, kp.WH)];
          const f3 p00 = mk(kp.p00x, kp.p00y, kp.p00z);
          const f3 du = mk(kp.dux, kp.duy, kp.duz);
          const f3 dv = mk(kp.dvx, kp.dvy, kp.dvz);
          const f3 ps = (p00 + du * ((float)x + (nz.x - 0.5f))) + dv * ((float)gy + (nz.y - 0.5f));
          WfPath r;
          r.ro = mk(kp.cx, kp.cy, kp.cz);
          r.rd = ps - r.ro;
          r.tmax = __builtin_inff();
          r.pix = (uint32_t)pl;
          r.T = mk(1.0f, 1.0f, 1.0f);
          r.color = mk(0.0f, 0.0f, 0.0f);
          r.gy = gy;
          r.fidx = fi;
          r.q0 = r.q1 = r.nd = mk(0.0f, 0.0f, 0.0f);
          r.flags = (uint32_t)kp.max_depth & 0xFFu;
          r.bounces = 0;
          r.randIndex = 0;
          wf_store(w, s, r);
          trace = true;
        }
      }
    }
  }
  if (valid) {
    if (trace) w.state[s] = WF_TRACE;
    else if (shade) w.state[s] = WF_HIT;
    else if (st == WF_RET || want) w.state[s] = WF_EMPTY;
  }
  wf_append(&ctl[WQ_RAYS], w.rayq, trace, s);
  wf_append(&ctl[WQ_HITS], w.hitq, shade, s);
  const unsigned long long live = __ballot(trace || shade || (valid && st == WF_TRACE) || (valid && st == WF_HIT));
  if (live != 0ull && lane == __ffsll((long long)live) - 1) atomicAdd(&ctl[WQ_LIVE], (uint32_t)__popcll(live));
}

// ---------------------------------------------------------------------------
// the shading kernel: one thread per queued hit
// ---------------------------------------------------------------------------
template <bool TEX>
__global__ __launch_bounds__(256) void wf_shade_kernel(KParams kp, WfParams w) {
  uint32_t* ctl = w.ctl + (size_t)WQ_WORDS * (size_t)w.iter;
  const uint32_t n = *reinterpret_cast<volatile uint32_t*>(&ctl[WQ_HITS]);
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (blockIdx.x * 256u >= n) return;  // whole block past the queue
  const bool mine = i < n;
  bool next_ray = false, shadow = false;
  uint32_t s = 0;
  if (mine) {
    s = w.hitq[i];
    WfPath r = wf_load(w, s);
    Lane ln;
    ln.stk = nullptr;
    ln.stride = 0;
    ln.gstk = nullptr;
    ln.gstride = 0;
    ln.base = r.gy * kp.H + (int)(r.pix & 0xFFFFu);
    Counters c;
    int depth = (int)(r.flags & 0xFFu);
    bool term = false;
    float tmax = 0.0f;
    const int next = shade_hit<false, false, TEX>(kp, ln, c, __float_as_uint(r.q0.x), -1, r.tmax, r.ro, r.rd, tmax,
                                                  r.T, depth, r.randIndex, r.bounces, term, r.q0, r.q1, r.nd);
    r.tmax = tmax;
    if (next == kShadeDone) {
      wf_finish(kp, r);
      w.state[s] = WF_EMPTY;
    } else {
      shadow = next == kShadeShadow;
      r.flags = ((uint32_t)depth & 0xFFu) | (shadow ? kWfFlagShadow : 0u) | (term ? kWfFlagTerm : 0u);
      wf_store(w, s, r);
      w.state[s] = WF_TRACE;
      next_ray = true;
    }
  }
  wf_append(&ctl[WQ_RAYS], w.rayq, next_ray, s | (shadow ? kWfShadowBit : 0u));
}

// ---------------------------------------------------------------------------
// the trace kernel: persistent; lanes take queued rays and run CheckHit
// (raytrace_compute.glsl:143-162) with sample_kernel's resumable traversal
// ---------------------------------------------------------------------------
template <bool PACK, bool FUSE, int GW>
__global__ __launch_bounds__(256, GW) void wf_trace_kernel(KParams kp, WfParams w) {
  constexpr int RING = global_ring(GW);
  const int tid = threadIdx.x, lane = tid & 63;
  uint32_t* ctl = w.ctl + (size_t)WQ_WORDS * (size_t)w.iter;
  const uint32_t n = *reinterpret_cast<volatile uint32_t*>(&ctl[WQ_RAYS]);
  Lane ln;
  ln.stk = reinterpret_cast<uint32_t*>(g_smem) + tid;
  ln.stride = 256;
  ln.gstk = kp.gstack + (size_t)blockIdx.x * 256 + tid;
  ln.gstride = kp.gstack_stride;
  ln.base = 0;
  Counters c;
  Trav tr;
  tr.active = false;
  tr.start = false;
  tr.hit = kNoneRef;
  tr.dist = 0.0f;
  f3 ro = mk(0.f, 0.f, 0.f), rd = mk(0.f, 0.f, 1.f);
  bool has = false, shadow = false, exhausted = false;
  uint32_t s = 0;
  for (;;) {
    // lanes without a ray take the next queued ones
    const unsigned long long idle = __ballot(!has);
    if (idle != 0ull && !exhausted) {
      const int f = __ffsll((long long)idle) - 1;
      uint32_t base = 0;
      if (lane == f) base = atomicAdd(&ctl[WQ_CLAIM], (uint32_t)__popcll(idle));
      base = __builtin_amdgcn_readfirstlane(__shfl(base, f));
      if (base + (uint32_t)__popcll(idle) >= n) exhausted = true;
      if (!has) {
        const uint32_t pos = base + (uint32_t)lane_rank(idle, lane);
        if (pos < n) {
          const uint32_t e = w.rayq[pos];
          s = e & ~kWfShadowBit;
          shadow = (e & kWfShadowBit) != 0u;
          const float4 a = *wf_field(w, 0, s), b = *wf_field(w, 1, s);
          ro = mk(a.x, a.y, a.z);
          rd = mk(b.x, b.y, b.z);
          has = true;
          tr.dist = a.w;
          tr.hit = kNoneRef;
          tr.bi = 0;
          tr.active = true;
          tr.start = false;
          trav_begin_bvh<false, false>(kp, c, tr, ro, rd);
          if (tr.cnt == kNoneCnt) {  // root box missed: next BVH, or done
            if (kp.bvh_count > 1) tr.start = true, tr.bi = 1;
            else tr.active = false;
          }
        }
      }
    }
    if (__ballot(has) == 0ull) break;
    // traverse until too few lanes are still traversing (then the finished lanes take new rays)
    const int work_lim = __popcll(__ballot(has)) * kp.trav_frac16;
    for (;;) {
      const unsigned long long trav = __ballot(tr.active);
      if (trav == 0ull || __popcll(trav) * 16 < work_lim) break;
      if (tr.active) trav_step<false, false, PACK, FUSE, RING>(kp, ln, c, tr, ro, rd, shadow);
    }
    if (has && !tr.active) {
      w.res[s] = make_uint2(tr.hit, __float_as_uint(tr.dist));
      w.state[s] = WF_RET;
      has = false;
    }
  }
}

// ---------------------------------------------------------------------------
// treelet scheduling (trees past the Infinity Cache): the trace stage split at the treelet depth.
// The reference's traversal is a depth-first walk, so once the walk makes a node current it finishes
// that node's whole subtree before it pops anything older.  A subtree visit therefore needs only the ray,
// its running distance and hit, and the subtree's root: wf_top_kernel walks the top levels (a copy of the
// node array whose treelet roots carry kTreeletCnt and the treelet's id) and suspends a ray where a
// treelet root becomes current; wf_scatter_kernel groups the suspended rays by treelet; wf_bottom_kernel
// walks each ray through its treelet, treelet after treelet, so a treelet's lines are read from memory
// once for all the rays that visit it in the iteration; the next iteration's top kernel resumes the ray
// with its saved top-level stack (the next pop).  Each ray's steps are the reference's, in order.
// ---------------------------------------------------------------------------
constexpr int kTopStack = 16;  // top-level stack entries saved per suspended ray (treelet depth < this)

// a suspended ray: (o, dist) (d, hit) (inv, root) (bvh, sp, 0, 0), o/d/inv in the current BVH's frame
__device__ __forceinline__ float4* wf_tray(const WfParams& w, int k, uint32_t s) {
  return w.tray + (size_t)k * w.slots + s;
}

template <bool PACK, bool FUSE>
__global__ __launch_bounds__(256, 4) void wf_top_kernel(KParams kp, WfParams w) {
  constexpr int RING = kShortStack;
  static_assert(kTopStack <= kShortStack, "the top-level stack lives in the LDS ring");
  const int tid = threadIdx.x, lane = tid & 63;
  uint32_t* ctl = w.ctl + (size_t)WQ_WORDS * (size_t)w.iter;
  const uint32_t n_fresh = *reinterpret_cast<volatile uint32_t*>(&ctl[WQ_RAYS]);
  const uint32_t n_res = w.iter > 0 ? *reinterpret_cast<volatile uint32_t*>(&ctl[WQ_RES - WQ_WORDS]) : 0u;
  const uint32_t* res_in = w.rlist[(w.iter + 1) & 1];  // the previous iteration's bottom kernel wrote it
  const uint32_t n = n_fresh + n_res;
  Lane ln;
  ln.stk = reinterpret_cast<uint32_t*>(g_smem) + tid;
  ln.stride = 256;
  ln.gstk = kp.gstack + (size_t)blockIdx.x * 256 + tid;
  ln.gstride = kp.gstack_stride;
  ln.base = 0;
  Counters c;
  Trav tr;
  tr.active = false;
  tr.start = false;
  tr.hit = kNoneRef;
  tr.dist = 0.0f;
  tr.cnt = kNoneCnt;
  tr.sp = 0;
  tr.lo = 0;
  f3 ro = mk(0.f, 0.f, 0.f), rd = mk(0.f, 0.f, 1.f);
  bool has = false, shadow = false, exhausted = false;
  uint32_t s = 0;
  for (;;) {
    const unsigned long long idle = __ballot(!has);
    if (idle != 0ull && !exhausted) {
      const int f = __ffsll((long long)idle) - 1;
      uint32_t base = 0;
      if (lane == f) base = atomicAdd(&ctl[WQ_CLAIM], (uint32_t)__popcll(idle));
      base = __builtin_amdgcn_readfirstlane(__shfl(base, f));
      if (base + (uint32_t)__popcll(idle) >= n) exhausted = true;
      if (!has) {
        const uint32_t pos = base + (uint32_t)lane_rank(idle, lane);
        if (pos < n) {
          const uint32_t e = pos < n_fresh ? w.rayq[pos] : res_in[pos - n_fresh];
          s = e & ~kWfShadowBit;
          shadow = (e & kWfShadowBit) != 0u;
          const float4 a = *wf_field(w, 0, s), b = *wf_field(w, 1, s);
          ro = mk(a.x, a.y, a.z);
          rd = mk(b.x, b.y, b.z);
          has = true;
          tr.active = true;
          tr.start = false;
          if (pos < n_fresh) {  // a new ray: CheckHit from the first BVH's root
            tr.dist = a.w;
            tr.hit = kNoneRef;
            tr.bi = 0;
            trav_begin_bvh<false, false>(kp, c, tr, ro, rd);
            if (tr.cnt == kNoneCnt) {
              if (kp.bvh_count > 1) tr.start = true, tr.bi = 1;
              else tr.active = false;
            }
          } else {  // back from a treelet: pop the next top-level entry
            const float4 r0 = *wf_tray(w, 0, s), r1 = *wf_tray(w, 1, s), r2 = *wf_tray(w, 2, s),
                         r3 = *wf_tray(w, 3, s);
            tr.o = mk(r0.x, r0.y, r0.z);
            tr.dist = r0.w;
            tr.d = mk(r1.x, r1.y, r1.z);
            tr.hit = __float_as_uint(r1.w);
            tr.inv = mk(r2.x, r2.y, r2.z);
            tr.bi = __float_as_uint(r3.x);
            tr.sp = __float_as_int(r3.y);
            tr.lo = 0;
            tr.cnt = kNoneCnt;
            const uint32_t* ts = w.tstk + (size_t)s * (3 * kTopStack);
            for (int k = 0; k < tr.sp; ++k)
              slot_write<PACK>(ln.stk, ln.stride, k, ts[3 * k], ts[3 * k + 1], __uint_as_float(ts[3 * k + 2]));
            if (shadow && tr.hit != kNoneRef) tr.active = false;  // the treelet held the shadow ray's hit
          }
        }
      }
    }
    if (__ballot(has) == 0ull) break;
    const int work_lim = __popcll(__ballot(has)) * kp.trav_frac16;
    for (;;) {
      const unsigned long long trav = __ballot(tr.active);
      if (trav == 0ull || __popcll(trav) * 16 < work_lim) break;
      if (tr.active) {
        trav_step<false, false, PACK, FUSE, RING, true>(kp, ln, c, tr, ro, rd, shadow);
        if (tr.cnt == kTreeletCnt) tr.active = false;  // a treelet root is current: suspend there
      }
    }
    const bool susp = has && !tr.active && tr.cnt == kTreeletCnt;
    if (susp) {
      *wf_tray(w, 0, s) = make_float4(tr.o.x, tr.o.y, tr.o.z, tr.dist);
      *wf_tray(w, 1, s) = make_float4(tr.d.x, tr.d.y, tr.d.z, __uint_as_float(tr.hit));
      *wf_tray(w, 2, s) = make_float4(tr.inv.x, tr.inv.y, tr.inv.z, __uint_as_float(w.troot[tr.ref]));
      *wf_tray(w, 3, s) = make_float4(__uint_as_float(tr.bi), __int_as_float(tr.sp), 0.0f, 0.0f);
      uint32_t* ts = w.tstk + (size_t)s * (3 * kTopStack);
      for (int k = 0; k < tr.sp; ++k) {
        uint32_t r, cn;
        float et;
        slot_read<PACK>(ln.stk, ln.stride, k, r, cn, et);
        ts[3 * k] = r;
        ts[3 * k + 1] = cn;
        ts[3 * k + 2] = __float_as_uint(et);
      }
      atomicAdd(&w.tcount[tr.ref], 1u);
    }
    {  // the suspended rays and their treelets, compacted
      const unsigned long long m = __ballot(susp);
      if (m != 0ull) {
        const int f = __ffsll((long long)m) - 1;
        uint32_t base = 0;
        if (lane == f) base = atomicAdd(&ctl[WQ_SUSP], (uint32_t)__popcll(m));
        base = __shfl(base, f);
        if (susp) {
          const uint32_t pos = base + (uint32_t)lane_rank(m, lane);
          w.slist[pos] = s | (shadow ? kWfShadowBit : 0u);
          w.skey[pos] = tr.ref;
        }
      }
    }
    if (has && !tr.active && !susp) {  // CheckHit is complete
      w.res[s] = make_uint2(tr.hit, __float_as_uint(tr.dist));
      w.state[s] = WF_RET;
    }
    if (has && !tr.active) {
      has = false;
      tr.cnt = kNoneCnt;
      tr.sp = 0;
    }
  }
}

// Exclusive offsets of the per-treelet counts (one block); the counts are reset for the next iteration.
__global__ __launch_bounds__(1024) void wf_scan_kernel(WfParams w) {
  __shared__ uint32_t part[1024];
  const int t = threadIdx.x;
  const uint32_t n = w.n_treelets;
  const uint32_t per = (n + 1023u) / 1024u;
  const uint32_t lo = (uint32_t)t * per, hi = lo + per < n ? lo + per : n;
  uint32_t sum = 0;
  for (uint32_t i = lo; i < hi; ++i) sum += w.tcount[i];
  part[t] = sum;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {  // inclusive scan of the partial sums
    const uint32_t v = t >= d ? part[t - d] : 0u;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint32_t off = part[t] - sum;
  for (uint32_t i = lo; i < hi; ++i) {
    const uint32_t cnt = w.tcount[i];
    w.tfill[i] = off;
    w.tcount[i] = 0u;
    off += cnt;
  }
}

// The suspended rays into blist, grouped by treelet (in treelet order).
__global__ __launch_bounds__(256) void wf_scatter_kernel(WfParams w) {
  uint32_t* ctl = w.ctl + (size_t)WQ_WORDS * (size_t)w.iter;
  const uint32_t n = *reinterpret_cast<volatile uint32_t*>(&ctl[WQ_SUSP]);
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  w.blist[atomicAdd(&w.tfill[w.skey[i]], 1u)] = w.slist[i];
}

// Each suspended ray walks its treelet (from the root, with an empty stack of its own) and goes back to
// the top kernel with its new distance and hit.
template <bool PACK, bool FUSE, int GW>
__global__ __launch_bounds__(256, GW) void wf_bottom_kernel(KParams kp, WfParams w) {
  constexpr int RING = global_ring(GW);
  const int tid = threadIdx.x, lane = tid & 63;
  uint32_t* ctl = w.ctl + (size_t)WQ_WORDS * (size_t)w.iter;
  const uint32_t n = *reinterpret_cast<volatile uint32_t*>(&ctl[WQ_SUSP]);
  uint32_t* res_out = w.rlist[w.iter & 1];
  Lane ln;
  ln.stk = reinterpret_cast<uint32_t*>(g_smem) + tid;
  ln.stride = 256;
  ln.gstk = kp.gstack + (size_t)blockIdx.x * 256 + tid;
  ln.gstride = kp.gstack_stride;
  ln.base = 0;
  Counters c;
  Trav tr;
  tr.active = false;
  tr.start = false;
  tr.cnt = kNoneCnt;
  tr.sp = 0;
  tr.lo = 0;
  bool has = false, shadow = false, exhausted = false;
  uint32_t s = 0, e = 0;
  for (;;) {
    const unsigned long long idle = __ballot(!has);
    if (idle != 0ull && !exhausted) {
      const int f = __ffsll((long long)idle) - 1;
      uint32_t base = 0;
      if (lane == f) base = atomicAdd(&ctl[WQ_BCLAIM], (uint32_t)__popcll(idle));
      base = __builtin_amdgcn_readfirstlane(__shfl(base, f));
      if (base + (uint32_t)__popcll(idle) >= n) exhausted = true;
      if (!has) {
        const uint32_t pos = base + (uint32_t)lane_rank(idle, lane);
        if (pos < n) {
          e = w.blist[pos];
          s = e & ~kWfShadowBit;
          shadow = (e & kWfShadowBit) != 0u;
          const float4 r0 = *wf_tray(w, 0, s), r1 = *wf_tray(w, 1, s), r2 = *wf_tray(w, 2, s);
          tr.o = mk(r0.x, r0.y, r0.z);
          tr.dist = r0.w;
          tr.d = mk(r1.x, r1.y, r1.z);
          tr.hit = __float_as_uint(r1.w);
          tr.inv = mk(r2.x, r2.y, r2.z);
          tr.ref = __float_as_uint(r2.w);  // the treelet root is current (its box passed in the top kernel)
          tr.cnt = 0u;
          tr.sp = 0;
          tr.lo = 0;
          tr.active = true;
          has = true;
        }
      }
    }
    if (__ballot(has) == 0ull) break;
    const int work_lim = __popcll(__ballot(has)) * kp.trav_frac16;
    for (;;) {
      const unsigned long long trav = __ballot(tr.active);
      if (trav == 0ull || __popcll(trav) * 16 < work_lim) break;
      if (tr.active) {
        trav_substeps<false, false, PACK, FUSE, 0, RING>(kp, ln, c, tr, shadow);
        if ((tr.cnt == kNoneCnt) & (tr.sp == 0)) tr.active = false;  // the treelet is done
      }
    }
    const bool back = has && !tr.active;
    if (back) {
      wf_tray(w, 0, s)->w = tr.dist;
      wf_tray(w, 1, s)->w = __uint_as_float(tr.hit);
      has = false;
    }
    wf_append(&ctl[WQ_RES], res_out, back, e);
  }
}

}  // namespace srt
