// pathtrace.hip -- the device context behind the C ABI: scene / noise / light
// uploads, image buffers, launches of the kernels in kernels.hpp, statistics.
//
// Kernels (kernels.hpp; DESIGN.md sections 4-5):
//   sample_kernel      persistent: waves claim 64-item batches (an 8x8 tile of
//                      one frame) from a launch-wide counter; each lane runs one
//                      path sample at a time (camera ray, bounces, shadow rays)
//                      with resumable, order-exact BVH traversal, and writes the
//                      sample's radiance to an HBM sample buffer;
//   accumulate_kernel  the ordered per-pixel sum (bit-identical to per-frame
//                      image read-modify-writes) and the sRGB8 image.
// Scene residency: LDS mode copies nodes + triangles into each block's LDS
// (1024-lane blocks, packed LDS stacks); global-scene mode reads them from HBM
// through L2/MALL with an LDS ring of stack entries backed by HBM stacks.
// Device layout (re-laid from the std430 SSBOs):
//   nodes  : 32 B per node (min.xyz|first, max.xyz|count), base offset 32 B so
//            each sibling pair is one 64-B aligned block;
//   tris   : 48 B per triangle = v0, e1 = v1 - v0, e2 = v2 - v0, material id,
//            padded with kTriPad zero records;
//   mats   : 32 B shading material (albedo|roughness, specular) precomputed
//            from MaterialFromOBJ (raytrace_utils.glsl:140-175);
//   lights : 32 B, one zero record appended (lights[lightCount] reads zero);
//   noise  : noiseTex as .xy float2 (8 B), noiseUniformTex as .x float (4 B):
//            the only channels the kernel reads.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstdio>
#include <cstddef>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include <zlib.h>

#include "kernels.hpp"
#include "pool.hpp"
#include "wavefront.hpp"

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
  std::vector<std::pair<uint32_t, uint32_t>> bvh_tris;  // triangle range [lo, hi) of each record's tree
  uint32_t n_nodes = 0, n_tris = 0, n_mats = 0;
  uint32_t ref_or = 0;  // KParams::ref_or of the uploaded node layout
  // textures (srt_upload_textures) and, when materials sample them, the
  // per-triangle vertex uvs (2 float4: uv0 uv1 | uv2 0 0)
  void* d_tex = nullptr;         // texels: RGBA8 (SRT_TEX8) or RGBA32F
  uint4* d_tex_info = nullptr;  // first texel, width, height, 0
  uint32_t n_tex = 0;
  float4* d_tri_uv = nullptr;
  bool sample_textures = false;
  int stack_entries = 1;
  bool scene_ok = false;
  bool lds_ok = false;        // scene indices fit the packed LDS stack entry
  bool pairs_aligned = false; // every internal node's child pair starts at an odd slot (LDS mode's node_pair)
  bool force_global = false;  // SRT_FORCE_GLOBAL_SCENE=1 disables LDS mode
  bool fused = false;         // global-scene mode's fused sub-steps (set at upload: trees the Infinity Cache holds)
  int top_f4 = 0, top_depth = 0;  // the node array's top-level region (LayoutNodes) the fused instance copies to LDS
  int launch_top_f4 = 0;           // the region the last global-scene launch copied (0: none)
  bool launch_overlap = false;     // the last render's sample launches ran piped and overlapped (launch.overlap)
  int launch_per_cu = 0, launch_block = 0;  // resident blocks per CU and lanes per block of the last sample launch
  int launch_mats_lds = 0;                  // the last launch read the material records from LDS
  int global_waves = 4;       // the fused instance's waves per SIMD (set at upload: 5 for small trees)
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
  // tile schedule: per-tile costs recorded by the last launch and the next
  // launch's order (order_tiles_kernel); costs_for = the tile count they describe
  uint32_t* d_tile_cost = nullptr;
  uint32_t* d_tile_order = nullptr;
  int tile_cap = 0, tile_costs_for = -1;
  bool tile_schedule = true;  // SRT_TILE_ORDER=0: natural tile order
  int* d_row_map = nullptr;           // nranks > 1: global row of each local row (KParams::row_map)
  long long row_map_key = -1;         // the (rank, nranks, band_rows, rows) it was built for
  unsigned long long* d_batch_ctr = nullptr;  // one batch counter per chunk launch
  int batch_ctr_cap = 0;
  size_t lbuf_bytes = 0;
  // SRT_SAMPLE_BUFFER_MB: every sample buffer of the context together (its own, used by counting and
  // unpipelined launches, and one per pipeline slot), split equally: 21 GiB each with the 2 default slots
  size_t lbuf_total = (size_t)64 << 30;
  int tail_claims = 16;  // SRT_TAIL_CLAIMS: claims per wave before the end from which claims take one batch
  int tail_claims_gw5 = 8;  // the untextured fused 5-wave instance's (torus knot +1.4% against 16 with two slots;
                            // the textured Airplane material loses 0.6% and keeps 16;
                            // profiles/r05_experiments/tail_window_overlap.txt); SRT_TAIL_CLAIMS sets it too
  int tail_claims_sph = 1;  // the sphere launch's (C2, 8 per claim: tail 16 6.20 ms, 1 3.17 ms; its batches
                            // are cheap, the counter's atomic rate bounds it); SRT_TAIL_CLAIMS sets both
  int trav_frac16 = 9;                 // SRT_TRAV_FRAC16 (measured best on Rubik 1080p with the 16-sub-step pattern)
  int bounce_cap = 1 << 20;            // SRT_BOUNCE_CAP: bounces after which a path is cut (counted)
  int trav_frac16_global = 9;          // SRT_TRAV_FRAC16_GLOBAL: the same threshold for global-scene mode
  bool trav_frac16_global_env = false; // (set: every global instance uses it; else the fused 4-wave one takes 7, the timed IL one 8)
  bool pool_launched = false;          // the last render ran pool_kernel (srt_finish checks its watchdog)
  int pool = 0;                        // SRT_POOL=1: LDS mode runs pool_kernel (workgroup ray pools)
  int pool_batch = 64;                 // SRT_POOL_BATCH: queued hits a shading wave waits for
  int pool_tlow = 32;                  // SRT_POOL_TLOW: trace + spare records under which shading waves take fewer
  int pool_slots_max = 4096;           // SRT_POOL_SLOTS: at most this many records
  int pool_deadline_ms = 30000;        // SRT_POOL_DEADLINE_MS: pool_kernel's watchdog
  int num_cus = 256;
  int sphere_blocks = 5;               // SRT_SPHERE_BLOCKS: sphere_kernel blocks per CU (at most)
  // wavefront mode (wavefront.hpp): global-scene launches through wf_logic / wf_shade / wf_trace
  int wavefront = -1;                  // SRT_WAVEFRONT=1/0 forces it on / off; -1: by scene (wf_scene)
  bool wf_scene = false;               // chosen at upload
  uint32_t wf_slots = 1u << 21;        // SRT_WF_SLOTS: path slots in HBM
  int wf_waves = 6;                    // SRT_WF_WAVES: waves per SIMD of wf_trace_kernel (4, 5, 6 or 8)
  float4* d_wf_rec = nullptr;
  uint2* d_wf_res = nullptr;
  uint32_t *d_wf_state = nullptr, *d_wf_rayq = nullptr, *d_wf_hitq = nullptr, *d_wf_ctl = nullptr,
           *d_wf_items = nullptr;
  uint32_t wf_cap = 0;
  uint32_t* h_wf_poll = nullptr;       // pinned: (live, items) of two polled iterations
  hipEvent_t wf_poll_ev[2] = {nullptr, nullptr};
  bool wf_launched = false;            // the last render went through wavefront mode
  // treelet scheduling of wavefront mode's trace stage (wavefront.hpp wf_top_kernel / wf_bottom_kernel)
  int treelets = -1;                   // SRT_TREELETS=1/0 forces it on / off; -1: by scene (tl_scene)
  bool tl_scene = false;               // chosen at upload
  int treelet_depth = 0;               // SRT_TREELET_DEPTH: depth of the treelet roots (0: by scene size)
  uint32_t n_treelets = 0;             // of the uploaded scene (0: no flagged copy)
  float4* d_nodes_t = nullptr;         // the node array with treelet roots flagged
  uint32_t* d_troot = nullptr;         // per treelet: its root's child index
  float4* d_tl_ray = nullptr;
  uint32_t *d_tl_stk = nullptr, *d_tl_slist = nullptr, *d_tl_skey = nullptr, *d_tl_blist = nullptr,
           *d_tl_rlist = nullptr, *d_tl_count = nullptr, *d_tl_fill = nullptr;
  uint32_t tl_cap = 0, tl_count_cap = 0;
  // stats
  unsigned long long* d_stats = nullptr;
  unsigned long long* d_nan = nullptr;  // NaN path samples since the last srt_reset_stats
  srt_stats stats{};
  uint64_t shadow_rays = 0;  // of stats.rays (srt_ray_kinds)
  // per-chunk HIP events around the sample kernel of the last render call
  std::vector<hipEvent_t> ev;
  struct Occupancy {
    const void* fn;
    size_t lds;
    int per_cu;
  };
  std::vector<Occupancy> occupancy;  // resident blocks per CU of each sample_kernel instance
#ifdef SRT_WAVE_TRACE
  unsigned long long* d_trace = nullptr;
  size_t trace_bytes = 0;
  int trace_waves = 0;
#endif
  int ev_used = 0;
  // Pipelined sample launches (SRT_PIPELINE slots, default 3; 1: every launch on `stream`).  A timed
  // sample_kernel / sphere_kernel launch goes on the next slot's own stream with the slot's sample
  // buffer, batch counter, tile order and stacks; its accumulate_kernel stays on `stream` behind it.  A
  // slot's next launch waits only for that slot's last accumulation, so launch k+1 fills the CUs that
  // launch k's last waves leave idle (the drain) and the accumulations run beside them, instead of
  // sample and accumulate alternating on one stream.  The tile order of a slot's launch comes from the
  // costs of that slot's previous launch (the order decides which wave traces which sample, never a
  // value).  Counting, pool and wavefront launches run on `stream` with the context's own buffers.
  struct Slot {
    hipStream_t stream = nullptr;
    hipEvent_t sampled = nullptr, accumulated = nullptr;
    bool pending = false;  // `accumulated` recorded since the slot's buffers were last known idle
    float4* lbuf = nullptr;
    size_t lbuf_bytes = 0;
    unsigned long long* batch_ctr = nullptr;
    int batch_ctr_cap = 0;
    uint32_t* tile_cost = nullptr;
    uint32_t* tile_order = nullptr;
    int tile_cap = 0, tile_costs_for = -1;
    uint32_t* gstack = nullptr;
    size_t gstack_bytes = 0;
  };
  std::vector<Slot> slots;
  // SRT_PIPELINE: launch slots, each its own stream and buffers.  Two, since launches overlap: a third slot's
  // stream shares one of the process's 4 hardware queues (GPU_MAX_HW_QUEUES) with another, which serialises
  // them (C2 52 -> 57 G rays/s, torus knot +2.8%, metric +0.2% with 2)
  int pipe = 2;
  // SRT_PIPELINE_OVERLAP: whether a sample launch may start before the previous one ends (2, the default:
  // always; 1: on a rank's share of a multi-GPU split (nranks > 1) only; 0: never).  An overlapped launch's
  // dispatch-to-end time (rocprofv3) and span include its wait for the CUs other launches hold, so kernel
  // time is the union of the launches' spans (srt_kernel_time; tools/trace_intervals.py takes the same
  // union over rocprofv3's kernel trace).
  int pipe_overlap = 2;
  hipEvent_t last_sampled = nullptr;  // the last sample launch's end (a slot's `sampled`, or plain_done)
  hipEvent_t plain_done = nullptr;    // recorded on `stream` after a launch outside the slots
  unsigned long long pipe_seq = 0;
  hipStream_t lstream = nullptr;   // the stream the current launch's sample kernel goes on
  // Kernel time of sample_kernel / sphere_kernel launches: each writes its span (first wave's start,
  // last wave's end; s_memrealtime) into a record of this ring (HIP events around a pipelined launch
  // would also time its wait for the CUs its predecessor still holds).
  unsigned long long* d_span = nullptr;
  static constexpr int kSpanCap = 4096;
  unsigned long long span_seq = 0, span_read = 0;  // records written / summed by srt_kernel_time
  unsigned long long span_done = 0;                 // the latest end srt_kernel_time has counted (a tick)
  std::vector<long long> chunk_span;               // per chunk of the last render: its record (or -1)
  hipEvent_t lidle = nullptr;      // synchronized before the current launch frees a launch buffer
  hipEvent_t lidle2 = nullptr;     // (and this: the previous launch, for the buffers launches in series share)
};

namespace {

void FreeDev(void* p) {
  if (p) (void)hipFree(p);
}

int HipFail(const char* what) {
  const hipError_t e = hipGetLastError();
  srt::SetError(std::string(what) + ": " + hipGetErrorString(e));
  return SRT_ERR_HIP;
}

// Waits until no pipelined sample launch is in flight: before anything rewrites or frees device data
// those launches read (scene, lights, BVH records, noise, row map).
int Quiesce(srt_context* c) {
  for (auto& s : c->slots)
    if (s.stream) HIP_OK(hipStreamSynchronize(s.stream));
  return SRT_OK;
}

// Before the launch being set up frees one of its buffers: the launches that may still read it are done.
int WaitLaunchIdle(srt_context* c) {
  if (c->lidle) HIP_OK(hipEventSynchronize(c->lidle));
  if (c->lidle2) HIP_OK(hipEventSynchronize(c->lidle2));
  return SRT_OK;
}

// The span record of the launch being set up (kernels.hpp sample_body), initialised on its stream.
int TakeSpan(srt_context* c, srt::KParams& kp) {
  if (!c->d_span) HIP_OK(hipMalloc(&c->d_span, sizeof(unsigned long long) * 2 * srt_context::kSpanCap));
  const unsigned long long seq = c->span_seq++;
  kp.span = c->d_span + 2 * (seq % srt_context::kSpanCap);
  const size_t chunk = (size_t)(c->ev_used / 2);
  if (c->chunk_span.size() <= chunk) c->chunk_span.resize(chunk + 1, -1);
  c->chunk_span[chunk] = (long long)seq;
  hipLaunchKernelGGL(srt::span_init_kernel, dim3(1), dim3(64), 0, c->lstream, kp.span);
  HIP_OK(hipGetLastError());
  return SRT_OK;
}

// The launch buffers of the context and of pipeline slot `s` trade places (in, launch, out again).
// Launches in series share the context's tile costs and order (each orders its tiles by the costs of
// the launch just before it, which has ended) and its global stacks; overlapping launches each keep
// their slot's.
void SwapSlot(srt_context* c, srt_context::Slot& s, bool own) {
  std::swap(c->d_lbuf, s.lbuf);
  std::swap(c->lbuf_bytes, s.lbuf_bytes);
  std::swap(c->d_batch_ctr, s.batch_ctr);
  std::swap(c->batch_ctr_cap, s.batch_ctr_cap);
  if (own) {
    std::swap(c->d_tile_cost, s.tile_cost);
    std::swap(c->d_tile_order, s.tile_order);
    std::swap(c->tile_cap, s.tile_cap);
    std::swap(c->tile_costs_for, s.tile_costs_for);
    std::swap(c->d_gstack, s.gstack);
    std::swap(c->gstack_bytes, s.gstack_bytes);
  }
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
  for (uint32_t i = 0; i < need && i < c->h_bvhs.size(); ++i) {
    recs[i] = c->h_bvhs[i];
    // pad0/pad1 carry the triangle range of the record's tree, empty for a
    // record whose frame zeroes every direction (it never hits: the ghost
    // of src/main.cpp:683); texture sampling finds the hit's BVH by it
    const float* f = recs[i].frame;
    bool can_hit = false;
    for (int k : {0, 1, 2, 4, 5, 6, 8, 9, 10}) can_hit = can_hit || f[k] != 0.0f;
    recs[i].pad0 = can_hit ? c->bvh_tris[i].first : 0u;
    recs[i].pad1 = can_hit ? c->bvh_tris[i].second : 0u;
  }
  if (c->sample_textures) {
    for (uint32_t i = 0; i < need; ++i)
      for (uint32_t j = 0; j < i; ++j)
        if (recs[i].pad0 < recs[i].pad1 && recs[j].pad0 < recs[j].pad1 && recs[i].pad0 < recs[j].pad1 &&
            recs[j].pad0 < recs[i].pad1) {
          srt::SetError("texture sampling needs BVH records with disjoint triangle ranges");
          return SRT_ERR_INVALID;
        }
  }
  if (int rq = Quiesce(c)) return rq;
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
  if (int rq = Quiesce(c)) return rq;
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
  // sample_kernel packs a pixel as x | local_row << 16 (kernels.hpp refill)
  if (c->W > 65535 || LocalRows(c, c->H) > 32767) {
    srt::SetError("Width > 65535 or more than 32767 rows per rank");
    return SRT_ERR_LIMIT;
  }
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
  kp->tri_uv = c->d_tri_uv;
  kp->top_f4 = 0;  // (set per launch: the fused instance's LDS copy of the top levels)
  kp->top_lds_f4 = 0;
  kp->tex_texels = static_cast<const float4*>(c->d_tex);
  kp->tex_texels8 = static_cast<const uint32_t*>(c->d_tex);
  kp->tex_info = c->d_tex_info;
  kp->n_tex = c->d_tex ? c->n_tex : 0u;
  kp->lights = c->d_lights;
  kp->bvhs = c->d_bvhs;
  kp->noise_xy = c->d_noise_xy;
  kp->noise_u = c->d_noise_u;
  kp->accum = c->d_accum;
  kp->out = c->d_out;
  kp->stats = c->d_stats;
  kp->nan_ctr = c->d_nan;
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
  kp->band_shift = -1;
  for (int s = 0; s < 31; ++s)
    if ((1 << s) == c->band_rows) kp->band_shift = s;
  kp->local_rows = LocalRows(c, c->H);
  if (c->nranks > 1) {  // the row bands' global rows, one table read per new sample in the kernels
    const long long key = ((((long long)c->rank * 4096 + c->nranks) * 65536 + c->band_rows) << 20) + kp->local_rows;
    if (key != c->row_map_key) {
      std::vector<int> rows((size_t)std::max(kp->local_rows, 1));
      for (int ly = 0; ly < kp->local_rows; ++ly) {
        const int band = ly / c->band_rows;
        rows[ly] = (band * c->nranks + c->rank) * c->band_rows + (ly - band * c->band_rows);
      }
      if (int rq = Quiesce(c)) return rq;
      FreeDev(c->d_row_map);
      c->d_row_map = nullptr;
      c->row_map_key = -1;
      HIP_OK(hipMalloc(&c->d_row_map, rows.size() * sizeof(int)));
      HIP_OK(hipMemcpyAsync(c->d_row_map, rows.data(), rows.size() * sizeof(int), hipMemcpyHostToDevice, c->stream));
      HIP_OK(hipStreamSynchronize(c->stream));
      c->row_map_key = key;
    }
    kp->row_map = c->d_row_map;
  }
  kp->local_pixels = kp->local_rows * c->W;
  kp->ext_w = c->W;
  kp->ext_h = c->H;
  kp->stack_entries = c->stack_entries;
  kp->nodes_f4 = (int)(2 * ((size_t)c->n_nodes + 1));
  kp->nodes_lds_f4 = (int)((((size_t)kp->nodes_f4 + 3) >> 2) * srt::kNodeBlkF4);  // padded pair blocks
  kp->ref_or = c->ref_or;
  kp->tris_f4 = (int)(3 * ((size_t)c->n_tris + srt::kTriPad));  // with the padding records
  CameraParams(c, kp);
  return SRT_OK;
}

// LDS budget per CU (gfx950: 160 KiB; one 1024-thread block per CU in LDS mode)
constexpr size_t kLdsBytes = 160 * 1024;
// LDS mode's block (one per CU, the scene copied into its LDS): 1024 threads = 4 waves per SIMD.  An
// experiment build with 768 (3 waves per SIMD) measures what a wave per SIMD is worth
#ifndef SRT_LDS_BLOCK
#define SRT_LDS_BLOCK 1024
#endif
constexpr int kLdsBlock = SRT_LDS_BLOCK;
// Global-scene mode's block: 256 lanes, except the timed fused instance at 5 waves per SIMD, whose blocks
// hold SRT_GW5_BLOCK lanes (a multiple of 64 dividing 1280, the 20 waves 5 per SIMD make): with 640, two
// blocks per CU, so the tree's top levels are copied into LDS twice per CU instead of five times and the
// LDS a block may take beside its rings (80 KB) holds one level more
#ifndef SRT_GW5_BLOCK
#define SRT_GW5_BLOCK 256
#endif
constexpr int kGw5Block = SRT_GW5_BLOCK;
static_assert(kGw5Block % 64 == 0 && 1280 % kGw5Block == 0, "SRT_GW5_BLOCK: 64-lane waves, 1280 lanes per CU");
// Lanes per block of a global-scene launch of `gw` waves per SIMD (timed fused instance or not)
constexpr int GlobalBlock(bool timed_fused, int gw) { return (timed_fused && gw == 5) ? kGw5Block : 256; }
// gfx950 hands a block its LDS in units of 1/128 of the CU's 160 KiB (1,280 B), so n blocks run together
// only when each asks at most floor(128 / n) units: 5 blocks fit at 32,000 B each, not at 32,001, while
// hipOccupancyMaxActiveBlocksPerMultiprocessor still answers 5 up to 32,768 (and 3, 6, 7 likewise past their
// limits; tools/probes/lds_fit.hip, profiles/r06_experiments/lds_fit.json).  The blocks per CU a launch's LDS
// size allows:
constexpr size_t kLdsGran = kLdsBytes / 128;
constexpr int LdsBlocksPerCu(size_t lds) { return lds == 0 ? 1 << 30 : (int)(128 / ((lds + kLdsGran - 1) / kLdsGran)); }
// The occupancy API's resident blocks per CU, capped by that allocation rule
static int ResidentPerCu(int api_per_cu, size_t lds) { return std::max(1, std::min(api_per_cu, LdsBlocksPerCu(lds))); }
// The LDS one such block may take: its whole units of the CU's 160 KiB at gw waves per SIMD (4 SIMDs x 64
// lanes, gw * 256 / block blocks per CU)
constexpr size_t GlobalBlockLds(int block, int gw) { return (128 / ((size_t)gw * 256 / (size_t)block)) * kLdsGran; }
static_assert(GlobalBlockLds(256, 5) == 32000 && GlobalBlockLds(256, 4) == 40960 && GlobalBlockLds(640, 5) == 81920,
              "the LDS shares the probe measured");

template <bool COUNT, bool LDSM, bool PACK, int BLOCK, bool TEX, bool FUSE = false, int GW = 4>
int LaunchSamples(srt_context* c, srt::KParams kp, size_t lds) {
  // resident blocks per CU, queried once per (kernel instance, LDS size): the
  // query runs on the host between the launch's timing events otherwise
  const void* fn = reinterpret_cast<const void*>(&srt::sample_kernel<COUNT, LDSM, PACK, BLOCK, TEX, FUSE, GW>);
  int per_cu = 0;
  for (const auto& e : c->occupancy)
    if (e.fn == fn && e.lds == lds) per_cu = e.per_cu;
  if (per_cu == 0) {
    HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, srt::sample_kernel<COUNT, LDSM, PACK, BLOCK, TEX, FUSE, GW>,
                                                          BLOCK, lds));
    per_cu = ResidentPerCu(per_cu, lds);
    c->occupancy.push_back({fn, lds, per_cu});
  }
  const int blocks = c->num_cus * per_cu;
  c->launch_per_cu = per_cu;
  c->launch_block = BLOCK;
  if constexpr (!LDSM) {  // global-scene mode: every lane's full stack in HBM (backing the LDS ring)
    const size_t lanes = (size_t)blocks * BLOCK;
    const size_t need = lanes * (PACK ? 2 : 3) * sizeof(uint32_t) * (size_t)kp.stack_entries;
    if (need > c->gstack_bytes) {
      if (int rw = WaitLaunchIdle(c)) return rw;
      FreeDev(c->d_gstack);
      c->d_gstack = nullptr;
      c->gstack_bytes = 0;
      HIP_OK(hipMalloc(&c->d_gstack, need));
      c->gstack_bytes = need;
    }
    kp.gstack = c->d_gstack;
    kp.gstack_stride = (int)lanes;
  }
#ifdef SRT_WAVE_TRACE
  {  // diagnostic build: 4 realtime stamps per wave of the last launch
    const size_t need = (size_t)blocks * (BLOCK / 64) * 4 * sizeof(unsigned long long);
    if (need > c->trace_bytes) {
      FreeDev(c->d_trace);
      HIP_OK(hipMalloc(&c->d_trace, need));
      c->trace_bytes = need;
    }
    c->trace_waves = blocks * (BLOCK / 64);
    kp.wave_trace = c->d_trace;
  }
#endif
  {  // single-batch claims for the last tail_claims * kClaim batches per wave (sample_kernel; measured
     // in round 1: 2 -> 16 halves the launch's tail)
    const long long waves = (long long)blocks * (BLOCK / 64);
    const long long n_batches = (long long)((kp.W + 7) >> 3) * ((kp.local_rows + 7) >> 3) * kp.nframes;
    const int tail_claims = (FUSE && GW == 5 && !TEX) ? c->tail_claims_gw5 : c->tail_claims;
    kp.tail_start = (int)std::max<long long>(0, n_batches - (long long)tail_claims * srt::kClaim * waves);
  }
  // the early-break threshold of the fused 4-wave instance (trees of 48-600 MB): 7, where the
  // latency-bound soups gain (1 M: 1,370 -> 1,413-1,418 Mrays/s; 3 M: 939 -> 971) and the 5-wave
  // (torus knot) and IL (C5) instances lose
  if constexpr (!LDSM && FUSE && GW == 4)
    if (!c->trav_frac16_global_env) kp.trav_frac16 = 7;
  // ... and of the timed IL instance (trees past 600 MB): 8 (C5, kernel ms on one box: 9 771-773,
  // 8 762-767, 10 793; profiles/r03_experiments/c5_pattern_threshold.txt)
  if constexpr (!LDSM && !FUSE && !COUNT)
    if (!c->trav_frac16_global_env) kp.trav_frac16 = 8;
  if (int rs = TakeSpan(c, kp)) return rs;
  HIP_OK(hipEventRecord(c->ev[c->ev_used], c->lstream));
  hipLaunchKernelGGL((srt::sample_kernel<COUNT, LDSM, PACK, BLOCK, TEX, FUSE, GW>), dim3(blocks), dim3(BLOCK), lds, c->lstream,
                     kp);
  HIP_OK(hipGetLastError());
  HIP_OK(hipEventRecord(c->ev[c->ev_used + 1], c->lstream));
  return SRT_OK;
}

// The sphere scene (showModel false): sphere_kernel, one 256-lane block per resident slot (no stacks,
// so its LDS holds only the light records).
template <bool COUNT>
int LaunchSpheres(srt_context* c, srt::KParams kp, size_t lds) {
  const void* fn = reinterpret_cast<const void*>(&srt::sphere_kernel<COUNT>);
  int per_cu = 0;
  for (const auto& e : c->occupancy)
    if (e.fn == fn && e.lds == lds) per_cu = e.per_cu;
  if (per_cu == 0) {
    HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, srt::sphere_kernel<COUNT>, 256, lds));
    per_cu = ResidentPerCu(per_cu, lds);
    c->occupancy.push_back({fn, lds, per_cu});
  }
  // resident blocks per CU: as many as its registers allow (C2 on one box, ms per launch: 3 blocks 3.23,
  // 4 3.00, 5 2.93; while the launch counter's atomic rate bound it, round 3, 3 were best)
  const int blocks = c->num_cus * std::min(per_cu, c->sphere_blocks);
  c->launch_per_cu = std::min(per_cu, c->sphere_blocks);
  c->launch_block = 256;
  {
    const long long waves = (long long)blocks * 4;
    const long long n_batches = (long long)((kp.W + 7) >> 3) * ((kp.local_rows + 7) >> 3) * kp.nframes;
    kp.tail_start = (int)std::max<long long>(0, n_batches - (long long)c->tail_claims_sph * srt::kClaimSph * waves);
  }
  if (int rs = TakeSpan(c, kp)) return rs;
  HIP_OK(hipEventRecord(c->ev[c->ev_used], c->lstream));
  hipLaunchKernelGGL(srt::sphere_kernel<COUNT>, dim3(blocks), dim3(256), lds, c->lstream, kp);
  HIP_OK(hipGetLastError());
  HIP_OK(hipEventRecord(c->ev[c->ev_used + 1], c->lstream));
  return SRT_OK;
}

// The sample_kernel instance for the launch: counting or not, LDS-resident
// scene or global (packed stack entries when indices fit 24 bits; the timed
// global instance's schedule and waves per SIMD chosen at upload), and with
// or without the texture-sampling branch (TEX, only when a material samples).
template <bool TEX>
int LaunchMode(srt_context* c, const srt::KParams& kc, size_t lds, bool count, bool ldsm, bool pack) {
  if (!kc.show_model) return count ? LaunchSpheres<true>(c, kc, lds) : LaunchSpheres<false>(c, kc, lds);
  if (count && ldsm) return LaunchSamples<true, true, true, kLdsBlock, TEX>(c, kc, lds);
  if (count) return pack ? LaunchSamples<true, false, true, 256, TEX>(c, kc, lds)
                         : LaunchSamples<true, false, false, 256, TEX>(c, kc, lds);
  if (ldsm) return LaunchSamples<false, true, true, kLdsBlock, TEX>(c, kc, lds);
  if (c->fused && c->global_waves == 5) return pack ? LaunchSamples<false, false, true, kGw5Block, TEX, true, 5>(c, kc, lds)
                                                   : LaunchSamples<false, false, false, kGw5Block, TEX, true, 5>(c, kc, lds);
  if (c->fused) return pack ? LaunchSamples<false, false, true, 256, TEX, true>(c, kc, lds)
                            : LaunchSamples<false, false, false, 256, TEX, true>(c, kc, lds);
  return pack ? LaunchSamples<false, false, true, 256, TEX>(c, kc, lds)
              : LaunchSamples<false, false, false, 256, TEX>(c, kc, lds);
}

// pool_kernel (pool.hpp): one 1024-thread block per CU, as sample_kernel's LDS mode.
template <bool COUNT>
int LaunchPool(srt_context* c, srt::KParams kp, size_t lds) {
  const int blocks = c->num_cus;
  c->launch_per_cu = 1;
  c->launch_block = 1024;
  kp.tail_start = (int)std::max<long long>(
      0, (long long)((kp.W + 7) >> 3) * ((kp.local_rows + 7) >> 3) * kp.nframes -
             (long long)c->tail_claims * srt::kClaim * blocks * srt::kPoolTravWaves);
  HIP_OK(hipEventRecord(c->ev[c->ev_used], c->stream));
  hipLaunchKernelGGL(srt::pool_kernel<COUNT>, dim3(blocks), dim3(1024), lds, c->stream, kp);
  HIP_OK(hipGetLastError());
  HIP_OK(hipEventRecord(c->ev[c->ev_used + 1], c->stream));
  return SRT_OK;
}

// Wavefront mode (wavefront.hpp): the trace-stage kernels' instances (stack entry packing, fused
// sub-steps or the IL pattern, waves per SIMD) and their grids: as many 256-lane blocks as are resident.
template <typename F>
int Resident(srt_context* c, F* fn, size_t lds, int* blocks) {
  const void* key = reinterpret_cast<const void*>(fn);
  int per_cu = 0;
  for (const auto& e : c->occupancy)
    if (e.fn == key && e.lds == lds) per_cu = e.per_cu;
  if (per_cu == 0) {
    HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 256, lds));
    per_cu = ResidentPerCu(per_cu, lds);
    c->occupancy.push_back({key, lds, per_cu});
  }
  *blocks = c->num_cus * per_cu;
  return SRT_OK;
}
// The trace stage of one iteration: wf_trace_kernel, or with treelets (kp_top: the flagged node copy)
// wf_top_kernel -> wf_scan_kernel -> wf_scatter_kernel -> wf_bottom_kernel.  With `launch` false it
// only sizes the grids: *lanes = the most lanes any of them runs (their HBM stacks).
template <bool PACK, bool FUSE, int GW>
int WfStage(srt_context* c, const srt::KParams& kp, const srt::KParams& kp_top, const srt::WfParams& w, bool tl,
            bool launch, size_t* lanes) {
  const size_t ring_bytes = (size_t)256 * (PACK ? 2 : 3) * sizeof(uint32_t);
  const size_t lds = ring_bytes * (size_t)srt::global_ring(GW);
  int blocks = 0;
  if (!tl) {
    int rc = Resident(c, srt::wf_trace_kernel<PACK, FUSE, GW>, lds, &blocks);
    if (rc) return rc;
    if (lanes) *lanes = (size_t)blocks * 256;
    if (launch) {
      hipLaunchKernelGGL((srt::wf_trace_kernel<PACK, FUSE, GW>), dim3(blocks), dim3(256), lds, c->stream, kp, w);
      HIP_OK(hipGetLastError());
    }
    return SRT_OK;
  }
  const size_t lds_top = ring_bytes * (size_t)srt::kShortStack;
  int tblocks = 0;
  int rc = Resident(c, srt::wf_top_kernel<PACK, FUSE>, lds_top, &tblocks);
  if (rc) return rc;
  rc = Resident(c, srt::wf_bottom_kernel<PACK, FUSE, GW>, lds, &blocks);
  if (rc) return rc;
  if (lanes) *lanes = (size_t)std::max(blocks, tblocks) * 256;
  if (launch) {
    hipLaunchKernelGGL((srt::wf_top_kernel<PACK, FUSE>), dim3(tblocks), dim3(256), lds_top, c->stream, kp_top, w);
    hipLaunchKernelGGL(srt::wf_scan_kernel, dim3(1), dim3(1024), 0, c->stream, w);
    hipLaunchKernelGGL(srt::wf_scatter_kernel, dim3((w.slots + 255) / 256), dim3(256), 0, c->stream, w);
    hipLaunchKernelGGL((srt::wf_bottom_kernel<PACK, FUSE, GW>), dim3(blocks), dim3(256), lds, c->stream, kp, w);
    HIP_OK(hipGetLastError());
  }
  return SRT_OK;
}
template <bool PACK, bool FUSE>
int WfStageWaves(srt_context* c, const srt::KParams& kp, const srt::KParams& kt, const srt::WfParams& w, bool tl,
                 bool launch, size_t* lanes) {
  switch (c->wf_waves) {
    case 4: return WfStage<PACK, FUSE, 4>(c, kp, kt, w, tl, launch, lanes);
    case 5: return WfStage<PACK, FUSE, 5>(c, kp, kt, w, tl, launch, lanes);
    case 8: return WfStage<PACK, FUSE, 8>(c, kp, kt, w, tl, launch, lanes);
    default: return WfStage<PACK, FUSE, 6>(c, kp, kt, w, tl, launch, lanes);
  }
}
int WfTrace(srt_context* c, const srt::KParams& kp, const srt::KParams& kt, const srt::WfParams& w, bool tl,
            bool launch, size_t* lanes) {
  const bool pack = c->lds_ok;
  if (c->fused) return pack ? WfStageWaves<true, true>(c, kp, kt, w, tl, launch, lanes)
                            : WfStageWaves<false, true>(c, kp, kt, w, tl, launch, lanes);
  return pack ? WfStageWaves<true, false>(c, kp, kt, w, tl, launch, lanes)
              : WfStageWaves<false, false>(c, kp, kt, w, tl, launch, lanes);
}

// One chunk of frames through the wavefront kernels: iterations of logic -> shade -> trace over
// c->wf_slots path slots until every sample item is taken and no slot is live.  The host polls the
// live count of every 8th iteration one group late (a pinned copy and an event), so the stream stays
// full; the few iterations issued past the end find empty queues and return at once.
int LaunchWavefront(srt_context* c, srt::KParams kp, bool tex) {
  c->launch_per_cu = c->launch_block = 0;  // (its stage kernels' grids differ: no single value)
  constexpr int kMaxIters = 1 << 16;
  const uint32_t P = c->wf_slots;
  if (P > c->wf_cap) {
    FreeDev(c->d_wf_rec); FreeDev(c->d_wf_res); FreeDev(c->d_wf_state); FreeDev(c->d_wf_rayq); FreeDev(c->d_wf_hitq);
    c->d_wf_rec = nullptr; c->d_wf_res = nullptr; c->d_wf_state = c->d_wf_rayq = c->d_wf_hitq = nullptr;
    c->wf_cap = 0;
    HIP_OK(hipMalloc(&c->d_wf_rec, sizeof(float4) * 7 * (size_t)P));
    HIP_OK(hipMalloc(&c->d_wf_res, sizeof(uint2) * (size_t)P));
    HIP_OK(hipMalloc(&c->d_wf_state, sizeof(uint32_t) * (size_t)P));
    HIP_OK(hipMalloc(&c->d_wf_rayq, sizeof(uint32_t) * (size_t)P));
    HIP_OK(hipMalloc(&c->d_wf_hitq, sizeof(uint32_t) * (size_t)P));
    c->wf_cap = P;
  }
  if (!c->d_wf_ctl) {
    HIP_OK(hipMalloc(&c->d_wf_ctl, sizeof(uint32_t) * srt::WQ_WORDS * (size_t)kMaxIters));
    HIP_OK(hipMalloc(&c->d_wf_items, sizeof(uint32_t)));
    HIP_OK(hipHostMalloc(&c->h_wf_poll, 4 * sizeof(uint32_t), hipHostMallocDefault));
  }
  const long long n_items = 64LL * ((kp.W + 7) >> 3) * ((kp.local_rows + 7) >> 3) * kp.nframes;
  if (n_items >= (1LL << 31)) {  // Launch bounds the frames per chunk so this cannot happen
    srt::SetError("wavefront mode: more than 2^31 sample items in one chunk");
    return SRT_ERR_LIMIT;
  }
  HIP_OK(hipMemsetAsync(c->d_wf_state, 0, sizeof(uint32_t) * (size_t)P, c->stream));
  HIP_OK(hipMemsetAsync(c->d_wf_items, 0, sizeof(uint32_t), c->stream));
  HIP_OK(hipMemsetAsync(c->d_wf_ctl, 0, sizeof(uint32_t) * srt::WQ_WORDS * (size_t)kMaxIters, c->stream));
  srt::WfParams w;
  w.rec = c->d_wf_rec;
  w.res = c->d_wf_res;
  w.state = c->d_wf_state;
  w.rayq = c->d_wf_rayq;
  w.hitq = c->d_wf_hitq;
  w.ctl = c->d_wf_ctl;
  w.items = c->d_wf_items;
  w.slots = P;
  w.n_items = (uint32_t)n_items;
  w.iter = 0;
  kp.lights_lds = 0;  // the wavefront kernels keep no LDS copies of lights / materials
  kp.mats_lds = 0;
  const bool tl = c->n_treelets > 0 && (c->treelets >= 0 ? c->treelets == 1 : c->tl_scene);
  if (tl) {
    if (P > c->tl_cap) {
      FreeDev(c->d_tl_ray); FreeDev(c->d_tl_stk); FreeDev(c->d_tl_slist); FreeDev(c->d_tl_skey);
      FreeDev(c->d_tl_blist); FreeDev(c->d_tl_rlist);
      c->d_tl_ray = nullptr;
      c->d_tl_stk = c->d_tl_slist = c->d_tl_skey = c->d_tl_blist = c->d_tl_rlist = nullptr;
      c->tl_cap = 0;
      HIP_OK(hipMalloc(&c->d_tl_ray, sizeof(float4) * 4 * (size_t)P));
      HIP_OK(hipMalloc(&c->d_tl_stk, sizeof(uint32_t) * 3 * srt::kTopStack * (size_t)P));
      HIP_OK(hipMalloc(&c->d_tl_slist, sizeof(uint32_t) * (size_t)P));
      HIP_OK(hipMalloc(&c->d_tl_skey, sizeof(uint32_t) * (size_t)P));
      HIP_OK(hipMalloc(&c->d_tl_blist, sizeof(uint32_t) * (size_t)P));
      HIP_OK(hipMalloc(&c->d_tl_rlist, sizeof(uint32_t) * 2 * (size_t)P));
      c->tl_cap = P;
    }
    if (c->n_treelets > c->tl_count_cap) {
      FreeDev(c->d_tl_count); FreeDev(c->d_tl_fill);
      c->d_tl_count = c->d_tl_fill = nullptr;
      c->tl_count_cap = 0;
      HIP_OK(hipMalloc(&c->d_tl_count, sizeof(uint32_t) * (size_t)c->n_treelets));
      HIP_OK(hipMalloc(&c->d_tl_fill, sizeof(uint32_t) * (size_t)c->n_treelets));
      c->tl_count_cap = c->n_treelets;
    }
    HIP_OK(hipMemsetAsync(c->d_tl_count, 0, sizeof(uint32_t) * (size_t)c->n_treelets, c->stream));
    w.tray = c->d_tl_ray;
    w.tstk = c->d_tl_stk;
    w.slist = c->d_tl_slist;
    w.skey = c->d_tl_skey;
    w.blist = c->d_tl_blist;
    w.rlist[0] = c->d_tl_rlist;
    w.rlist[1] = c->d_tl_rlist + P;
    w.tcount = c->d_tl_count;
    w.tfill = c->d_tl_fill;
    w.troot = c->d_troot;
    w.n_treelets = c->n_treelets;
  } else {
    w.tray = nullptr;
    w.tstk = w.slist = w.skey = w.blist = w.rlist[0] = w.rlist[1] = w.tcount = w.tfill = nullptr;
    w.troot = nullptr;
    w.n_treelets = 0;
  }
  srt::KParams kt = kp;  // the top kernel walks the flagged node copy
  if (tl) kt.nodes = c->d_nodes_t;
  size_t lanes = 0;
  int rc = WfTrace(c, kp, kt, w, tl, false, &lanes);
  if (rc) return rc;
  {  // every trace lane's full stack in HBM, behind its LDS ring
    const size_t need = lanes * (c->lds_ok ? 2 : 3) * sizeof(uint32_t) * (size_t)kp.stack_entries;
    if (need > c->gstack_bytes) {
      FreeDev(c->d_gstack);
      c->d_gstack = nullptr;
      c->gstack_bytes = 0;
      HIP_OK(hipMalloc(&c->d_gstack, need));
      c->gstack_bytes = need;
    }
    kp.gstack = kt.gstack = c->d_gstack;
    kp.gstack_stride = kt.gstack_stride = (int)lanes;
  }
  const dim3 sgrid((P + 255) / 256);
  if (!c->wf_poll_ev[0]) {
    HIP_OK(hipEventCreateWithFlags(&c->wf_poll_ev[0], hipEventDisableTiming));
    HIP_OK(hipEventCreateWithFlags(&c->wf_poll_ev[1], hipEventDisableTiming));
  }
  hipEvent_t* poll_ev = c->wf_poll_ev;
  HIP_OK(hipEventRecord(c->ev[c->ev_used], c->stream));
  int it = 0;
  bool done = false;
  for (; it < kMaxIters && !done; ++it) {
    w.iter = it;
    hipLaunchKernelGGL(srt::wf_logic_kernel, sgrid, dim3(256), 0, c->stream, kp, w);
    if (tex) hipLaunchKernelGGL(srt::wf_shade_kernel<true>, sgrid, dim3(256), 0, c->stream, kp, w);
    else hipLaunchKernelGGL(srt::wf_shade_kernel<false>, sgrid, dim3(256), 0, c->stream, kp, w);
    HIP_OK(hipGetLastError());
    rc = WfTrace(c, kp, kt, w, tl, true, nullptr);
    if (rc) break;
    if ((it & 7) == 7) {
      const int g = (it >> 3) & 1;
      HIP_OK(hipMemcpyAsync(c->h_wf_poll + 2 * g, c->d_wf_ctl + (size_t)srt::WQ_WORDS * it + srt::WQ_LIVE,
                            sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
      HIP_OK(hipMemcpyAsync(c->h_wf_poll + 2 * g + 1, c->d_wf_items, sizeof(uint32_t), hipMemcpyDeviceToHost,
                            c->stream));
      HIP_OK(hipEventRecord(poll_ev[g], c->stream));
      if (it >= 15) {  // the previous group's poll
        HIP_OK(hipEventSynchronize(poll_ev[g ^ 1]));
        const uint32_t live = c->h_wf_poll[2 * (g ^ 1)], items = c->h_wf_poll[2 * (g ^ 1) + 1];
        done = live == 0 && (long long)items >= n_items;
      }
    }
  }
  if (rc) return rc;
  if (!done) {
    srt::SetError("wavefront mode: iteration limit reached");
    return SRT_ERR_LIMIT;
  }
  HIP_OK(hipEventRecord(c->ev[c->ev_used + 1], c->stream));
  c->wf_launched = true;
  return SRT_OK;
}

// LDS bytes of the light records a launch keeps in LDS (behind the rest of its layout, when they fit the
// kernel's cap, as Launch places them)
size_t LightLdsBytes(const srt::KParams& kp) {
  const size_t light_bytes = 2 * sizeof(float4) * ((size_t)kp.light_records + 1);
  return light_bytes <= 8192 ? light_bytes : 0;
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
  // (node pairs at the padded LDS stride; only for node arrays whose pairs are all 64-B aligned)
  const size_t scene_bytes = ((size_t)kp.nodes_lds_f4 + (size_t)kp.tris_f4) * sizeof(float4);
  const size_t lds_mode_bytes = scene_bytes + (size_t)kLdsBlock * 2 * sizeof(uint32_t) * (size_t)kp.stack_entries;
  const bool ldsm = kp.show_model && c->lds_ok && c->pairs_aligned && !c->force_global && lds_mode_bytes <= kLdsBytes;
  const int gw = (!count && c->fused) ? c->global_waves : 4;  // global-scene mode: LaunchMode's instance
  const int block = ldsm ? kLdsBlock : GlobalBlock(!count && c->fused, gw);
  // pool mode (pool.hpp): LDS mode with stacks for the traversal waves only, then the ray records;
  // laid out first, and sample_kernel's layout when the records do not fit
  bool pool = ldsm && c->pool && !c->sample_textures && kp.max_depth >= 0 && kp.max_depth <= 255;
  size_t lds = 0;
  for (int attempt = 0; attempt < 2; ++attempt) {
    if (pool) {
      kp.stack_base_f4 = kp.nodes_lds_f4 + kp.tris_f4;
      lds = scene_bytes + (size_t)srt::kPoolTravLanes * 2 * sizeof(uint32_t) * (size_t)kp.stack_entries;
    } else if (ldsm) {
      kp.stack_base_f4 = kp.nodes_lds_f4 + kp.tris_f4;
      lds = lds_mode_bytes;
    } else if (kp.show_model) {  // LDS rings of global_ring(waves) entries per lane, backed by HBM stacks
      kp.stack_base_f4 = 0;
      lds = (size_t)block * (c->lds_ok ? 2 : 3) * sizeof(uint32_t) * (size_t)srt::global_ring(gw);
      if (SRT_COOP && !count && c->fused) {  // the fused sub-steps' load stages, one per wave
        lds = (lds + 15) & ~(size_t)15;
        kp.coop_off = (int)lds;
        lds += (size_t)(block / 64) * srt::kCoopWaveBytes;
      }
      // the top levels' pairs (LayoutNodes' first region) for the fused instance, when they fit beside the
      // rings and this launch's light records (placed behind it, below) within the LDS one of the
      // instance's blocks may take; the material records follow only if they still fit that share, else
      // shading reads them from HBM, so neither costs a resident block per CU, and the region,
      // worth ~10% on a surface mesh, is never given up for them; wavefront mode's kernels read none
      kp.top_f4 = 0;
      const bool wf_launch = !count && (c->wavefront >= 0 ? c->wavefront == 1 : c->wf_scene);
      if (!count && c->fused && !wf_launch && c->top_f4 > 0) {
        lds = (lds + 15) & ~(size_t)15;
        const size_t tb = ((size_t)c->top_f4 + 3) / 4 * srt::kNodeBlkF4 * sizeof(float4);
        if (lds + tb + LightLdsBytes(kp) <= GlobalBlockLds(block, gw)) {
          kp.top_f4 = c->top_f4;
          kp.top_lds_f4 = (int)(lds / sizeof(float4));
          lds += tb;
        }
      }
      c->launch_top_f4 = kp.top_f4;
    } else {  // the sphere scene (sphere_kernel): no traversal stacks
      kp.stack_base_f4 = 0;
      lds = 0;
    }
    {  // light and material records in LDS behind the rest, when they fit (shading reads them there) within
       // the LDS one block may take: all of it in LDS mode, a global-scene block's share at its instance's
       // blocks per CU (records past it would cost a resident block per CU; they are read from HBM instead)
      const size_t cap = (!ldsm && kp.show_model) ? GlobalBlockLds(block, gw) : kLdsBytes;
      lds = (lds + 15) & ~(size_t)15;
      const size_t light_bytes = 2 * sizeof(float4) * ((size_t)kp.light_records + 1);
      kp.lights_lds = (light_bytes <= 8192 && lds + light_bytes <= cap) ? 1 : 0;
      if (kp.lights_lds) {
        kp.lights_base_f4 = (int)(lds / sizeof(float4));
        lds += light_bytes;
      }
      kp.mat_records = (int)c->n_mats + 1;
      const size_t mat_bytes = 2 * sizeof(float4) * (size_t)kp.mat_records;
      kp.mats_lds = (kp.show_model && c->d_mats && mat_bytes <= 16384 && lds + mat_bytes <= cap) ? 1 : 0;
      if (kp.mats_lds) {
        kp.mats_base_f4 = (int)(lds / sizeof(float4));
        lds += mat_bytes;
      }
      c->launch_mats_lds = kp.mats_lds;
    }
    if (!pool) break;
    // control words, 3 rings of u32 record ids (power-of-two capacity), 112-B records
    kp.pool_ctl_off = (int)lds;
    lds += 16 * sizeof(uint32_t);
    int slots = 0, cap = 1;
    for (int r = std::min(c->pool_slots_max, 65534); r >= 64 && slots == 0; --r) {
      int cp = 1;
      while (cp < r) cp <<= 1;
      if (lds + (size_t)3 * cp * sizeof(uint32_t) + (size_t)r * 112 <= kLdsBytes) {
        slots = r;
        cap = cp;
      }
    }
    if (slots == 0) {  // no room for 64 records
      pool = false;
      continue;
    }
    kp.pool_ring_off = (int)lds;
    lds += (size_t)3 * cap * sizeof(uint32_t);
    kp.pool_rec_off = (int)lds;
    lds += (size_t)slots * 112;
    kp.pool_cap = cap;
    kp.pool_slots = slots;
    kp.pool_batch = c->pool_batch;
    kp.pool_tlow = c->pool_tlow;
    kp.pool_deadline = (unsigned long long)c->pool_deadline_ms * 100000ull;  // s_memrealtime runs at 100 MHz
    break;
  }
  // sample buffer: as many frames per chunk as the buffer cap allows
  const size_t per_frame = (size_t)npx * sizeof(float4);
  // frames per launch: what the sample buffer holds, and n_tiles * frames < 2^31 (the kernel's batch index)
  const size_t n_tiles = (size_t)((kp.W + 7) >> 3) * (size_t)((kp.local_rows + 7) >> 3);
  // (less 2^20: the batch counter overshoots the end by up to (max(kClaim, kClaimSph) + 1) claims per wave)
  // wavefront mode (global-scene, timed launches): its sample items (64 per batch) < 2^31 per chunk
  const bool wf = !ldsm && !count && kp.show_model && (c->wavefront >= 0 ? c->wavefront == 1 : c->wf_scene);
  const size_t max_frames = std::max<size_t>(
      1, ((size_t)0x7FFFFFFF - ((size_t)1 << 20)) / std::max<size_t>(1, n_tiles) / (wf ? 64 : 1));
  // the context's sample buffers share SRT_SAMPLE_BUFFER_MB: its own and, with pipeline slots, one per slot
  const size_t lbuf_cap = c->lbuf_total / (size_t)(c->pipe > 1 ? c->pipe + 1 : 1);
  const int chunk = (int)std::max<size_t>(
      1, std::min<size_t>(std::min<size_t>((size_t)kp.nframes, max_frames), lbuf_cap / per_frame));
  const size_t need = per_frame * (size_t)chunk;
  const bool piped = !count && !pool && !wf && c->pipe > 1;
  // (a counting launch, the untimed first launch of a measurement, sets the slots up for the timed ones)
  if ((piped || (count && c->pipe > 1)) && c->slots.empty()) {
    c->slots.resize((size_t)c->pipe);
    for (auto& sl : c->slots) {
      HIP_OK(hipStreamCreateWithFlags(&sl.stream, hipStreamNonBlocking));
      HIP_OK(hipEventCreateWithFlags(&sl.sampled, hipEventDisableTiming));
      HIP_OK(hipEventCreateWithFlags(&sl.accumulated, hipEventDisableTiming));
    }
  }
  kp.trav_frac16 = ldsm ? c->trav_frac16 : c->trav_frac16_global;
  kp.bounce_cap = c->bounce_cap;
  // (ST_POOLERR, the last entry, is sticky: a watchdog that fired in an earlier launch of this
  // render must still reach srt_finish, which reads and clears it)
  static_assert(srt::ST_POOLERR + 1 == srt::ST_TOTAL, "ST_POOLERR must stay the last stats entry");
  HIP_OK(hipMemsetAsync(c->d_stats, 0, sizeof(unsigned long long) * srt::ST_POOLERR, c->stream));
  const int out_frames = kp.frame_first + kp.nframes - 1;
  const int nchunks = (kp.nframes + chunk - 1) / chunk;
  while ((int)c->ev.size() < 2 * nchunks) {
    hipEvent_t e;
    HIP_OK(hipEventCreate(&e));
    c->ev.push_back(e);
  }
  c->ev_used = 0;
  c->chunk_span.assign((size_t)nchunks, -1);
  // The launch buffers: the context's own on `stream`, or (piped) one slot's per chunk on the slot's
  // stream.  A piped chunk's batch counter is the slot's one word (its previous launch is accumulated).
  const int ctr_need = piped ? 1 : nchunks;
  const bool overlap = c->pipe_overlap == 2 || (c->pipe_overlap == 1 && c->nranks > 1);
  c->launch_overlap = piped && overlap;
  if (piped || (count && c->pipe > 1)) {  // every slot's sample buffer now: a timed loop allocates none
    for (auto& sl : c->slots) {
      if (sl.lbuf_bytes >= need) continue;
      if (sl.pending) HIP_OK(hipEventSynchronize(sl.accumulated));
      FreeDev(sl.lbuf);
      sl.lbuf = nullptr;
      sl.lbuf_bytes = 0;
      HIP_OK(hipMalloc(&sl.lbuf, need));
      sl.lbuf_bytes = need;
    }
  }
  for (int f0 = 0; f0 < kp.nframes; f0 += chunk) {
    srt_context::Slot* sl = piped ? &c->slots[(size_t)(c->pipe_seq++ % (unsigned long long)c->pipe)] : nullptr;
    if (sl) {
      if (sl->pending) HIP_OK(hipStreamWaitEvent(sl->stream, sl->accumulated, 0));
      if (!overlap && c->last_sampled) HIP_OK(hipStreamWaitEvent(sl->stream, c->last_sampled, 0));
      SwapSlot(c, *sl, overlap);
      c->lstream = sl->stream;
      c->lidle = sl->pending ? sl->accumulated : nullptr;
      c->lidle2 = overlap ? nullptr : c->last_sampled;
    }
    if (!sl) {  // launches in series may still read the shared stacks and tile arrays
      c->lidle = nullptr;
      c->lidle2 = c->last_sampled;
    }
    const hipStream_t ls = c->lstream;
    int rc = SRT_OK;
    do {  // (one pass: `break` on an error, so the slot's buffers are swapped back)
      const bool grow = need > c->lbuf_bytes || ctr_need > c->batch_ctr_cap || (int)n_tiles > c->tile_cap;
      if (grow && WaitLaunchIdle(c) != SRT_OK) { rc = SRT_ERR_HIP; break; }  // earlier launches still read them
      if (need > c->lbuf_bytes) {
        FreeDev(c->d_lbuf);
        c->d_lbuf = nullptr;
        c->lbuf_bytes = 0;
        if (hipMalloc(&c->d_lbuf, need) != hipSuccess) { srt::SetError("hipMalloc(sample buffer) failed"); rc = SRT_ERR_HIP; break; }
        c->lbuf_bytes = need;
      }
      if (ctr_need > c->batch_ctr_cap) {
        FreeDev(c->d_batch_ctr);
        c->d_batch_ctr = nullptr;
        c->batch_ctr_cap = 0;
        if (hipMalloc(&c->d_batch_ctr, sizeof(unsigned long long) * (size_t)ctr_need) != hipSuccess) {
          srt::SetError("hipMalloc(batch counters) failed");
          rc = SRT_ERR_HIP;
          break;
        }
        c->batch_ctr_cap = ctr_need;
      }
      if (!sl && f0 == 0)
        if (hipMemsetAsync(c->d_batch_ctr, 0, sizeof(unsigned long long) * (size_t)nchunks, ls) != hipSuccess) { rc = HipFail("sample launch"); break; }
      if (sl && hipMemsetAsync(c->d_batch_ctr, 0, sizeof(unsigned long long), ls) != hipSuccess) { rc = HipFail("sample launch"); break; }
      srt::KParams kc = kp;
      kc.lbuf = c->d_lbuf;
      kc.frame_first = kp.frame_first + f0;
      kc.nframes = std::min(chunk, kp.nframes - f0);
      kc.write_output = (f0 + chunk >= kp.nframes) ? kp.write_output : 0;
      kc.batch_ctr = reinterpret_cast<uint32_t*>(c->d_batch_ctr + (sl ? 0 : f0 / chunk));
      {  // tile order: the tiles the last launch found most expensive first (SRT_TILE_ORDER=0: natural order)
        const int nt = (int)n_tiles;
        if (nt > c->tile_cap) {
          FreeDev(c->d_tile_cost);
          FreeDev(c->d_tile_order);
          c->d_tile_cost = c->d_tile_order = nullptr;
          c->tile_cap = 0;
          if (hipMalloc(&c->d_tile_cost, sizeof(uint32_t) * (size_t)nt) != hipSuccess ||
              hipMalloc(&c->d_tile_order, sizeof(uint32_t) * (size_t)nt) != hipSuccess) {
            srt::SetError("hipMalloc(tile order) failed");
            rc = SRT_ERR_HIP;
            break;
          }
          c->tile_cap = nt;
          c->tile_costs_for = -1;
        }
        if (c->tile_schedule && c->tile_costs_for == nt) {
          hipLaunchKernelGGL(srt::order_tiles_kernel, dim3(1), dim3(1024), 0, ls, c->d_tile_cost, c->d_tile_order, nt);
        } else {
          hipLaunchKernelGGL(srt::iota_kernel, dim3((nt + 255) / 256), dim3(256), 0, ls, c->d_tile_order, nt);
          if (c->tile_schedule && hipMemsetAsync(c->d_tile_cost, 0, sizeof(uint32_t) * (size_t)nt, ls) != hipSuccess) {
            rc = HipFail("sample launch");
            break;
          }
        }
        if (hipGetLastError() != hipSuccess) { rc = HipFail("sample launch"); break; }
        kc.tile_order = c->d_tile_order;
        kc.tile_cost = c->tile_schedule ? c->d_tile_cost : nullptr;
        c->tile_costs_for = c->tile_schedule ? nt : -1;
      }
      // LDS mode: packed entries (lds_ok); global-scene mode: packed when indices fit 24 bits
      const bool pack = c->lds_ok;
      if (pool) rc = count ? LaunchPool<true>(c, kc, lds) : LaunchPool<false>(c, kc, lds);
      else if (wf) rc = LaunchWavefront(c, kc, c->sample_textures);
      else rc = c->sample_textures ? LaunchMode<true>(c, kc, lds, count, ldsm, pack)
                                   : LaunchMode<false>(c, kc, lds, count, ldsm, pack);
      if (rc) break;
      c->pool_launched |= pool;
      c->ev_used += 2;  // LaunchSamples recorded the pair around the launch
      if (!sl) {  // a later launch in series (sharing the tile order) waits for this one
        if (!c->plain_done && hipEventCreateWithFlags(&c->plain_done, hipEventDisableTiming) != hipSuccess) {
          rc = HipFail("sample launch");
          break;
        }
        if (hipEventRecord(c->plain_done, c->stream) != hipSuccess) { rc = HipFail("sample launch"); break; }
        c->last_sampled = c->plain_done;
      }
      if (sl) {  // the accumulation follows the samples on `stream`
        c->last_sampled = sl->sampled;
        if (hipEventRecord(sl->sampled, ls) != hipSuccess || hipStreamWaitEvent(c->stream, sl->sampled, 0) != hipSuccess) {
          rc = HipFail("sample launch");
          break;
        }
      }
      hipLaunchKernelGGL(srt::accumulate_kernel, pgrid, dim3(256), 0, c->stream, kc, out_frames);
      if (hipGetLastError() != hipSuccess) { rc = HipFail("sample launch"); break; }
      if (sl) {
        if (hipEventRecord(sl->accumulated, c->stream) != hipSuccess) { rc = HipFail("sample launch"); break; }
        sl->pending = true;
      }
    } while (false);
    if (sl) {
      SwapSlot(c, *sl, overlap);
      c->lstream = c->stream;
    }
    c->lidle = c->lidle2 = nullptr;
    if (rc) return rc;
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
    c->stats.bounce_cap += s[srt::ST_BOUNCECAP];
    c->stats.max_stack = std::max<uint64_t>(c->stats.max_stack, s[srt::ST_MAXSTACK]);
    c->shadow_rays += s[srt::ST_SHADOW];
  }
  return SRT_OK;
}

// Depth of each BVH (root depth 0) and index validation.
// Every node some traversal can reach is checked: the trees of the BVH records and node 0's (the
// ghost records past n_bvhs traverse from node 0, raytrace_compute.glsl:144-147).  `reach` marks
// them; the layouts and the upload touch no other node, so an unreachable record may hold anything.
int ValidateNodes(const srt_bvh_node* nodes, uint32_t n_nodes, uint32_t n_tris, const srt_bvh_record* bvhs,
                  uint32_t n_bvhs, int* max_depth, std::vector<std::pair<uint32_t, uint32_t>>* tri_ranges,
                  std::vector<uint8_t>* reach) {
  *max_depth = 0;
  tri_ranges->assign(n_bvhs, {0u, 0u});
  reach->assign(n_nodes, 0);
  std::vector<std::pair<uint32_t, int>> st;
  std::vector<uint8_t> seen(n_nodes, 0);
  for (uint32_t b = 0; b <= n_bvhs; ++b) {  // b == n_bvhs: node 0's tree
    uint32_t lo = 0xFFFFFFFFu, hi = 0;
    const uint32_t root = b < n_bvhs ? bvhs[b].first_index : 0u;
    if (root >= n_nodes) {
      srt::SetError("BVH first_index out of range");
      return SRT_ERR_INVALID;
    }
    st.push_back({root, 0});
    while (!st.empty()) {
      auto [i, d] = st.back();
      st.pop_back();
      (*reach)[i] = 1;
      *max_depth = std::max(*max_depth, d);
      const srt_bvh_node& n = nodes[i];
      if (n.prim_count > 0) {
        if ((uint64_t)n.first_child_or_prim_index + n.prim_count > n_tris || n.prim_count >= 0x80000000u) {
          srt::SetError("BVH leaf references triangles out of range");
          return SRT_ERR_INVALID;
        }
        lo = std::min(lo, n.first_child_or_prim_index);
        hi = std::max(hi, n.first_child_or_prim_index + n.prim_count);
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
    if (b < n_bvhs) (*tri_ranges)[b] = lo < hi ? std::make_pair(lo, hi) : std::make_pair(0u, 0u);
  }
  return SRT_OK;
}

// Device node layout.  An internal step reads the current node's child pair
// and, speculatively, the pair after it (traversal.hpp, trav_internal): when
// the right child -- the one the traversal visits first -- is internal and its
// own child pair is that next pair, the step expands it too, so a descent along
// right children takes one memory round trip per two levels.  The device array
// therefore holds the pairs in the traversal's order (pre-order, right child
// first), where a right child's pair directly follows its parent's.  Only
// addresses change: every record keeps its bounds, leaf triangle range and
// count; an internal node's child index and each BVH's root are remapped.  Slot
// 0 keeps node 0 (the ghost zero records traverse from it); other roots take a
// pair's first slot with a zero record beside it.  Returns false (the identity
// layout is used) for inputs whose sibling pairs overlap, which no
// reference-built tree has.  A child pair reached from two BVH records' trees
// keeps its first placement; srt_upload_scene sets a node's "right child's
// pair follows" flag only where the remapped slots confirm it.
// `top_depth` > 0 (global-scene scenes, SRT_TOP_DEPTH): the pairs of every node at depth < top_depth are
// laid out first, in the same order, so they form the array's first `*n_top_slots` slots -- the region the
// fused instance copies into each block's LDS (traversal.hpp trav_fused) -- and the rest follows.  A pair
// on the region's last level keeps no right-spine flag (its right child's pair lies past the region).
bool LayoutNodes(const srt_bvh_node* nodes, uint32_t n_nodes, const srt_bvh_record* bvhs, uint32_t n_bvhs,
                 bool align, std::vector<uint32_t>* remap, uint32_t* n_slots, int top_depth = 0,
                 uint32_t* n_top_slots = nullptr) {
  constexpr uint32_t kUnset = 0xFFFFFFFFu;
  remap->assign(n_nodes, kUnset);
  auto& m = *remap;
  m[0] = 0;
  uint32_t next = 1;  // pairs start at odd slots (64-B aligned behind the 32-B pad)
  std::vector<uint32_t> roots{0};
  for (uint32_t b = 0; b < n_bvhs; ++b) {
    const uint32_t r = bvhs[b].first_index;
    if (m[r] == kUnset) {
      m[r] = next;
      next += 2;
    }
    roots.push_back(r);
  }
  // `align`: a chain of right-child pairs starts on a 128-B line (slot = 3 mod
  // 4: a zero pair pads before it when needed), so a step that reads a pair and
  // its right child's pair touches one line (see srt_upload_scene for when).
  uint32_t chain_next = kUnset;  // the node whose pair continues the current chain
  std::vector<uint8_t> top(top_depth > 0 ? n_nodes : 0, 0);  // nodes whose pair the first pass laid out
  std::vector<std::pair<uint32_t, int>> st;                    // (node, depth)
  for (int pass = top_depth > 0 ? 0 : 1; pass < 2; ++pass) {
    chain_next = kUnset;
    for (uint32_t r : roots) {
      st.push_back({r, 0});
      while (!st.empty()) {
        const uint32_t i = st.back().first;
        const int d = st.back().second;
        st.pop_back();
        const srt_bvh_node& n = nodes[i];
        if (n.prim_count > 0) continue;
        const uint32_t c0 = n.first_child_or_prim_index, c1 = c0 + 1;
        if (pass == 1 && !top.empty() && top[i]) {  // laid out by the first pass: descend only
          st.push_back({c0, d + 1});
          st.push_back({c1, d + 1});
          continue;
        }
        if (pass == 0 && d >= top_depth) continue;
        if (m[c0] == kUnset && m[c1] == kUnset) {
          if (align && i != chain_next && nodes[c1].prim_count == 0 && (next & 3u) != 3u) next += 2;
          m[c0] = next;
          m[c1] = next + 1;
          next += 2;
          if (pass == 0) top[i] = 1;
          chain_next = nodes[c1].prim_count == 0 ? c1 : kUnset;
          st.push_back({c0, d + 1});  // popped after c1's subtree: c1 is visited first
          st.push_back({c1, d + 1});
        } else if (m[c0] == kUnset || m[c1] != m[c0] + 1) {
          return false;  // a shared or overlapping pair
        }
      }
    }
    if (pass == 0 && n_top_slots) *n_top_slots = next;
  }
  if (top_depth <= 0 && n_top_slots) *n_top_slots = 0;
  *n_slots = next;
  return true;
}

// The slots LayoutNodes(..., top_depth) gives its top region: its first pass alone (the pairs of the nodes
// at depth < top_depth, bounded by the depth, not the tree's size); false where LayoutNodes would fail.
bool TopRegionSlots(const srt_bvh_node* nodes, uint32_t n_nodes, const srt_bvh_record* bvhs, uint32_t n_bvhs,
                    bool align, int top_depth, uint32_t* n_top) {
  std::unordered_map<uint32_t, uint32_t> m;  // the few nodes the pass places -> slot
  m[0] = 0;
  uint32_t next = 1;
  std::vector<uint32_t> roots{0};
  for (uint32_t b = 0; b < n_bvhs; ++b) {
    const uint32_t r = bvhs[b].first_index;
    if (!m.count(r)) {
      m[r] = next;
      next += 2;
    }
    roots.push_back(r);
  }
  constexpr uint32_t kUnset = 0xFFFFFFFFu;
  uint32_t chain_next = kUnset;
  std::vector<std::pair<uint32_t, int>> st;
  for (uint32_t r : roots) {
    st.push_back({r, 0});
    while (!st.empty()) {
      const uint32_t i = st.back().first;
      const int d = st.back().second;
      st.pop_back();
      const srt_bvh_node& n = nodes[i];
      if (n.prim_count > 0 || d >= top_depth) continue;
      const uint32_t c0 = n.first_child_or_prim_index, c1 = c0 + 1;
      const auto f0 = m.find(c0), f1 = m.find(c1);
      if (f0 == m.end() && f1 == m.end()) {
        if (align && i != chain_next && nodes[c1].prim_count == 0 && (next & 3u) != 3u) next += 2;
        m[c0] = next;
        m[c1] = next + 1;
        next += 2;
        chain_next = nodes[c1].prim_count == 0 ? c1 : kUnset;
        st.push_back({c0, d + 1});
        st.push_back({c1, d + 1});
      } else if (f0 == m.end() || f1 == m.end() || f1->second != f0->second + 1) {
        return false;
      }
    }
  }
  *n_top = next;
  return true;
}

// Device triangle slots for scenes read through L2 (global-scene mode).  A leaf
// of one or two triangles (the midpoint builder's leaves on a triangle soup) is
// read by one leaf step; at 48 B per record, 5 of every 8 such reads straddle
// two 128-B lines.  Here each such leaf starts at a slot whose records
// lie in one line (slot mod 8 in {0, 1, 3, 4, 6, 7} for one record, {0, 3, 6}
// for two), zero records filling the gaps; larger leaves are not padded.  The
// map is monotone, so the order is kept and a BVH's triangle range stays one
// slot range.  Returns false (identity) when two leaves' ranges partly overlap.
bool LayoutTris(const srt_bvh_node* nodes, uint32_t n_nodes, const std::vector<uint8_t>& reach, uint32_t n_tris,
                std::vector<uint32_t>* slot, uint32_t* n_slots) {
  constexpr uint32_t kUnset = 0xFFFFFFFFu;
  std::vector<uint32_t> owner(n_tris, kUnset), lead(n_tris, 0);
  for (uint32_t i = 0; i < n_nodes; ++i) {
    const srt_bvh_node& n = nodes[i];
    if (n.prim_count == 0 || !reach[i]) continue;  // (ValidateNodes range-checked the reachable leaves)
    const uint32_t f = n.first_child_or_prim_index;
    if (lead[f] != 0 && lead[f] != n.prim_count) return false;  // two leaves from one triangle, different sizes
    if (lead[f] == n.prim_count) continue;                      // the same leaf again (a shared subtree)
    for (uint32_t t = f; t < f + n.prim_count; ++t) {
      if (owner[t] != kUnset) return false;
      owner[t] = f;
    }
    lead[f] = n.prim_count;
  }
  slot->resize(n_tris);
  uint32_t s = 0;
  for (uint32_t t = 0; t < n_tris; ++t) {
    if (lead[t] == 1) {
      while ((s & 7u) == 2u || (s & 7u) == 5u) ++s;
    } else if (lead[t] == 2) {
      while ((s & 7u) % 3u != 0u) ++s;  // {0, 3, 6}
    }
    (*slot)[t] = s++;
  }
  *n_slots = s;
  return true;
}

}  // namespace

namespace srt {

// The multi-GPU root's assembly kernels on a given stream (srt_assemble_bands /
// srt_assemble_output_bands use the context's own; the device group its gather stream).
int AssembleBandsOn(srt_context* c, void* stream, const void* gathered, int nranks, int rows_pad, int band_rows,
                    int frames, void* accum_full, void* out_full) {
  if (!c || !gathered || nranks < 1 || rows_pad < 1 || band_rows < 1 || frames < 1 || c->W <= 0 || c->H <= 0)
    return SRT_ERR_INVALID;
  HIP_OK(hipSetDevice(c->device));
  const size_t n = (size_t)c->W * (size_t)c->H;
  hipLaunchKernelGGL(srt::assemble_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), static_cast<const float4*>(gathered), nranks, rows_pad, c->W,
                     c->H, band_rows, frames, static_cast<float4*>(accum_full), static_cast<uint32_t*>(out_full));
  HIP_OK(hipGetLastError());
  return SRT_OK;
}

int AssembleOutputOn(srt_context* c, void* stream, const void* gathered_rgba8, int nranks, int rows_pad,
                     int band_rows, int ext_w, int ext_h, void* out_full) {
  if (!c || !gathered_rgba8 || !out_full || nranks < 1 || rows_pad < 1 || band_rows < 1 || c->W <= 0 || c->H <= 0)
    return SRT_ERR_INVALID;
  HIP_OK(hipSetDevice(c->device));
  const size_t n = (size_t)c->W * (size_t)c->H;
  hipLaunchKernelGGL(srt::assemble_out_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), static_cast<const uint32_t*>(gathered_rgba8), nranks, rows_pad,
                     c->W, c->H, band_rows, std::min(ext_w, c->W), std::min(ext_h, c->H),
                     static_cast<uint32_t*>(out_full));
  HIP_OK(hipGetLastError());
  return SRT_OK;
}

int DetachImages(srt_context* c) {
  if (!c) return SRT_ERR_INVALID;
  HIP_OK(hipSetDevice(c->device));
  HIP_OK(hipStreamSynchronize(c->stream));
  if (int rq = Quiesce(c)) return rq;
  if (!c->images_external) { FreeDev(c->d_accum); FreeDev(c->d_out); }
  c->d_accum = nullptr;
  c->d_out = nullptr;
  c->images_external = false;
  c->img_w = c->img_rows = 0;
  c->rank = 0;
  c->nranks = 1;
  return SRT_OK;
}

}  // namespace srt

// ===========================================================================
// C ABI (context part)
// ===========================================================================
extern "C" {

const char* srt_last_error(void) { return srt::LastError(); }
int srt_abi_version(void) { return SRT_ABI_VERSION; }
#ifndef SRT_CODE_HASH
#define SRT_CODE_HASH "unknown"
#endif
const char* srt_code_hash(void) { return SRT_CODE_HASH; }

int srt_create(int device, void* stream, srt_context** out) {
  if (!out) return SRT_ERR_INVALID;
  HIP_OK(hipSetDevice(device));
  auto* c = new srt_context();
  c->device = device;
  if (const char* e = std::getenv("SRT_FORCE_GLOBAL_SCENE")) c->force_global = e[0] == '1';
  if (const char* e = std::getenv("SRT_SAMPLE_BUFFER_MB")) c->lbuf_total = (size_t)std::max(1L, std::atol(e)) << 20;
  if (const char* e = std::getenv("SRT_SAMPLE_BUFFER_KB")) c->lbuf_total = (size_t)std::max(1L, std::atol(e)) << 10;
  if (const char* e = std::getenv("SRT_BOUNCE_CAP")) c->bounce_cap = std::max(1, std::atoi(e));
  if (const char* e = std::getenv("SRT_POOL")) c->pool = e[0] == '1';
  if (const char* e = std::getenv("SRT_POOL_BATCH")) c->pool_batch = std::max(1, std::min(64, std::atoi(e)));
  if (const char* e = std::getenv("SRT_POOL_TLOW")) c->pool_tlow = std::max(1, std::atoi(e));
  if (const char* e = std::getenv("SRT_POOL_SLOTS")) c->pool_slots_max = std::max(64, std::atoi(e));
  if (const char* e = std::getenv("SRT_POOL_DEADLINE_MS")) c->pool_deadline_ms = std::max(1, std::atoi(e));
  if (const char* e = std::getenv("SRT_SPHERE_BLOCKS")) c->sphere_blocks = std::max(1, std::atoi(e));
  if (const char* e = std::getenv("SRT_WAVEFRONT")) c->wavefront = e[0] == '1' ? 1 : 0;
  if (const char* e = std::getenv("SRT_WF_SLOTS")) c->wf_slots = (uint32_t)std::max(256L, std::min(1L << 28, std::atol(e)));
  if (const char* e = std::getenv("SRT_WF_WAVES")) c->wf_waves = std::atoi(e);
  if (const char* e = std::getenv("SRT_TREELETS")) c->treelets = e[0] == '1' ? 1 : 0;
  if (const char* e = std::getenv("SRT_TREELET_DEPTH")) c->treelet_depth = std::max(0, std::min(srt::kTopStack - 1, std::atoi(e)));
  if (const char* e = std::getenv("SRT_PIPELINE")) c->pipe = std::max(1, std::min(8, std::atoi(e)));
  if (const char* e = std::getenv("SRT_PIPELINE_OVERLAP")) c->pipe_overlap = std::max(0, std::min(2, std::atoi(e)));
  if (const char* e = std::getenv("SRT_TAIL_CLAIMS"))
    c->tail_claims = c->tail_claims_sph = c->tail_claims_gw5 = std::max(0, std::atoi(e));
  if (const char* e = std::getenv("SRT_TILE_ORDER")) c->tile_schedule = e[0] != '0';
  if (const char* e = std::getenv("SRT_TRAV_FRAC16")) c->trav_frac16 = std::max(0, std::min(16, std::atoi(e)));
  if (const char* e = std::getenv("SRT_TRAV_FRAC16_GLOBAL"))
    c->trav_frac16_global = std::max(0, std::min(16, std::atoi(e))), c->trav_frac16_global_env = true;
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
  c->lstream = c->stream;
  if (hipMalloc(&c->d_stats, sizeof(unsigned long long) * srt::ST_TOTAL) != hipSuccess ||
      hipMemset(c->d_stats, 0, sizeof(unsigned long long) * srt::ST_TOTAL) != hipSuccess ||
      hipMalloc(&c->d_nan, sizeof(unsigned long long)) != hipSuccess ||
      hipMemset(c->d_nan, 0, sizeof(unsigned long long)) != hipSuccess) {
    FreeDev(c->d_stats);
    FreeDev(c->d_nan);
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
  (void)Quiesce(c);
  for (auto& sl : c->slots) {
    FreeDev(sl.lbuf); FreeDev(sl.batch_ctr); FreeDev(sl.tile_cost); FreeDev(sl.tile_order); FreeDev(sl.gstack);
    if (sl.sampled) (void)hipEventDestroy(sl.sampled);
    if (sl.accumulated) (void)hipEventDestroy(sl.accumulated);
    if (sl.stream) (void)hipStreamDestroy(sl.stream);
  }
  c->slots.clear();
  if (c->plain_done) (void)hipEventDestroy(c->plain_done);
  FreeDev(c->d_nodes); FreeDev(c->d_tris); FreeDev(c->d_mats); FreeDev(c->d_bvhs); FreeDev(c->d_lights);
  FreeDev(c->d_tex); FreeDev(c->d_tex_info); FreeDev(c->d_tri_uv);
  FreeDev(c->d_noise_xy); FreeDev(c->d_noise_u); FreeDev(c->d_stats); FreeDev(c->d_nan); FreeDev(c->d_lbuf); FreeDev(c->d_gstack);
  FreeDev(c->d_batch_ctr); FreeDev(c->d_tile_cost); FreeDev(c->d_tile_order); FreeDev(c->d_row_map); FreeDev(c->d_span);
  FreeDev(c->d_wf_rec); FreeDev(c->d_wf_res); FreeDev(c->d_wf_state); FreeDev(c->d_wf_rayq); FreeDev(c->d_wf_hitq);
  FreeDev(c->d_wf_ctl); FreeDev(c->d_wf_items);
  FreeDev(c->d_nodes_t); FreeDev(c->d_troot); FreeDev(c->d_tl_ray); FreeDev(c->d_tl_stk); FreeDev(c->d_tl_slist);
  FreeDev(c->d_tl_skey); FreeDev(c->d_tl_blist); FreeDev(c->d_tl_rlist); FreeDev(c->d_tl_count); FreeDev(c->d_tl_fill);
  if (c->h_wf_poll) (void)hipHostFree(c->h_wf_poll);
  for (hipEvent_t e : c->wf_poll_ev)
    if (e) (void)hipEventDestroy(e);
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

int srt_device(srt_context* c) { return c ? c->device : -1; }

int srt_get_int(srt_context* c, const char* name, int* v) {
  if (!c || !name || !v) return SRT_ERR_INVALID;
  const std::string n(name);
  if (n == "Width") *v = c->W;
  else if (n == "Height") *v = c->H;
  else if (n == "accumFrames") *v = c->accum_frames;
  else if (n == "lightCount") *v = c->light_count;
  else if (n == "maxDepth") *v = c->max_depth;
  else if (n == "bvh_count") *v = (int)c->bvh_count;
  else if (n == "resetAccumBuffer") *v = c->reset;
  else if (n == "showModel") *v = c->show_model;
  else if (n == "scene.fused") *v = c->fused ? 1 : 0;
  else if (n == "scene.top_depth") *v = c->top_depth;  // levels in the fused instance's LDS copy (0: none)
  else if (n == "scene.top_f4") *v = c->top_f4;
  else if (n == "launch.top_f4") *v = c->launch_top_f4;
  else if (n == "scene.global_waves") *v = c->global_waves;
  else if (n == "scene.wavefront") *v = c->wavefront >= 0 ? c->wavefront : (c->wf_scene ? 1 : 0);
  else if (n == "scene.wf_waves") *v = c->wf_waves;
  else if (n == "scene.treelets") *v = (int)c->n_treelets;
  else if (n == "scene.tri_slots") *v = (int)c->n_tris;  // device triangle records (LayoutTris gaps included)
  else if (n == "launch.chunks") *v = c->ev_used / 2;   // sample launches of the last render or dispatch
  else if (n == "launch.overlap") *v = c->launch_overlap ? 1 : 0;  // what the last render's launches did
  else if (n == "launch.blocks_per_cu") *v = c->launch_per_cu;      // resident blocks per CU of the last sample launch
  else if (n == "launch.block") *v = c->launch_block;               // its lanes per block
  else if (n == "launch.mats_lds") *v = c->launch_mats_lds;          // 1: it read the material records from LDS
  else return SRT_ERR_NOT_FOUND;
  return SRT_OK;
}

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
  rc = Launch(c, kp, count != 0);
  if (rc == SRT_OK) c->accum_frames = frame_first + nframes - 1;  // the uniform as the last dispatch leaves it
  return rc;
}

int srt_finish(srt_context* c) {
  if (!c) return SRT_ERR_INVALID;
  HIP_OK(hipStreamSynchronize(c->stream));
  if (c->pool_launched) {  // pool_kernel's watchdog (pool.hpp): a launch that overran its deadline
    unsigned long long err = 0;
    HIP_OK(hipMemcpy(&err, c->d_stats + srt::ST_POOLERR, sizeof(err), hipMemcpyDeviceToHost));
    HIP_OK(hipMemset(c->d_stats + srt::ST_POOLERR, 0, sizeof(err)));
    c->pool_launched = false;
    if (err) {
      srt::SetError("pool_kernel: watchdog expired (the render is incomplete)");
      return SRT_ERR_HIP;
    }
  }
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

#ifdef SRT_WAVE_TRACE
// Diagnostic build: copies the last launch's per-wave stamps (start, scene in
// LDS, batches exhausted, end; s_memrealtime ticks) into out[4 * n], n <= waves.
extern "C" int srt_debug_wave_trace(srt_context* c, unsigned long long* out, int n) {
  if (!c || !out || !c->d_trace) return -1;
  n = std::min(n, c->trace_waves);
  HIP_OK(hipMemcpyAsync(out, c->d_trace, (size_t)n * 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                        c->stream));
  HIP_OK(hipStreamSynchronize(c->stream));
  return n;
}
#endif

// Kernel time of sample launches from their span records (first wave's start, last wave's end; 100 MHz
// ticks): the time during which some sample launch of the context runs, i.e. the union of the spans.
// Launches in series add their spans.  Overlapped pipeline slots dispatch a launch while its
// predecessor still runs -- it starts in the CUs the drain frees, or, when the host has enqueued several
// ahead, the hardware may run two slots' launches side by side or the later one first -- so a span then
// includes the wait for CUs another launch holds, and only the union is the launches' device time.
namespace {
bool SpanRecord(const srt_context* c, const unsigned long long* ring, unsigned long long q, unsigned long long* t0,
                unsigned long long* t1) {
  if (q >= c->span_seq || q + srt_context::kSpanCap < c->span_seq) return false;  // not written, or overwritten
  const unsigned long long* sp = ring + 2 * (q % srt_context::kSpanCap);
  if (sp[1] < sp[0]) return false;
  *t0 = sp[0];
  *t1 = sp[1];
  return true;
}
// Union of the spans of records [from, to) in ms, counting only time after `after` (a tick); *last_end
// receives the latest end seen (or `after`).
double SpanUnionMs(const srt_context* c, const unsigned long long* ring, unsigned long long from,
                   unsigned long long to, unsigned long long after, unsigned long long* last_end) {
  std::vector<std::pair<unsigned long long, unsigned long long>> iv;
  for (unsigned long long q = from; q < to; ++q) {
    unsigned long long t0, t1;
    if (SpanRecord(c, ring, q, &t0, &t1)) iv.push_back({std::max(t0, after), std::max(t1, after)});
  }
  std::sort(iv.begin(), iv.end());
  unsigned long long covered = 0, reach = after;
  for (const auto& [a, b] : iv) {
    const unsigned long long lo = std::max(a, reach);
    if (b > lo) covered += b - lo;
    reach = std::max(reach, b);
  }
  if (last_end) *last_end = reach;
  return (double)covered * 1e-5;
}
}  // namespace

int srt_last_kernel_ms(srt_context* c, float* ms) {
  if (!c || !ms) return SRT_ERR_INVALID;
  *ms = 0.0f;
  std::vector<unsigned long long> ring;
  unsigned long long lo = ~0ull, hi = 0;  // the render's span records (its chunks' launches are consecutive)
  for (int i = 0; i + 1 < c->ev_used; i += 2) {
    HIP_OK(hipEventSynchronize(c->ev[i + 1]));
    const size_t chunk = (size_t)(i / 2);
    const long long rec = chunk < c->chunk_span.size() ? c->chunk_span[chunk] : -1;
    if (rec >= 0 && (unsigned long long)rec + srt_context::kSpanCap >= c->span_seq) {  // the launch's own span
      lo = std::min(lo, (unsigned long long)rec);
      hi = std::max(hi, (unsigned long long)rec + 1);
      continue;
    }
    float t = 0.0f;  // pool and wavefront launches: the HIP events around them
    HIP_OK(hipEventElapsedTime(&t, c->ev[i], c->ev[i + 1]));
    *ms += t;
  }
  if (lo < hi) {
    ring.resize(2 * srt_context::kSpanCap);
    HIP_OK(hipMemcpy(ring.data(), c->d_span, sizeof(unsigned long long) * ring.size(), hipMemcpyDeviceToHost));
    *ms += (float)SpanUnionMs(c, ring.data(), lo, hi, 0ull, nullptr);
  }
  return SRT_OK;
}

int srt_kernel_time(srt_context* c, double* total_ms, int* launches) {
  if (!c || !total_ms || !launches) return SRT_ERR_INVALID;
  *total_ms = 0.0;
  *launches = 0;
  HIP_OK(hipStreamSynchronize(c->stream));
  if (int rq = Quiesce(c)) return rq;
  const unsigned long long from = c->span_read;
  c->span_read = c->span_seq;
  if (c->span_seq - from > (unsigned long long)srt_context::kSpanCap) {  // records were overwritten unread
    srt::SetError("srt_kernel_time: more than 4096 sample launches since the last call (span records lost)");
    return SRT_ERR_LIMIT;
  }
  if (c->span_seq > from) {
    std::vector<unsigned long long> ring(2 * srt_context::kSpanCap);
    HIP_OK(hipMemcpy(ring.data(), c->d_span, sizeof(unsigned long long) * ring.size(), hipMemcpyDeviceToHost));
    // (time before the end of the launches read by the previous call was counted there)
    *total_ms = SpanUnionMs(c, ring.data(), from, c->span_seq, c->span_done, &c->span_done);
    *launches = (int)(c->span_seq - from);
  }
  return SRT_OK;
}

int srt_get_stats(srt_context* c, srt_stats* out) {
  if (!c || !out) return SRT_ERR_INVALID;
  *out = c->stats;
  return SRT_OK;
}

int srt_ray_kinds(srt_context* c, uint64_t kinds[3]) {
  if (!c || !kinds) return SRT_ERR_INVALID;
  kinds[0] = c->stats.samples;  // one camera ray per path sample
  kinds[1] = c->shadow_rays;
  kinds[2] = c->stats.rays - c->stats.samples - c->shadow_rays;
  return SRT_OK;
}

int srt_reset_stats(srt_context* c) {
  if (!c) return SRT_ERR_INVALID;
  c->stats = srt_stats{};
  c->shadow_rays = 0;
  HIP_OK(hipSetDevice(c->device));
  HIP_OK(hipMemsetAsync(c->d_nan, 0, sizeof(unsigned long long), c->stream));
  HIP_OK(hipStreamSynchronize(c->stream));
  return SRT_OK;
}

int srt_nan_samples(srt_context* c, uint64_t* out) {
  if (!c || !out) return SRT_ERR_INVALID;
  unsigned long long v = 0;
  HIP_OK(hipSetDevice(c->device));
  HIP_OK(hipMemcpyAsync(&v, c->d_nan, sizeof(v), hipMemcpyDeviceToHost, c->stream));
  HIP_OK(hipStreamSynchronize(c->stream));
  *out = v;
  return SRT_OK;
}

int srt_upload_scene(srt_context* c, const srt_bvh_record* bvhs, uint32_t n_bvhs, const srt_bvh_node* nodes,
                     uint32_t n_nodes, const srt_material_obj* mats, const float* tex_albedo, uint32_t n_mats,
                     const srt_triangle* tris, uint32_t n_tris, const srt_vertex* verts, uint32_t n_verts) {
  if (!c || (n_bvhs && !bvhs) || (n_nodes && !nodes) || (n_mats && !mats) || (n_tris && !tris) ||
      (n_verts && !verts))
    return SRT_ERR_INVALID;
  if (int rq = Quiesce(c)) return rq;  // pipelined launches still read the old scene
  if (n_nodes == 0 || n_bvhs == 0) {
    srt::SetError("scene needs at least one BVH and one node");
    return SRT_ERR_INVALID;
  }
  int depth = 0;
  std::vector<std::pair<uint32_t, uint32_t>> tri_ranges;
  std::vector<uint8_t> reach;
  int rc = ValidateNodes(nodes, n_nodes, n_tris, bvhs, n_bvhs, &depth, &tri_ranges, &reach);
  if (rc) return rc;
  HIP_OK(hipSetDevice(c->device));
  // nodes: 32-B records behind a 32-B pad so sibling pairs are 64-B aligned,
  // in the traversal's order (LayoutNodes; unreachable nodes are dropped), and
  // one zero pair past the end for the internal step's speculative read
  std::vector<uint32_t> remap;
  uint32_t n_slots = n_nodes;
  const char* lay_env = std::getenv("SRT_NODE_LAYOUT");
  // Line-aligned chains pay where the tree streams from HBM: fewer lines per
  // step (C5, 10 M triangles: 505 -> 578 Mrays/s; 3 M: 774 -> 823).  A scene
  // the 256-MB Infinity Cache holds runs latency-bound and is faster dense
  // (300 k: 1929 vs 1695; 1 M: 1234 vs 1088), though it then misses more
  // often in L2.  Measured crossover between 100 and 300 MB of nodes +
  // triangles; SRT_NODE_ALIGN=1/0 forces either.
  const char* al_env = std::getenv("SRT_NODE_ALIGN");
  const double scene_mb = (32.0 * n_nodes + 48.0 * n_tris) / (1 << 20);
  const bool align = al_env ? al_env[0] == '1' : scene_mb >= 192.0;
  // Global-scene traversal schedule: fused sub-steps (trav_fused: one memory
  // round trip per step for both node kinds) while the kernel waits on latency
  // (1 M, 101 MB: 1232 -> 1373 Mrays/s; 262 k torus knot 4576 -> 5432; 3 M,
  // 336 MB: 832 -> 869); the IL pattern once the tree streams from HBM and
  // the bytes bound it (10 M, 1.1 GB, at 1080p: 543 vs 528).  Crossover taken
  // at 600 MB; SRT_GLOBAL_FUSED_MODE=1/0 forces either.
  const char* fu_env = std::getenv("SRT_GLOBAL_FUSED_MODE");
  c->fused = fu_env ? fu_env[0] == '1' : scene_mb < 600.0;
  // Waves per SIMD of the fused instance: 5 (8-entry rings, some spills) while the tree is small
  // enough that the extra rays in flight pay (torus knot 262 k, 20 MB: 5,405 -> 5,650 Mrays/s; Rubik
  // forced global +6%; 100 k +2%; 300 k, 30 MB: +1%), else 4 (1 M, 101 MB: -7% with 5; 3 M: -7%).
  // Crossover taken at 48 MB; SRT_GLOBAL_WAVES_MODE=4/5 forces either.
  const char* gw_env = std::getenv("SRT_GLOBAL_WAVES_MODE");
  c->global_waves = gw_env ? (gw_env[0] == '5' ? 5 : 4) : (scene_mb < 48.0 ? 5 : 4);
  // Triangle slots (LayoutTris) for every scene read through L2 (none of 1 MB fits the LDS copy):
  // fewer lines per leaf step (A/B on one box, kernel ms: C5 10 M 4096² 820 -> 773 with the IL leaf
  // step's own-record reads, 3 M 58.4 -> 56.5, 1 M 34.1 -> 32.6, torus knot 27.4 -> 27.4, Rubik
  // unchanged).  SRT_TRI_ALIGN=1/0 forces either.  Leaves and each BVH's triangle range are
  // remapped; a record keeps its triangle's input index (C.z) for the closest-hit query.
  const char* ta_env = std::getenv("SRT_TRI_ALIGN");
  const bool tri_align = ta_env ? ta_env[0] == '1' : scene_mb >= 1.0;
  std::vector<uint32_t> tslot;
  uint32_t n_tslots = n_tris;
  // (the slots stay below 3 n_tris: a gap is at most two records per leaf)
  const bool tris_laid =
      tri_align && n_tris < (1u << 30) && LayoutTris(nodes, n_nodes, reach, n_tris, &tslot, &n_tslots);
  uint32_t max_leaf = 0;
  for (uint32_t i = 0; i < n_nodes; ++i)
    if (reach[i]) max_leaf = std::max(max_leaf, nodes[i].prim_count);
  // The fused instance's LDS copy of the tree's top levels (traversal.hpp trav_fused): LDS reads bypass
  // the vector-memory pipeline that bounds these kernels.  Laid out first, as deep
  // as fits the LDS one block may take beside its rings and the light records (SRT_TOP_DEPTH=d forces d
  // levels, 0 none).  The ring's entry size is the one Launch will use
  // (lds_ok below, with the dense node count: a line-aligned layout's padding only matters past 2^24
  // slots, where Launch then finds the region too large and skips it).  A depth's region size comes from
  // the layout's first pass alone (TopRegionSlots, bounded by the depth); the full layout runs once.
  uint32_t n_top = 0;
  int top_depth = 0;
  {
    const char* td_env = std::getenv("SRT_TOP_DEPTH");
    if (c->fused && scene_mb >= 1.0 && !(td_env && std::atoi(td_env) <= 0)) {
      const bool pack = n_tslots < (1u << 24) && n_nodes + srt::kNodePad < (1u << 24) && max_leaf < 256;
      const int gblock = GlobalBlock(true, c->global_waves);
      const size_t ring = (size_t)gblock * (pack ? 2 : 3) * sizeof(uint32_t) * (size_t)srt::global_ring(c->global_waves);
      // beside the light records (the ones set, at least the reference's six, src/main.cpp:584-589, and the
      // zero record) when they fit their LDS cap, as Launch places them (LightLdsBytes); the material
      // records take what the region leaves (Launch)
      const size_t lb = 2 * sizeof(float4) * (std::max<size_t>(c->h_lights.size(), 6) + 1);
      const size_t lm = lb <= 8192 ? lb : 0;
      const size_t share = GlobalBlockLds(gblock, c->global_waves);
      const size_t budget = share > ring + lm + 64 ? share - ring - lm - 64 : 0;
      top_depth = td_env ? std::atoi(td_env) : 12;
      for (; top_depth > 0; --top_depth) {  // the deepest whole levels that fit
        if (!TopRegionSlots(nodes, n_nodes, bvhs, n_bvhs, align, top_depth, &n_top)) {
          top_depth = 0;
          break;
        }
        if (td_env || ((2 * (size_t)n_top + 2 + 3) / 4) * srt::kNodeBlkF4 * sizeof(float4) <= budget) break;
      }
    }
  }
  bool laid = !(lay_env && lay_env[0] == '0') &&
              LayoutNodes(nodes, n_nodes, bvhs, n_bvhs, align, &remap, &n_slots, top_depth, &n_top);
  if (!laid) n_top = 0;
  auto tsl = [&](uint32_t t) { return tris_laid ? tslot[t] : t; };
  for (auto& r : tri_ranges)
    if (r.first < r.second) r = {tsl(r.first), tsl(r.second - 1) + 1};
  if (!laid) {
    remap.resize(n_nodes);
    for (uint32_t i = 0; i < n_nodes; ++i) remap[i] = i;
    n_slots = n_nodes;
  }
  std::vector<float4> hn(2 * ((size_t)n_slots + 1 + srt::kNodePad), make_float4(0, 0, 0, 0));
  bool pairs_aligned = true;
  for (uint32_t i = 0; i < n_nodes; ++i) {
    // (a node no traversal reaches keeps a zero record: its indices were never range-checked)
    if (remap[i] == 0xFFFFFFFFu || !reach[i]) continue;
    const srt_bvh_node& n = nodes[i];
    uint32_t first = n.first_child_or_prim_index;
    if (n.prim_count == 0) {  // internal: c0's slot, less 1 when c1 is internal (its pair then follows)
      // The flag promises that c1's own child pair is the next pair of the array.  LayoutNodes
      // places it there whenever it lays the pair out itself; a pair shared with an earlier
      // BVH record's tree keeps its first placement, so the flag is set only when the
      // remapped slots say so.
      const uint32_t c0 = n.first_child_or_prim_index;
      const srt_bvh_node& n1 = nodes[c0 + 1];
      first = remap[first];
      if (laid && n1.prim_count == 0 && remap[n1.first_child_or_prim_index] == remap[c0] + 2) first -= 1;
      if (((first | (laid ? 1u : 0u)) & 1u) == 0) pairs_aligned = false;  // overlapping sibling pairs
    } else {
      first = tsl(first);
    }
    float w0, w1;
    std::memcpy(&w0, &first, 4);
    std::memcpy(&w1, &n.prim_count, 4);
    hn[2 * (size_t)remap[i] + 2] = make_float4(n.min_bounds[0], n.min_bounds[1], n.min_bounds[2], w0);
    hn[2 * (size_t)remap[i] + 3] = make_float4(n.max_bounds[0], n.max_bounds[1], n.max_bounds[2], w1);
  }
  // Treelet scheduling (wavefront mode, wavefront.hpp): a copy of the node array in which every internal
  // node at depth td of some tree (walked from every BVH root and from slot 0, where the ghost records
  // start) is a treelet root -- its count kTreeletCnt, its child index the treelet's id -- and whose
  // nodes with a treelet root as right child lose the right-spine flag (the top kernel must make the root
  // current, not expand it).  Every path deeper than td passes a root, so the top-level stack holds < td
  // entries.  Chosen for trees past the Infinity Cache, with ~1 MB treelets (SRT_TREELETS=1/0 forces it,
  // SRT_TREELET_DEPTH sets td).
  FreeDev(c->d_nodes_t);
  FreeDev(c->d_troot);
  c->d_nodes_t = nullptr;
  c->d_troot = nullptr;
  c->n_treelets = 0;
  {
    uint32_t max_leaf_in = 0;
    for (uint32_t i = 0; i < n_nodes; ++i)
      if (reach[i]) max_leaf_in = std::max(max_leaf_in, nodes[i].prim_count);
    int td = c->treelet_depth;
    if (td == 0) {  // ~1 MB of nodes + triangles per treelet
      td = 1;
      while (td < srt::kTopStack - 1 && scene_mb / (double)(1u << (td + 1)) >= 1.0) ++td;
    }
    c->tl_scene = false;  // opt-in (measured slower than sample_kernel: DESIGN.md section 5, "Wavefront mode")
    const bool want = c->treelets >= 0 ? c->treelets == 1 : c->tl_scene;
    if (want && max_leaf_in < srt::kTreeletCnt && depth > td) {
      std::vector<float4> hf(hn);
      std::vector<uint32_t> troot;
      std::vector<int32_t> tid_of(n_slots, -1);
      auto u32 = [](float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; };
      auto f32 = [](uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; };
      std::vector<uint32_t> roots{0};
      for (uint32_t b = 0; b < n_bvhs; ++b) roots.push_back(remap[bvhs[b].first_index]);
      std::vector<std::pair<uint32_t, int>> st;
      const uint32_t ror = laid ? 1u : 0u;
      for (uint32_t r : roots) {
        st.push_back({r, 0});
        while (!st.empty()) {
          auto [sl, d] = st.back();
          st.pop_back();
          if (u32(hn[2 * (size_t)sl + 3].w) != 0u || tid_of[sl] >= 0) continue;  // a leaf, or a root already
          const uint32_t first = u32(hn[2 * (size_t)sl + 2].w);
          if (d == td) {
            tid_of[sl] = (int32_t)troot.size();
            troot.push_back(first);
            hf[2 * (size_t)sl + 2].w = f32((uint32_t)tid_of[sl]);
            hf[2 * (size_t)sl + 3].w = f32(srt::kTreeletCnt);
            continue;
          }
          const uint32_t ref0 = first | ror;
          st.push_back({ref0, d + 1});
          st.push_back({ref0 + 1, d + 1});
        }
      }
      for (uint32_t sl = 0; sl < n_slots && ror; ++sl) {  // no right-spine step onto a treelet root
        const uint32_t first = u32(hn[2 * (size_t)sl + 2].w);
        if (tid_of[sl] >= 0 || u32(hn[2 * (size_t)sl + 3].w) != 0u || (first & 1u)) continue;
        if (first + 2 < n_slots && tid_of[first + 2] >= 0) hf[2 * (size_t)sl + 2].w = f32(first | 1u);
      }
      if (!troot.empty()) {
        HIP_OK(hipMalloc(&c->d_nodes_t, hf.size() * sizeof(float4)));
        HIP_OK(hipMalloc(&c->d_troot, troot.size() * sizeof(uint32_t)));
        HIP_OK(hipMemcpyAsync(c->d_nodes_t, hf.data(), hf.size() * sizeof(float4), hipMemcpyHostToDevice, c->stream));
        HIP_OK(hipMemcpyAsync(c->d_troot, troot.data(), troot.size() * sizeof(uint32_t), hipMemcpyHostToDevice,
                              c->stream));
        HIP_OK(hipStreamSynchronize(c->stream));
        c->n_treelets = (uint32_t)troot.size();
      }
    }
  }
  // materials -> shading materials (raytrace_utils.glsl:140-175); one zero
  // record appended for out-of-range material indices (OOB SSBO reads = 0)
  std::vector<float4> hm(2 * ((size_t)n_mats + 1), make_float4(0, 0, 0, 0));
  bool sampled = false;
  for (uint32_t i = 0; i <= n_mats; ++i) {
    srt_material_obj m{};
    if (i < n_mats) m = mats[i];
    float alb[3] = {m.diffuse[0], m.diffuse[1], m.diffuse[2]};
    uint32_t tex = 0;  // sampled texture + 1 (0: constant albedo)
    if (m.use_texture) {
      for (int k = 0; k < 3; ++k) alb[k] = tex_albedo ? tex_albedo[3 * (size_t)i + k] : 0.0f;
      if (!tex_albedo) {
        const uint64_t h = (uint64_t)m.handle[0] | ((uint64_t)m.handle[1] << 32);
        tex = h < 0xFFFFFFFFull ? (uint32_t)h + 1 : 0xFFFFFFFFu;  // unknown handles sample zero
        sampled = true;
      }
    }
    const float rough = 1.0f / (m.specular_ex + 0.0000001f);
    float tf;
    std::memcpy(&tf, &tex, 4);
    hm[2 * (size_t)i] = make_float4(alb[0], alb[1], alb[2], rough);
    hm[2 * (size_t)i + 1] = make_float4(m.specular[0], m.specular[1], m.specular[2], tf);
  }
  // triangles (at their slots): v0, e1 = v1 - v0, e2 = v2 - v0, material, input index
  // kTriPad zero records past the end: a multi-triangle leaf step may read (and discard) them
  std::vector<float4> ht(3 * ((size_t)n_tslots + srt::kTriPad), make_float4(0, 0, 0, 0));
  auto vert = [&](uint32_t i, int k) -> float { return i < n_verts ? verts[i].vertex[k] : 0.0f; };
  for (uint32_t t = 0; t < n_tris; ++t) {
    const size_t st = tsl(t);
    const srt_triangle& tr = tris[t];
    float v0[3], e1[3], e2[3];
    for (int k = 0; k < 3; ++k) {
      v0[k] = vert(tr.v0_idx, k);
      e1[k] = vert(tr.v1_idx, k) - v0[k];
      e2[k] = vert(tr.v2_idx, k) - v0[k];
    }
    const uint32_t mi = tr.material_idx < n_mats ? tr.material_idx : n_mats;
    float mf, tf;
    std::memcpy(&mf, &mi, 4);
    std::memcpy(&tf, &t, 4);
    ht[3 * st + 0] = make_float4(v0[0], v0[1], v0[2], e1[0]);
    ht[3 * st + 1] = make_float4(e1[1], e1[2], e2[0], e2[1]);
    ht[3 * st + 2] = make_float4(e2[2], mf, tf, 0.0f);
  }
  // vertex uvs per triangle, for the materials that sample a texture
  std::vector<float4> huv;
  if (sampled) {
    huv.assign(2 * (size_t)n_tslots, make_float4(0, 0, 0, 0));
    auto uv = [&](uint32_t i, int k) -> float { return i < n_verts ? verts[i].texture[k] : 0.0f; };
    for (uint32_t t = 0; t < n_tris; ++t) {
      const srt_triangle& tr = tris[t];
      const size_t st = tsl(t);
      huv[2 * st] = make_float4(uv(tr.v0_idx, 0), uv(tr.v0_idx, 1), uv(tr.v1_idx, 0), uv(tr.v1_idx, 1));
      huv[2 * st + 1] = make_float4(uv(tr.v2_idx, 0), uv(tr.v2_idx, 1), 0.0f, 0.0f);
    }
  }
  FreeDev(c->d_nodes); FreeDev(c->d_mats); FreeDev(c->d_tris); FreeDev(c->d_tri_uv);
  c->d_nodes = nullptr; c->d_mats = nullptr; c->d_tris = nullptr; c->d_tri_uv = nullptr;
  c->scene_ok = false;
  if (sampled && n_tris) {
    HIP_OK(hipMalloc(&c->d_tri_uv, huv.size() * sizeof(float4)));
    HIP_OK(hipMemcpyAsync(c->d_tri_uv, huv.data(), huv.size() * sizeof(float4), hipMemcpyHostToDevice, c->stream));
  }
  HIP_OK(hipMalloc(&c->d_nodes, hn.size() * sizeof(float4)));
  HIP_OK(hipMalloc(&c->d_mats, hm.size() * sizeof(float4)));
  HIP_OK(hipMalloc(&c->d_tris, ht.size() * sizeof(float4)));
  HIP_OK(hipMemcpyAsync(c->d_nodes, hn.data(), hn.size() * sizeof(float4), hipMemcpyHostToDevice, c->stream));
  HIP_OK(hipMemcpyAsync(c->d_mats, hm.data(), hm.size() * sizeof(float4), hipMemcpyHostToDevice, c->stream));
  HIP_OK(hipMemcpyAsync(c->d_tris, ht.data(), ht.size() * sizeof(float4), hipMemcpyHostToDevice, c->stream));
  HIP_OK(hipStreamSynchronize(c->stream));
  c->h_bvhs.assign(bvhs, bvhs + n_bvhs);
  for (auto& r : c->h_bvhs) r.first_index = remap[r.first_index];  // roots in the device layout
  c->bvh_tris = std::move(tri_ranges);
  c->sample_textures = sampled;
  c->bvhs_dirty = true;
  c->n_nodes = n_slots + srt::kNodePad;
  c->top_f4 = n_top > 0 ? 2 * (int)n_top + 2 : 0;  // float4 of slots [0, n_top)
  c->top_depth = n_top > 0 ? top_depth : 0;
  c->ref_or = laid ? 1u : 0u;
  c->n_tris = n_tslots;  // device records (slots)
  c->n_mats = n_mats;
  c->stack_entries = depth + 1;
  c->lds_ok = n_tslots < (1u << 24) && n_slots + srt::kNodePad < (1u << 24) && max_leaf < 256;
  // cooperative loads (SRT_COOP builds) carry a request's float4 index in kCoopIdxBits bits: larger
  // arrays (only reachable with SRT_GLOBAL_FUSED_MODE=1 past 600 MB) take the IL instance
  if (SRT_COOP && (2ull * ((uint64_t)c->n_nodes + 1) + 8 >= (1ull << srt::kCoopIdxBits) ||
                   3ull * ((uint64_t)n_tslots + srt::kTriPad) >= (1ull << srt::kCoopIdxBits)))
    c->fused = false;
  c->pairs_aligned = pairs_aligned;
  c->scene_ok = true;
  if (c->bvh_count == 0) c->bvh_count = n_bvhs;
  // the zero records beyond n_bvhs traverse from node 0 with a zero ray
  // (raytrace_compute.glsl:144-147 reading bvhs[i] out of bounds)
  return SRT_OK;
}

int srt_upload_textures(srt_context* c, const srt_texture* textures, uint32_t n) {
  if (!c || (n && !textures)) return SRT_ERR_INVALID;
  if (int rq = Quiesce(c)) return rq;
  std::vector<uint4> info(std::max<uint32_t>(n, 1), make_uint4(0, 0, 0, 0));
  size_t total = 0;
  for (uint32_t i = 0; i < n; ++i) {
    const srt_texture& t = textures[i];
    if (!t.texels || t.width <= 0 || t.height <= 0 || t.channels < 1 || t.channels > 4) {
      srt::SetError("texture " + std::to_string(i) + ": bad size, channel count or texel pointer");
      return SRT_ERR_INVALID;
    }
    info[i] = make_uint4((uint32_t)total, (uint32_t)t.width, (uint32_t)t.height, 0u);
    total += (size_t)t.width * (size_t)t.height;
    if (total >= (1ull << 32)) {
      srt::SetError("textures hold more than 2^32 texels");
      return SRT_ERR_LIMIT;
    }
  }
  // GL_RED reads (r, 0, 0), a 2-channel file (r, g, 0); channel values are c / 255 (unorm8)
#if SRT_TEX8
  // the file's bytes, RGBA8 (the kernel's unorm8 reads c / 255 exactly): 4 B a texel
  using Texel = uint32_t;
  std::vector<Texel> tx(std::max<size_t>(total, 1), 0u);
#else
  using Texel = float4;  // RGBA32F, c / 255
  std::vector<Texel> tx(std::max<size_t>(total, 1), make_float4(0, 0, 0, 0));
#endif
  for (uint32_t i = 0; i < n; ++i) {
    const srt_texture& t = textures[i];
    const size_t m = (size_t)t.width * (size_t)t.height;
    for (size_t k = 0; k < m; ++k) {
      const uint8_t* p = t.texels + k * t.channels;
      uint32_t v[3] = {0u, 0u, 0u};
      for (int ch = 0; ch < t.channels && ch < 3; ++ch) v[ch] = p[ch];
      if (t.channels == 2) v[2] = 0u;
#if SRT_TEX8
      tx[info[i].x + k] = v[0] | (v[1] << 8) | (v[2] << 16);
#else
      tx[info[i].x + k] = make_float4((float)v[0] / 255.0f, (float)v[1] / 255.0f, (float)v[2] / 255.0f, 1.0f);
#endif
    }
  }
  HIP_OK(hipSetDevice(c->device));
  FreeDev(c->d_tex); FreeDev(c->d_tex_info);
  c->d_tex = nullptr; c->d_tex_info = nullptr; c->n_tex = 0;
  HIP_OK(hipMalloc(&c->d_tex, tx.size() * sizeof(Texel)));
  HIP_OK(hipMalloc(&c->d_tex_info, info.size() * sizeof(uint4)));
  HIP_OK(hipMemcpyAsync(c->d_tex, tx.data(), tx.size() * sizeof(Texel), hipMemcpyHostToDevice, c->stream));
  HIP_OK(hipMemcpyAsync(c->d_tex_info, info.data(), info.size() * sizeof(uint4), hipMemcpyHostToDevice, c->stream));
  HIP_OK(hipStreamSynchronize(c->stream));
  c->n_tex = n;
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
  if (int rq = Quiesce(c)) return rq;
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

namespace {
constexpr char kCkptMagic[8] = {'S', 'R', 'T', 'C', 'K', 'P', 'T', '1'};
struct CkptHeader {
  char magic[8];
  int32_t version, width, local_rows, rank, nranks, band_rows, accum_frames, pad;
  float cam[12];  // cameraOrigin, cameraDirection, cameraUp, cameraRight
  uint64_t payload_bytes;
  uint32_t payload_crc, header_crc;
};
uint32_t Crc32(const void* p, size_t n) {
  return (uint32_t)crc32(0L, static_cast<const Bytef*>(p), (uInt)n);
}
}  // namespace

int srt_checkpoint_save(srt_context* c, const char* path) {
  if (!c || !path || !c->d_accum || c->img_w <= 0 || c->img_rows <= 0) return SRT_ERR_INVALID;
  std::vector<float> acc((size_t)c->img_w * c->img_rows * 4);
  int rc = srt_read_accum(c, acc.data(), acc.size() * sizeof(float));
  if (rc) return rc;
  CkptHeader h{};
  std::memcpy(h.magic, kCkptMagic, 8);
  h.version = 1;
  h.width = c->img_w;
  h.local_rows = c->img_rows;
  h.rank = c->rank;
  h.nranks = c->nranks;
  h.band_rows = c->band_rows;
  h.accum_frames = c->accum_frames;
  const float* cam[4] = {c->cam_origin, c->cam_dir, c->cam_up, c->cam_right};
  for (int i = 0; i < 4; ++i) std::memcpy(h.cam + 3 * i, cam[i], 3 * sizeof(float));
  h.payload_bytes = acc.size() * sizeof(float);
  h.payload_crc = Crc32(acc.data(), h.payload_bytes);
  h.header_crc = Crc32(&h, offsetof(CkptHeader, header_crc));
  const std::string tmp = std::string(path) + ".tmp";
  FILE* f = std::fopen(tmp.c_str(), "wb");
  if (!f) {
    srt::SetError(std::string("srt_checkpoint_save: cannot open ") + tmp);
    return SRT_ERR_IO;
  }
  const bool ok = std::fwrite(&h, sizeof h, 1, f) == 1 && std::fwrite(acc.data(), 1, h.payload_bytes, f) == h.payload_bytes;
  if (std::fclose(f) != 0 || !ok || std::rename(tmp.c_str(), path) != 0) {  // the old file survives a failed save
    std::remove(tmp.c_str());
    srt::SetError(std::string("srt_checkpoint_save: cannot write ") + path);
    return SRT_ERR_IO;
  }
  return SRT_OK;
}

int srt_checkpoint_load(srt_context* c, const char* path, int32_t* accum_frames) {
  if (!c || !path || !c->d_accum) return SRT_ERR_INVALID;
  FILE* f = std::fopen(path, "rb");
  if (!f) {
    srt::SetError(std::string("srt_checkpoint_load: cannot open ") + path);
    return SRT_ERR_IO;
  }
  CkptHeader h{};
  std::vector<float> acc;
  bool ok = std::fread(&h, sizeof h, 1, f) == 1 && std::memcmp(h.magic, kCkptMagic, 8) == 0 && h.version == 1 &&
            h.header_crc == Crc32(&h, offsetof(CkptHeader, header_crc));
  if (ok && (h.width != c->img_w || h.local_rows != c->img_rows || h.rank != c->rank || h.nranks != c->nranks ||
             h.band_rows != c->band_rows || h.payload_bytes != (uint64_t)c->img_w * c->img_rows * 16)) {
    std::fclose(f);
    srt::SetError("srt_checkpoint_load: the checkpoint's frame or tiling differs from the context's");
    return SRT_ERR_INVALID;
  }
  if (ok) {
    acc.resize(h.payload_bytes / sizeof(float));
    ok = std::fread(acc.data(), 1, h.payload_bytes, f) == h.payload_bytes &&
         Crc32(acc.data(), h.payload_bytes) == h.payload_crc;
  }
  std::fclose(f);
  if (!ok) {
    srt::SetError(std::string("srt_checkpoint_load: not a valid checkpoint (truncated or corrupt): ") + path);
    return SRT_ERR_IO;
  }
  const int rc = srt_write_accum(c, acc.data(), h.payload_bytes);
  if (rc) return rc;
  c->accum_frames = h.accum_frames;
  float* cam[4] = {c->cam_origin, c->cam_dir, c->cam_up, c->cam_right};
  for (int i = 0; i < 4; ++i) std::memcpy(cam[i], h.cam + 3 * i, 3 * sizeof(float));
  if (accum_frames) *accum_frames = h.accum_frames;
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
  return c ? srt::AssembleBandsOn(c, c->stream, gathered, nranks, rows_pad, band_rows, frames, accum_full, out_full)
           : SRT_ERR_INVALID;
}

int srt_assemble_output_bands(srt_context* c, const void* gathered_rgba8, int nranks, int rows_pad, int band_rows,
                              void* out_full) {
  return c ? srt::AssembleOutputOn(c, c->stream, gathered_rgba8, nranks, rows_pad, band_rows, c->W, c->H, out_full)
           : SRT_ERR_INVALID;
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
  kp.ref_or = c->ref_or;
  kp.tris = c->d_tris;
  kp.bvhs = c->d_bvhs;
  kp.bvh_count = c->bvh_count;
  kp.stack_entries = c->stack_entries;
  kp.stats = c->d_stats;
  // one 3-dword stack entry per tree level and lane: in LDS while 64 KiB hold a 256- (down to 64-)
  // lane block's stacks, else in HBM (lane-interleaved; trees deeper than ~85 levels)
  const size_t entry = 3 * sizeof(uint32_t) * (size_t)kp.stack_entries;
  int block = 256;
  while (block > 64 && (size_t)block * entry > 65536) block >>= 1;
  const bool hbm_stack = (size_t)block * entry > 65536;
  const size_t lds = hbm_stack ? 0 : (size_t)block * entry;
  // device buffers, freed on every path
  struct Buf {
    void* p = nullptr;
    ~Buf() { if (p) (void)hipFree(p); }
  } d_rays, d_hits, d_t, d_stk;
  HIP_OK(hipMalloc(&d_rays.p, sizeof(srt_ray) * n));
  HIP_OK(hipMalloc(&d_hits.p, sizeof(uint32_t) * n));
  HIP_OK(hipMalloc(&d_t.p, sizeof(float) * n));
  const size_t grid = (n + block - 1) / block;
  if (hbm_stack) HIP_OK(hipMalloc(&d_stk.p, entry * grid * (size_t)block));  // one area per block
  HIP_OK(hipMemcpyAsync(d_rays.p, rays, sizeof(srt_ray) * n, hipMemcpyHostToDevice, c->stream));
  HIP_OK(hipMemsetAsync(c->d_stats, 0, sizeof(unsigned long long) * srt::ST_N, c->stream));
  hipLaunchKernelGGL(srt::closest_kernel, dim3((unsigned)grid), dim3(block), lds, c->stream, kp,
                     static_cast<const srt_ray*>(d_rays.p), n, static_cast<uint32_t*>(d_hits.p),
                     static_cast<float*>(d_t.p), static_cast<uint32_t*>(d_stk.p));
  HIP_OK(hipGetLastError());
  unsigned long long s[srt::ST_N];
  HIP_OK(hipMemcpyAsync(hits, d_hits.p, sizeof(uint32_t) * n, hipMemcpyDeviceToHost, c->stream));
  HIP_OK(hipMemcpyAsync(t_out, d_t.p, sizeof(float) * n, hipMemcpyDeviceToHost, c->stream));
  HIP_OK(hipMemcpyAsync(s, c->d_stats, sizeof(s), hipMemcpyDeviceToHost, c->stream));
  HIP_OK(hipStreamSynchronize(c->stream));
  c->stats.rays += n;
  c->stats.nodes += s[srt::ST_NODES];
  c->stats.tris += s[srt::ST_TRIS];
  return SRT_OK;
}

}  // extern "C"
