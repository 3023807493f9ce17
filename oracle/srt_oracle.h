/*
 * srt_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement ("oracle") of the reference path tracer's hot path
 * (matteobir12/simple-ray-tracer, shaders/{raytrace_compute,ray_intersects,
 * brdf,raytrace_utils,raytrace_types}.glsl).  It is the checker for the HIP
 * kernels in simple-ray-tracer_amd/csrc: only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it.  Nothing in the product links
 * or calls it.
 *
 * The oracle consumes the scene in the REFERENCE std430 layouts (the arrays
 * that AssetUtils::UploadModelDataToGPU builds, src/asset_utils/gpu_loader.cpp:
 * 11-41), not the re-laid device layout the product uses, so the product's
 * re-layout is checked too.
 *
 * Parity status: the reference GLSL kernel cannot run in this container (no
 * GL context, no glm/GLFW), so this restatement is pinned by
 * the known answers the survey re-derived for the reference's own test scene
 * (Rubik ingest counts, the BVH_intergration_tests.cpp traversal KAT rays) and
 * by the arithmetic contract in DESIGN.md section 3 ("fp32 semantics").
 */
#ifndef SRT_ORACLE_H
#define SRT_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* std430 mirrors: raytrace_types.glsl:32-38 / gpu_loader.cpp:11-17 (80 B) */
typedef struct { uint32_t first_index, count, pad0, pad1; float frame[16]; } OrBVH;
/* raytrace_types.glsl:41-46 / gpu_loader.cpp:19-24 (32 B) */
typedef struct { float mn[3]; uint32_t first; float mx[3]; uint32_t count; } OrNode;
/* raytrace_types.glsl:19-27 / gpu_loader.cpp:26-34 (48 B) */
typedef struct { float diffuse[3]; float Ns; float Ks[3]; uint32_t use_texture;
                 uint32_t handle[2]; uint32_t pad[2]; } OrMaterial;
/* raytrace_types.glsl:50-55 / gpu_loader.cpp:36-41 (16 B) */
typedef struct { uint32_t v[3]; uint32_t mat; } OrTri;
/* raytrace_types.glsl:58-61 / asset_utils/types.h:17-23 (32 B) */
typedef struct { float pos[3]; float pad0; float uv[2]; float pad1[2]; } OrVertex;
/* raytrace_types.glsl:102-107 / raytracer/light.h:54-63 (32 B) */
typedef struct { float pos[3]; float intensity; float color[3]; float pad; } OrLight;
/* raytrace_types.glsl:89-94 / common/types.h:15-35 (32 B) */
typedef struct { float o[3]; float pad; float d[3]; float t; } OrRay;

typedef struct {
  const OrBVH* bvhs;       uint32_t n_bvhs;      /* real records; bvhs[i>=n] read as zeros */
  const OrNode* nodes;     uint32_t n_nodes;
  const OrMaterial* mats;  uint32_t n_mats;
  const float* tex_albedo; /* 3 floats per material: texture(sampler, uv) result, used when use_texture
                              (NULL: sample tex_* at the hit's uv) */
  const OrTri* tris;       uint32_t n_tris;
  const OrVertex* verts;   uint32_t n_verts;
  const OrLight* lights;   uint32_t n_lights;  /* lights[i >= n_lights] reads as zeros */
  const float* noise;      /* RGB32F, W*H texels (binding 1, noiseTex) */
  const float* noise_u;    /* RGB32F, W*H texels (binding 2, noiseUniformTex) */
  /* textures sampled by use_texture materials when tex_albedo is NULL:
   * texture h = material handle, tex_info[4h..4h+3] = first byte, width,
   * height, channels; tex_texels = 8-bit texels (stb_image layout) */
  const uint8_t* tex_texels;
  const uint32_t* tex_info;
  uint32_t n_tex;
} OrScene;

/* The per-dispatch uniforms (raytrace_compute.glsl:18-31,39; ray_intersects.glsl:8) */
typedef struct {
  int width, height;
  int accum_frames;
  int reset;
  int show_model;
  uint32_t bvh_count;
  int light_count;
  int max_depth;             /* settings.maxDepth, raytrace_compute.glsl:370 (5) */
  float cam_origin[3], cam_dir[3], cam_up[3], cam_right[3];
} OrFrame;

typedef struct {
  uint64_t rays;         /* CheckHit invocations (camera + bounce + shadow) */
  uint64_t nodes;        /* BVH node box tests */
  uint64_t tris;         /* triangle tests */
  uint64_t rng_u;        /* noiseUniformTex fetches */
  uint64_t rng_sq;       /* noiseTex (.xy) fetches */
  uint64_t light_reads;  /* light records read */
  uint64_t mat_reads;    /* mesh material fetches */
  uint64_t samples;      /* path samples */
  uint64_t stack_overflow; /* traversals that would overflow stack[64] */
  uint64_t max_stack;    /* deepest stack seen */
  uint64_t shadow_rays;  /* of `rays`: CheckLightOccluded's queries (raytrace_compute.glsl:167-176) */
} OrStats;

/* One glDispatchCompute of raytrace_compute.glsl over rows [y0, y1) and all
 * columns (accum = RGBA32F W*H*4 floats, out = RGBA8 W*H*4 bytes). */
void oracle_dispatch(const OrScene* s, const OrFrame* f, float* accum, uint8_t* out,
                     int y0, int y1, OrStats* st);

/* Consecutive dispatches frame_first .. frame_first+nframes-1 (accumFrames),
 * reset=false, over rows [y0,y1), optionally on `threads` OpenMP threads. */
void oracle_render(const OrScene* s, const OrFrame* f, int frame_first, int nframes,
                   float* accum, uint8_t* out, int y0, int y1, int threads, OrStats* st);

/* As oracle_render over an explicit list of rows (bounded CPU-baseline samples). */
void oracle_render_rows(const OrScene* s, const OrFrame* f, int frame_first, int nframes, float* accum,
                        uint8_t* out, const int* rows, int nrows, int threads, OrStats* st);

/* Closest-hit only: the (commented) test kernel ray_intersects.glsl:135-161. */
void oracle_trace_closest(const OrScene* s, uint32_t bvh_count, const OrRay* rays, int n,
                          uint32_t* hits, float* t_out, float* n_out, OrStats* st);

/* Arithmetic contract primitives, exported so tests can pin them. */
float oracle_sin(float x);
float oracle_cos(float x);
float oracle_pow(float x, float y);
float oracle_pow5(float x);
float oracle_rand_float(float sx, float sy);
/* 'A' + ORACLE_CONTRACT of this build (srt_oracle.c: the contract variants) */
int oracle_contract(void);

#ifdef __cplusplus
}
#endif
#endif
