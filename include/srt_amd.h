/*
 * srt_amd.h -- C ABI of the MI355X-native path-tracing inner loop.
 *
 * Drop-in boundary for matteobir12/simple-ray-tracer's GL compute path.  The
 * reference has no plugin system: its boundary is the GL program + uniform +
 * binding contract that src/main.cpp drives every frame.  Each entry point
 * below names the reference interface it replaces (file:line).  Plain
 * pointers and sizes only; status codes instead of std::terminate /
 * std::runtime_error.  Everything runs on one HIP stream per context.
 */
#ifndef SRT_AMD_H
#define SRT_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SRT_ABI_VERSION 2  /* 2: srt_stats.bounce_cap */

/* ---- status codes ---- */
enum {
  SRT_OK = 0,
  SRT_ERR_INVALID = 1,    /* bad argument / size mismatch */
  SRT_ERR_HIP = 2,        /* HIP runtime error (message: srt_last_error) */
  SRT_ERR_NOT_FOUND = 3,  /* unknown uniform name (reference: silently ignored) */
  SRT_ERR_IO = 4,         /* file open / parse failure */
  SRT_ERR_STATE = 5,      /* missing scene / noise / images before dispatch */
  SRT_ERR_LIMIT = 6       /* BVH deeper than the traversal stack supports */
};

/* ---- std430 records: the reference's SSBO / texel-buffer contents ----
 * These are the host structs AssetUtils::UploadModelDataToGPU packs
 * (src/asset_utils/gpu_loader.cpp:11-41) and the GLSL declares
 * (shaders/raytrace_types.glsl:19-107).  The library re-lays them on device. */
typedef struct { uint32_t first_index, count, pad0, pad1; float frame[16]; } srt_bvh_record;   /* 80 B, frame column-major (glm::mat4) */
typedef struct { float min_bounds[3]; uint32_t first_child_or_prim_index;
                 float max_bounds[3]; uint32_t prim_count; } srt_bvh_node;                    /* 32 B */
typedef struct { float diffuse[3]; float specular_ex; float specular[3]; uint32_t use_texture;
                 uint32_t handle[2]; uint32_t pad0, pad1; } srt_material_obj;                  /* 48 B */
typedef struct { uint32_t v0_idx, v1_idx, v2_idx, material_idx; } srt_triangle;                 /* 16 B */
typedef struct { float vertex[3]; float pad0; float texture[2]; float pad1[2]; } srt_vertex;    /* 32 B */
typedef struct { float position[3]; float intensity; float color[3]; float pad1; } srt_light;  /* 32 B, raytracer/light.h:54-63 */
/* A decoded 8-bit texture as stb_image returns it (gpu_texture.h:29-33): rows
 * top first, `channels` (1-4) interleaved bytes per texel. */
typedef struct { const uint8_t* texels; int32_t width, height, channels; } srt_texture;
typedef struct { float origin[3]; float pad0; float direction[3]; float intersection_distance; } srt_ray; /* 32 B, common/types.h:15-35 */

/* Work counters of a counting launch. */
typedef struct {
  uint64_t rays;        /* CheckHit queries: camera + bounce + shadow */
  uint64_t nodes;       /* BVH node box tests (32 B each) */
  uint64_t tris;        /* triangle tests (40 B each) */
  uint64_t rng_u;       /* noiseUniformTex fetches (4 B) */
  uint64_t rng_sq;      /* noiseTex .xy fetches (8 B) */
  uint64_t light_reads; /* light records (32 B) */
  uint64_t mat_reads;   /* mesh material fetches (48 B) */
  uint64_t samples;     /* path samples */
  uint64_t stack_overflow; /* traversal stack overflows (cannot happen for a BVH srt_upload_scene accepted) */
  uint64_t max_stack;      /* deepest traversal stack */
  uint64_t bounce_cap;     /* paths cut after 2^20 bounces (the reference's loop has no cap; env SRT_BOUNCE_CAP) */
} srt_stats;

typedef struct srt_context srt_context;
typedef struct srt_model srt_model;
typedef struct srt_scene srt_scene;

const char* srt_last_error(void);
int srt_abi_version(void);
/* Identity of this library's device code: a hash of the kernel sources and the hipcc flags they were
 * built with (16 hex digits).  Measurements keyed to code (profiles/counters.json) carry it. */
const char* srt_code_hash(void);

/* ===================== Graphics::Compute (the dispatch API) =====================
 * replaces Graphics::Compute(path) + Init() (include/graphics/shader.h:46-55,
 * src/graphics/Shader.cpp:14-26,125-157) and Compute::CreateComputeProgram
 * (include/compute/create_compute_program.h:46-72).  `stream` is a
 * hipStream_t (NULL = the context creates its own). */
int srt_create(int device, void* stream, srt_context** out);

/* Compute::CreateComputeProgram (include/compute/create_compute_program.h:46-72):
 * a program handle, or 0 with the log on stderr as the reference prints it
 * ("err opening<path>" when the file cannot be opened, :13-16; "compile
 * error:" for a program with no MI355X kernel, :31-40).  The program is the
 * file's basename: raytrace_compute.glsl -> SRT_PROGRAM_RAYTRACE (the path
 * tracer, srt_dispatch / srt_render_frames), ray_intersects.glsl ->
 * SRT_PROGRAM_INTERSECT (the closest-hit test kernel, srt_trace_closest).
 * "builtin:raytrace_compute" / "builtin:ray_intersects" name them without a
 * file.  The GLSL text is not compiled: the kernels are HIP code objects. */
#define SRT_PROGRAM_RAYTRACE 1u
#define SRT_PROGRAM_INTERSECT 2u
uint32_t srt_program_create(const char* path);
/* glDeleteProgram: SRT_OK for a handle srt_program_create returned, else SRT_ERR_INVALID. */
int srt_program_delete(uint32_t program);
int srt_destroy(srt_context* ctx);
void* srt_stream(srt_context* ctx);

/* Uniform setters (Shader.cpp:79-122,159-212): names are the GLSL uniforms
 * resetAccumBuffer, showModel (bool); Width, Height, accumFrames, lightCount,
 * maxDepth (int); bvh_count (uint); cameraOrigin, cameraDirection,
 * cameraUp, cameraRight (vec3).  Unknown name -> SRT_ERR_NOT_FOUND (the
 * reference silently ignores it: callers may too). */
int srt_set_bool(srt_context* ctx, const char* name, int v);
int srt_set_int(srt_context* ctx, const char* name, int v);
int srt_set_uint(srt_context* ctx, const char* name, uint32_t v);
int srt_set_float(srt_context* ctx, const char* name, float v);
int srt_set_vec3(srt_context* ctx, const char* name, float x, float y, float z);

/* glDispatchCompute(gx, gy, 1) of raytrace_compute.glsl (src/main.cpp:706):
 * one 8x8 invocation tile per group, one path sample per pixel. */
int srt_dispatch(srt_context* ctx, uint32_t groups_x, uint32_t groups_y);
/* glMemoryBarrier + glFinish (src/main.cpp:709-718). */
int srt_finish(srt_context* ctx);

/* Fused progressive render: equivalent to `nframes` consecutive dispatches
 * with accumFrames = frame_first .. frame_first+nframes-1 and
 * resetAccumBuffer = false (bit-identical accum buffer); the RGBA8 image is
 * written once, for the last frame, when write_output != 0.  Counting
 * launches (count != 0) also fill srt_get_stats.  Leaves the accumFrames
 * uniform at frame_first + nframes - 1, as the last dispatch would. */
int srt_render_frames(srt_context* ctx, int frame_first, int nframes, int write_output, int count);
int srt_get_stats(srt_context* ctx, srt_stats* out);
/* The counted rays by kind, of the same counting launches as srt_get_stats: [0] camera rays (one per
 * path sample, GetRay), [1] shadow rays (CheckLightOccluded, raytrace_compute.glsl:167-176), [2] bounce
 * rays (SampleIndirectNew's next ray, :224-290); they sum to srt_stats.rays. */
int srt_ray_kinds(srt_context* ctx, uint64_t kinds[3]);
/* Device time of the path-tracing kernel launches of the last render call: the
 * union of each sample_kernel / sphere_kernel launch's span (its first wave's
 * start to its last wave's end on the GPU's 100 MHz real-time clock), plus HIP
 * events around pool and wavefront launches.  Waits for the render.  Overlapped
 * pipeline slots (SRT_PIPELINE_OVERLAP) dispatch a launch while others run, so
 * its span may include time it shared the CUs with them. */
int srt_last_kernel_ms(srt_context* ctx, float* ms);
/* The device time of every sample_kernel / sphere_kernel launch since the
 * previous call -- the union of their spans, the time during which some launch
 * of the context ran (launches in series add their spans; overlapped ones, which
 * the hardware may also run side by side, count their shared time once) -- and
 * how many: a timed loop of renders enqueued without synchronising reads its
 * kernel time once.  Waits for them.  SRT_ERR_LIMIT when more than 4096 launches
 * went unread (their records are overwritten). */
int srt_kernel_time(srt_context* ctx, double* total_ms, int* launches);
int srt_reset_stats(srt_context* ctx);  /* also zeroes the NaN counter */
/* Failure detection: path samples with a NaN component accumulated since the
 * context was created or srt_reset_stats (always counted, by the ordered
 * per-pixel sum).  The reference tests each sample for NaN after adding it to
 * the accumulation and discards the result (raytrace_compute.glsl:408-410). */
int srt_nan_samples(srt_context* ctx, uint64_t* out);

/* Row-band sharding for multi-GPU: this context owns bands b of `band_rows`
 * rows with b % nranks == rank; its images hold only those rows, packed in
 * band order.  Default: rank 0 of 1 (whole frame). */
int srt_set_tiling(srt_context* ctx, int rank, int nranks, int band_rows);
int srt_local_rows(srt_context* ctx);
/* The context's HIP device, and a uniform's current value (glGetUniformiv): the int / uint / bool
 * uniforms above by name; SRT_ERR_NOT_FOUND for other names.  Read-only names report what the
 * uploaded scene's size chose for global-scene mode's timed kernel:
 *   "scene.fused"        1: fused sub-steps, 0: the IL pattern;
 *   "scene.global_waves" waves per SIMD of the fused instance;
 *   "scene.tri_slots"    device triangle records (more than the scene's triangles when small leaves are
 *                        laid out line by line for a tree streamed from HBM);
 *   "scene.top_depth", "scene.top_f4"  levels and float4 of the tree's top region the fused instance
 *                        copies into each block's LDS (0: none);
 *   "scene.wavefront", "scene.wf_waves", "scene.treelets"  the opt-in wavefront mode's choices;
 * and of the last render call:
 *   "launch.chunks"      its sample launches (one per sample-buffer chunk);
 *   "launch.overlap"     1 when its launches ran on the pipeline slots, each free to start while the
 *                        previous one drains (SRT_PIPELINE_OVERLAP), 0 otherwise (counting, pool and
 *                        wavefront launches run in series);
 *   "launch.top_f4"      the top region its global-scene launch copied (0: none: the region did not fit
 *                        beside the rings and the light and material records);
 *   "launch.blocks_per_cu", "launch.block"  resident blocks per CU and lanes per block of its last
 *                        sample_kernel, sphere_kernel or pool_kernel launch (0 after a wavefront-mode render);
 *                        the occupancy API's answer capped by gfx950's LDS allocation unit (1/128 of the
 *                        CU's 160 KiB: n blocks run together only up to floor(128 / n) * 1,280 B each);
 *   "launch.mats_lds"    1 when that launch read the material records from LDS (0: from HBM, where they
 *                        did not fit the LDS its blocks may take). */
int srt_device(srt_context* ctx);
int srt_get_int(srt_context* ctx, const char* name, int* v);

/* ===================== multi-GPU frame from one host process =====================
 * The reference's frame loop (src/main.cpp:657-725) drives one GL context.  A C++ embedder tiles the
 * same frame over the GPUs of a node with a group of contexts, one per device, each holding the scene,
 * noise and lights (srt_upload_scene etc. on every context): context i renders the row bands b of
 * `band_rows` rows with b % n == i, with global pixel coordinates, and encodes its own rows' sRGB8
 * (accumFrames is one uniform for all).  Per frame, one gather moves every context's sRGB8 rows
 * (4 B/px) to context 0 -- ncclGather over xGMI (RCCL, one communicator per device from
 * ncclCommInitAll, librccl loaded at srt_group_create) on a gather stream of its own per device,
 * double-buffered so frame k's gather overlaps frame k+1's render -- and context 0 de-interleaves
 * the bands.  The radiance (RGBA32F) stays distributed: it is gathered only when the full
 * accumulation image is asked for (srt_group_read_accum, srt_group_image_pointers' accum_dev).
 * The frame is bit-identical to one device's.  A device list that repeats a device (RCCL takes one rank
 * per device), or SRT_GROUP_TRANSPORT=copy, gathers with device-to-device copies instead.
 * Contexts stay owned by the caller and must outlive the group; srt_group_destroy detaches each from
 * the freed band images without allocating (tiling rank 0 of 1, no images: a dispatch returns
 * SRT_ERR_STATE until srt_alloc_images or srt_set_image_buffers gives it images again).
 * srt_group_create fails (SRT_ERR_HIP) unless every RCCL communicator counts exactly n ranks. */
typedef struct srt_group srt_group;
int srt_group_create(srt_context* const* ctxs, int n, int band_rows, srt_group** out);
int srt_group_destroy(srt_group* g);
/* "contexts"; "ranks" (ncclCommCount of the communicators, or the contexts under the copy
 * transport); "gathers.output" / "gathers.accum" (gathers issued so far); "bytes.output" /
 * "bytes.accum" (bytes one such gather moves into context 0, in KiB). */
int srt_group_get_int(srt_group* g, const char* name, int* v);
/* Each context's srt_last_kernel_ms (its sample launches' spans), n entries. */
int srt_group_last_kernel_ms(srt_group* g, float* ms, int n);
/* Each context's srt_kernel_time since the previous call (n entries each): a timed loop of group
 * renders enqueued back to back reads every device's kernel time once, after it. */
int srt_group_kernel_time(srt_group* g, double* total_ms, int* launches, int n);
/* Each context's part of the per-frame exchange since the previous call (n entries each), from HIP
 * events on its gather stream: from the frame's own rows being rendered to the end of its part of
 * the gather (the RCCL gather waits for every rank; copies for context 0's buffer), and for context
 * 0 to the end of the frame's assembly (the de-interleave); summed, with the frame count.
 * SRT_ERR_LIMIT when more than 4096 frames went unread. */
int srt_group_exchange_time(srt_group* g, double* total_ms, int* frames, int n);
/* Uniform setters broadcast to every context (the names of srt_set_*). */
int srt_group_set_bool(srt_group* g, const char* name, int v);
int srt_group_set_int(srt_group* g, const char* name, int v);
int srt_group_set_uint(srt_group* g, const char* name, uint32_t v);
int srt_group_set_vec3(srt_group* g, const char* name, float x, float y, float z);
/* After Width/Height: tiles the contexts (srt_set_tiling i of n), gives each an equal-size padded band
 * image (the gather's send buffer) and context 0 the full-frame images. */
int srt_group_alloc_images(srt_group* g);
/* glDispatchCompute on every context (srt_dispatch), then the sRGB8 gather and the full-frame image0
 * (not for a resetAccumBuffer dispatch, as the reference's reset dispatch returns before its store;
 * pixels outside the dispatch extent keep their values). */
int srt_group_dispatch(srt_group* g, uint32_t groups_x, uint32_t groups_y);
/* srt_render_frames on every context, then the sRGB8 gather and the image0 of the last frame. */
int srt_group_render_frames(srt_group* g, int frame_first, int nframes);
int srt_group_finish(srt_group* g);  /* glFinish on every device (render and gather streams) */
/* The full frame (Width x Height) on the host, or its device pointers on context 0's device (asking
 * for accum_dev enqueues the radiance gather; read after srt_group_finish). */
int srt_group_read_accum(srt_group* g, float* host_rgba32f, size_t bytes);
int srt_group_read_output(srt_group* g, uint8_t* host_rgba8, size_t bytes);
int srt_group_image_pointers(srt_group* g, void** accum_dev, void** out_dev);
/* "rccl" or "copy". */
const char* srt_group_transport(srt_group* g);

/* ===================== bindings (SSBOs / texel buffers / images) ===================== */
/* AssetUtils::UploadModelDataToGPU (include/asset_utils/gpu_loader.h:19,
 * src/asset_utils/gpu_loader.cpp:63-183): the five SSBOs at bindings 5..9.
 * Materials with use_texture take their albedo from `tex_albedo` (3 floats
 * per material: the texture() result, constant because the reference's
 * loader leaves every uv at (0,0), types.h:105) when it is non-NULL.  When it
 * is NULL they sample texture `handle` (64-bit, handle[0] | handle[1] << 32;
 * see srt_upload_textures) at the hit's interpolated uv, as
 * TriangleToSupportedMat does (raytrace_utils.glsl:144-166); an unknown
 * handle samples as zero.  Sampling needs the BVH records that can hit
 * (non-zero frame) to own disjoint triangle ranges, as UploadModelDataToGPU
 * builds them (checked at dispatch). */
int srt_upload_scene(srt_context* ctx,
                     const srt_bvh_record* bvhs, uint32_t n_bvhs,
                     const srt_bvh_node* nodes, uint32_t n_nodes,
                     const srt_material_obj* mats, const float* tex_albedo, uint32_t n_mats,
                     const srt_triangle* tris, uint32_t n_tris,
                     const srt_vertex* verts, uint32_t n_verts);
/* GPUTexture(file, true) + GetHandle() (gpu_texture.h:24-68,133-137): the
 * textures sampled by use_texture materials; texture i gets handle i.
 * Replaces any previous set.  Sampling contract:
 * level 0, GL_LINEAR, GL_REPEAT, texels c/255. */
int srt_upload_textures(srt_context* ctx, const srt_texture* textures, uint32_t n);
/* The same sampler on the host: texture(sampler2D, vec2(s, t)).xyz. */
int srt_texture_sample(const srt_texture* tex, float s, float t, float rgb[3]);
/* AssetUtils::UpdateModelMatrix (gpu_loader.cpp:185-196). */
int srt_update_model_matrix(srt_context* ctx, uint32_t index, const float frame[16]);
/* light SSBO at binding 4 (src/main.cpp:688-692). */
int srt_set_lights(srt_context* ctx, const srt_light* lights, uint32_t n);
/* noiseTex / noiseUniformTex texel buffers at units 1,2 (src/main.cpp:269-301):
 * RGB32F, `texels` = Width*Height each. */
int srt_set_noise(srt_context* ctx, const float* noise_rgb, const float* noise_uniform_rgb, size_t texels);
/* image0 (RGBA8 output) and image3 (RGBA32F accumulation), sized from the
 * current Width/Height uniforms (and tiling).  Read back packed local rows. */
int srt_alloc_images(srt_context* ctx);
int srt_read_accum(srt_context* ctx, float* host_rgba32f, size_t bytes);
int srt_read_output(srt_context* ctx, uint8_t* host_rgba8, size_t bytes);
int srt_write_accum(srt_context* ctx, const float* host_rgba32f, size_t bytes);
/* Checkpoint / resume of a progressive render (the reference has none: its
 * accumulation lives in a GL texture).  save writes the accumulation image
 * (this context's local rows), accumFrames and the camera uniforms, with
 * CRC32s, to `path` (via a temporary file, so an old checkpoint survives a
 * failed save).  load checks that the frame size and tiling match the context
 * (SRT_ERR_INVALID if not; SRT_ERR_IO for a missing, truncated or corrupt
 * file), restores the image and the uniforms and returns accumFrames; the
 * next frames (accumFrames + 1, ...) then continue bit-identically to an
 * uninterrupted render. */
int srt_checkpoint_save(srt_context* ctx, const char* path);
int srt_checkpoint_load(srt_context* ctx, const char* path, int32_t* accum_frames);
/* Output stage (replaces the GL display quad, src/main.cpp:303-349): write an
 * RGBA8 image to `path`, PNG (RGBA) or binary PPM (RGB) by extension.
 * flip_y != 0 writes the kernel's bottom row (j = 0) last, as displayed.
 * SRT_ERR_IO on a file error, SRT_ERR_INVALID for an unknown extension. */
int srt_image_write(const char* path, const uint8_t* rgba8, int width, int height, int flip_y);
/* The context's current image0 (its local rows) through srt_image_write. */
int srt_write_output(srt_context* ctx, const char* path, int flip_y);
/* Device pointers of the images (for RCCL gathers without a host copy). */
int srt_image_pointers(srt_context* ctx, void** accum_dev, void** out_dev);
/* Use caller-owned device buffers (>= local_rows * Width RGBA32F / RGBA8) as
 * image3 / image0, e.g. tensors an RCCL gather reads from. */
int srt_set_image_buffers(srt_context* ctx, void* accum_dev, void* out_dev);
/* Root side of the multi-GPU frame: `gathered` holds nranks blocks of
 * rows_pad packed local rows (rank order, bands of band_rows rows dealt
 * round-robin); writes the full-frame (Width x Height) RGBA32F accumulation
 * image and sRGB8 image for accumFrames = `frames` (either output may be
 * NULL).  Enqueued on the context's stream. */
int srt_assemble_bands(srt_context* ctx, const void* gathered, int nranks, int rows_pad, int band_rows, int frames,
                       void* accum_full, void* out_full);
/* The per-frame form: every rank encoded its own rows' sRGB8 (image0; accumFrames is one uniform
 * for all ranks), `gathered_rgba8` holds nranks blocks of rows_pad packed RGBA8 rows, and only the
 * full-frame image0 is written -- 4 B per pixel cross the interconnect instead of 16. */
int srt_assemble_output_bands(srt_context* ctx, const void* gathered_rgba8, int nranks, int rows_pad, int band_rows,
                              void* out_full);

/* Closest-hit query: the test kernel ray_intersects.glsl:135-161 fed through
 * AssetUtils::UpdateRays (gpu_loader.cpp:198-210); hits[i] = triangle index
 * or 0xFFFFFFFF, t_out[i] = the final intersection_distance.  Host arrays. */
int srt_trace_closest(srt_context* ctx, const srt_ray* rays, uint32_t n, uint32_t* hits, float* t_out);

/* ===================== scene producers (host, CPU) ===================== */
/* AssetUtils::LoadObject / ParseOBJ / ParseMTL / ConvertCPUGeometryToModel
 * (src/asset_utils/model_loader.cpp:20-365) + BVH<GPU::Triangle>
 * (include/intersection_utils/bvh.h:40-148).  `obj_path` is the .obj file;
 * MTL files resolve relative to its directory. */
int srt_model_load(const char* obj_path, srt_model** out);
/* srt_model_load with flags.  SRT_LOAD_TEXCOORDS gives each vertex the uv of
 * its face's `vt` index, i.e. the loader with has_texcoords set
 * (model_loader.cpp:322-324), which the reference never does. */
#define SRT_LOAD_TEXCOORDS 1u
int srt_model_load_ex(const char* obj_path, uint32_t flags, srt_model** out);
/* Build a model from raw triangles (one material). */
int srt_model_from_triangles(const float* xyz9, uint32_t n_tris, const float kd[3], const float ks[3], float ns,
                             srt_model** out);
int srt_model_free(srt_model* m);
/* counts: [0]=triangles [1]=vertices [2]=nodes [3]=leaves [4]=max depth [5]=materials [6]=faces dropped */
int srt_model_info(const srt_model* m, uint64_t counts[8], float root_min[3], float root_max[3]);
/* One model's host arrays in the reference's AssetUtils::Model shape, before
 * UploadModelDataToGPU flattens them (indices local to the model):
 * model_bvh.GetBVH() nodes (intersection_utils/bvh.h:23-30), GetPrims()
 * (asset_utils/types.h:25-28), model_materials (types.h:31-37; tex_albedo =
 * the texture's sample at uv (0,0)) and vertex_data_buffer (types.h:17-23).
 * A caller keeping the reference's own gpu_loader.cpp:63-133 flattening feeds
 * the result to srt_upload_scene (tests/cpp/test_ref_loader.cpp). */
typedef struct { float min_bounds[3]; float max_bounds[3];
                 uint32_t first_child, first_prim_index, prim_count; } srt_host_bvh_node;   /* 36 B */
typedef struct { float diffuse[3]; float specular[3]; float specular_ex; uint32_t use_texture;
                 float tex_albedo[3]; } srt_host_material;                                  /* 44 B */
/* sizes: [0]=nodes [1]=prims [2]=materials [3]=vertices */
int srt_model_sizes(const srt_model* m, uint32_t sizes[4]);
int srt_model_copy(const srt_model* m, srt_host_bvh_node* nodes, srt_triangle* prims, srt_host_material* mats,
                   srt_vertex* verts);
/* The BVH's primitive permutation (bvh.h:66-72: GetPrims()[i] is the loader's
 * all_triangles[input_index[i]], model_loader.cpp:299-331); sizes[1] entries. */
int srt_model_prim_order(const srt_model* m, uint32_t* input_index);

/* Flatten models exactly as UploadModelDataToGPU does (index rebasing). */
int srt_scene_build(const srt_model* const* models, uint32_t n_models, srt_scene** out);
int srt_scene_free(srt_scene* s);
/* sizes: [0]=bvhs [1]=nodes [2]=materials [3]=triangles [4]=vertices */
int srt_scene_sizes(const srt_scene* s, uint32_t sizes[5]);
int srt_scene_copy(const srt_scene* s, srt_bvh_record* bvhs, srt_bvh_node* nodes, srt_material_obj* mats,
                   float* tex_albedo, srt_triangle* tris, srt_vertex* verts);
/* Loader order of the flattened triangles: triangle i (the index srt_trace_closest
 * returns) is input triangle input_index[i] of the models' concatenated loader
 * order (each model's offset + srt_model_prim_order); sizes[3] entries.  The
 * reference's ray KAT (BVH_intergration_tests.cpp:94) is stated in that order. */
int srt_scene_tri_order(const srt_scene* s, uint32_t* input_index);
/* Textures of the scene's use_texture materials (material handle = index);
 * sample_textures = 1 when a model was loaded with SRT_LOAD_TEXCOORDS. */
int srt_scene_texture_count(const srt_scene* s, uint32_t* n, int* sample_textures);
/* Texture i; `out->texels` points into the scene (valid while it lives). */
int srt_scene_texture(const srt_scene* s, uint32_t i, srt_texture* out);
/* srt_upload_scene of the flattened arrays; with sample_textures it also
 * uploads the textures and passes tex_albedo = NULL. */
int srt_upload_scene_obj(srt_context* ctx, const srt_scene* s);

/* Noise texel buffers of UpdateNoiseTex (src/main.cpp:269-301) from the
 * never-seeded glibc rand() stream (include/common/utils.h:22-51).
 * vec3 argument draw order: gcc_order != 0 draws z, y, x (g++, the
 * reference's compiler); 0 draws x, y, z (clang).  Outputs RGB32F. */
int srt_noise_generate(uint32_t texels, int gcc_order, float* noise_rgb, float* noise_uniform_rgb);
/* glibc rand() (TYPE_3, seed 1) restated: first n outputs. */
int srt_glibc_rand(uint32_t n, int32_t* out);

/* Camera::Reset + UpdateCameraVectors (src/raytracer/camera.cpp:120-136,187-212):
 * origin/front/up/right for the model (show_model != 0) or sphere scene. */
int srt_camera_reset(int show_model, float origin[3], float front[3], float up[3], float right[3]);
/* Camera::Rotate(yaw, pitch) basis from angles in degrees (camera.cpp:107-136). */
int srt_camera_basis(float yaw_deg, float pitch_deg, float front[3], float up[3], float right[3]);

/* ---- interactive mode ---------------------------------
 * RayTracer::Camera's state (include/raytracer/camera.h:30-96).  frame_counter
 * is MoveAndRotate's function-static counter (camera.cpp:175), kept per camera
 * (the reference app has one camera, so the two agree). */
typedef struct {
  float position[3], front[3], up[3], right[3];
  float yaw, pitch;          /* degrees */
  int32_t show_model;
  int32_t frame_counter;
} srt_camera;
enum { SRT_MOVE_FORWARD = 0, SRT_MOVE_BACKWARD, SRT_MOVE_LEFT, SRT_MOVE_RIGHT, SRT_MOVE_UP, SRT_MOVE_DOWN };
/* Camera(settings) + Initialize + Reset as src/main.cpp:439-441 does; frame_counter = 0. */
int srt_camera_init(srt_camera* cam, int show_model);
/* Camera::Reset (camera.cpp:187-212); keeps frame_counter, as the static does. */
int srt_camera_state_reset(srt_camera* cam);
/* Camera::MoveForward .. MoveDown (camera.cpp:71-105); direction = SRT_MOVE_*. */
int srt_camera_move(srt_camera* cam, int direction, float delta);
/* Camera::Rotate (camera.cpp:107-118): pitch clamped to +-89, yaw unwrapped. */
int srt_camera_rotate(srt_camera* cam, float yaw_offset, float pitch_offset);
/* Camera::MoveAndRotate (camera.cpp:138-185).  SRT_ERR_INVALID (camera
 * unchanged) where the reference's yaw wrap loop would never end (an infinite
 * yaw, or one whose ulp exceeds 720). */
int srt_camera_move_and_rotate(srt_camera* cam, float delta_time, const float movement_delta[3],
                               const float rotation_delta[2], float movement_speed);
/* The frame loop's host side, src/main.cpp:622-659: resetAccumBuffer is set
 * (and *accum_frames zeroed) on any input -- |movement| > 1e-4, |rotation| >
 * 1e-4 or the left mouse button held -- or when the input handler's reset flag
 * is up (the flag is then cleared, input_handler.cpp:160-168); the camera moves
 * with MoveAndRotate(delta_time, ..., 1.0); *accum_frames is incremented.  The
 * caller then sets resetAccumBuffer = *reset_buffer, accumFrames and the camera
 * uniforms and dispatches, as main.cpp:668-706 does. */
int srt_progressive_frame(srt_camera* cam, const float movement_delta[3], const float rotation_delta[2],
                          int mouse_left, int32_t* should_reset_buffer, float delta_time, int32_t* accum_frames,
                          int32_t* reset_buffer);

#ifdef __cplusplus
}
#endif
#endif
