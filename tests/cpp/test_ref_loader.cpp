// test_ref_loader.cpp -- the reference's own upload path feeding the C ABI.
//
// AssetUtils::UploadModelDataToGPU (src/asset_utils/gpu_loader.cpp:63-183)
// flattens every Model into five process-global std430 arrays and hands them
// to glBufferData.  The drop-in keeps that code and replaces only the five
// glBufferData calls with one srt_upload_scene call.
// This test restates the reference's GPU structs (gpu_loader.cpp:11-41, with
// PackedVertexData from asset_utils/types.h:17-23) and its flattening loop
// verbatim in shape, over Models in the reference's host shape
// (AssetUtils::Model: model_bvh.GetBVH()/GetPrims(), model_materials,
// vertex_data_buffer; filled through srt_model_copy), then:
//   arrays  <objects_dir>            (CPU) the flattened bytes equal srt_scene_build's
//   render  <objects_dir> <out>      (GPU) srt_upload_scene of those arrays renders
//                                    the same frame as srt_upload_scene_obj; the frame is
//                                    written to <out>.accum for an oracle check
// Prints "OK" on success.
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "srt_amd.h"

namespace ref {  // the reference's types, restated (glm::vec3 = 3 floats, glm::mat4 = 16 floats column-major)
struct vec3 { float x, y, z; };
struct vec2 { float x, y; };
struct mat4 { float m[16]; };

// asset_utils/types.h:17-23
struct PackedVertexData {
  alignas(16) vec3 vertex;
  alignas(8) vec2 texture;
};
// asset_utils/types.h:25-28
struct Triangle {
  uint32_t vertex_idxs[3];
  uint32_t material_idx;
};
// intersection_utils/bvh.h:23-30
struct BVHNode {
  vec3 min_bounds;
  vec3 max_bounds;
  uint32_t first_child;
  uint32_t first_prim_index;
  uint32_t prim_count;
};
// asset_utils/types.h:31-37 (GPUTexture reduced to its handle)
struct Material {
  vec3 diffuse;
  vec3 specular;
  float specular_ex;
  uint64_t texture_handle;
  bool use_texture;
};
// asset_utils/types.h:39-52 with BVH<GPU::Triangle>'s accessors
struct BVH {
  std::vector<BVHNode> nodes;
  std::vector<Triangle> prims;
  const std::vector<BVHNode>& GetBVH() const { return nodes; }
  const std::vector<Triangle>& GetPrims() const { return prims; }
};
struct Model {
  BVH model_bvh;
  std::vector<Material> model_materials;
  std::vector<PackedVertexData> vertex_data_buffer;
};

// gpu_loader.cpp:11-41
struct GPUBVH {
  uint32_t first_index;
  uint32_t count;
  uint32_t _pad0;
  uint32_t _pad1;
  mat4 frame = {{1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1}};
};
struct GPUBVHNode {
  vec3 min_bounds;
  uint32_t first_child_or_prim_index;
  vec3 max_bounds;
  uint32_t prim_count;
};
struct GPUMaterial {
  vec3 diffuse;
  float specular_ex;
  vec3 specular;
  uint32_t use_texture = 0;
  uint64_t handle;
  uint32_t _pad0;
  uint32_t _pad1;
};
struct GPUTriangle {
  uint32_t v0_idx;
  uint32_t v1_idx;
  uint32_t v2_idx;
  uint32_t material_idx;
};

// the std430 records are the C ABI's records, byte for byte
static_assert(sizeof(GPUBVH) == sizeof(srt_bvh_record) && offsetof(GPUBVH, frame) == offsetof(srt_bvh_record, frame), "");
static_assert(sizeof(GPUBVHNode) == sizeof(srt_bvh_node) && offsetof(GPUBVHNode, max_bounds) == 16, "");
static_assert(sizeof(GPUMaterial) == sizeof(srt_material_obj) && offsetof(GPUMaterial, handle) == 32 &&
              offsetof(GPUMaterial, use_texture) == offsetof(srt_material_obj, use_texture), "");
static_assert(sizeof(GPUTriangle) == sizeof(srt_triangle), "");
static_assert(sizeof(PackedVertexData) == sizeof(srt_vertex) && offsetof(PackedVertexData, texture) == 16, "");

// gpu_loader.cpp:42-52
std::vector<GPUBVH> g_bvhs;
std::vector<GPUBVHNode> g_bvh_nodes;
std::vector<GPUMaterial> g_materials;
std::vector<GPUTriangle> g_triangles;
std::vector<PackedVertexData> g_vertices;
std::vector<float> g_tex_albedo;  // added by the drop-in: the texture() result per material (uv is (0,0))

// gpu_loader.cpp:63-133, unchanged in shape; the glBufferData calls (:135-182) become srt_upload_scene
void UploadModelDataToGPU(const std::vector<Model*>& models, srt_context* ctx) {
  g_bvhs.clear();
  g_bvh_nodes.clear();
  g_materials.clear();
  g_triangles.clear();
  g_vertices.clear();
  g_tex_albedo.clear();
  uint32_t cur_BVH_node_off = 0, cur_triangle_off = 0, cur_material_off = 0, cur_vertex_off = 0;
  for (const auto& model_ptr : models) {
    if (!model_ptr) throw std::runtime_error("Model was null!");
    const Model& model = *model_ptr;
    const uint32_t model_mat_off = cur_material_off;
    for (const auto& mat : model.model_materials) {
      GPUMaterial gpu_mat;
      gpu_mat.diffuse = mat.diffuse;
      gpu_mat.specular = mat.specular;
      gpu_mat.specular_ex = mat.specular_ex;
      gpu_mat.use_texture = mat.use_texture;
      gpu_mat.handle = mat.use_texture ? mat.texture_handle : 0;
      gpu_mat._pad0 = gpu_mat._pad1 = 0;
      g_materials.push_back(gpu_mat);
    }
    cur_material_off += (uint32_t)model.model_materials.size();
    const uint32_t model_vert_off = cur_vertex_off;
    for (const auto& v : model.vertex_data_buffer) g_vertices.push_back(v);
    cur_vertex_off += (uint32_t)model.vertex_data_buffer.size();
    const auto& bvh = model.model_bvh;
    GPUBVH gpu_BVH;
    gpu_BVH.first_index = cur_BVH_node_off;
    gpu_BVH.count = (uint32_t)bvh.GetBVH().size();
    gpu_BVH._pad0 = gpu_BVH._pad1 = 0;
    g_bvhs.push_back(gpu_BVH);
    const uint32_t local_tri_offset = cur_triangle_off;
    for (const auto& tri : bvh.GetPrims()) {
      GPUTriangle gpu_tri;
      gpu_tri.v0_idx = tri.vertex_idxs[0] + model_vert_off;
      gpu_tri.v1_idx = tri.vertex_idxs[1] + model_vert_off;
      gpu_tri.v2_idx = tri.vertex_idxs[2] + model_vert_off;
      gpu_tri.material_idx = tri.material_idx + model_mat_off;
      g_triangles.push_back(gpu_tri);
    }
    cur_triangle_off += (uint32_t)bvh.GetPrims().size();
    for (const auto& node : bvh.GetBVH()) {
      GPUBVHNode gpu_node;
      gpu_node.min_bounds = node.min_bounds;
      gpu_node.max_bounds = node.max_bounds;
      gpu_node.first_child_or_prim_index =
          node.prim_count > 0 ? node.first_prim_index + local_tri_offset : node.first_child + cur_BVH_node_off;
      gpu_node.prim_count = node.prim_count;
      g_bvh_nodes.push_back(gpu_node);
    }
    cur_BVH_node_off += gpu_BVH.count;
  }
  if (!ctx) return;
  // replaces glGenBuffers + glBufferData + glBindBufferBase (gpu_loader.cpp:135-182)
  const int rc = srt_upload_scene(ctx, reinterpret_cast<const srt_bvh_record*>(g_bvhs.data()), (uint32_t)g_bvhs.size(),
                                  reinterpret_cast<const srt_bvh_node*>(g_bvh_nodes.data()), (uint32_t)g_bvh_nodes.size(),
                                  reinterpret_cast<const srt_material_obj*>(g_materials.data()), g_tex_albedo.data(),
                                  (uint32_t)g_materials.size(), reinterpret_cast<const srt_triangle*>(g_triangles.data()),
                                  (uint32_t)g_triangles.size(),
                                  reinterpret_cast<const srt_vertex*>(g_vertices.data()), (uint32_t)g_vertices.size());
  if (rc != SRT_OK) throw std::runtime_error(std::string("srt_upload_scene: ") + srt_last_error());
}
}  // namespace ref

static int fail(const std::string& what) {
  std::printf("FAIL %s (%s)\n", what.c_str(), srt_last_error());
  return 1;
}

// A Model in the reference's host shape, from the loader + BVH builder (srt_model_copy).
static ref::Model HostModel(srt_model* m) {
  uint32_t sz[4];
  if (srt_model_sizes(m, sz) != SRT_OK) throw std::runtime_error("srt_model_sizes");
  std::vector<srt_host_bvh_node> nodes(sz[0]);
  std::vector<srt_triangle> prims(sz[1]);
  std::vector<srt_host_material> mats(sz[2]);
  std::vector<srt_vertex> verts(sz[3]);
  if (srt_model_copy(m, nodes.data(), prims.data(), mats.data(), verts.data()) != SRT_OK)
    throw std::runtime_error("srt_model_copy");
  ref::Model r;
  for (const auto& n : nodes)
    r.model_bvh.nodes.push_back({{n.min_bounds[0], n.min_bounds[1], n.min_bounds[2]},
                                 {n.max_bounds[0], n.max_bounds[1], n.max_bounds[2]},
                                 n.first_child, n.first_prim_index, n.prim_count});
  for (const auto& p : prims) r.model_bvh.prims.push_back({{p.v0_idx, p.v1_idx, p.v2_idx}, p.material_idx});
  for (const auto& a : mats)
    r.model_materials.push_back({{a.diffuse[0], a.diffuse[1], a.diffuse[2]},
                                 {a.specular[0], a.specular[1], a.specular[2]}, a.specular_ex, 0, a.use_texture != 0});
  for (const auto& v : verts) {
    ref::PackedVertexData p{};
    p.vertex = {v.vertex[0], v.vertex[1], v.vertex[2]};
    p.texture = {v.texture[0], v.texture[1]};
    r.vertex_data_buffer.push_back(p);
  }
  return r;
}

// the drop-in's one addition: texture() at uv (0,0) per material, in g_materials order
static void TexAlbedo(const std::vector<srt_model*>& ms) {
  for (srt_model* m : ms) {
    uint32_t sz[4];
    srt_model_sizes(m, sz);
    std::vector<srt_host_material> mats(sz[2]);
    srt_model_copy(m, nullptr, nullptr, mats.data(), nullptr);
    for (const auto& a : mats) ref::g_tex_albedo.insert(ref::g_tex_albedo.end(), a.tex_albedo, a.tex_albedo + 3);
  }
}

int main(int argc, char** argv) {
  if (argc < 3) return fail("usage: test_ref_loader arrays|render <objects_dir> [out_prefix]");
  const std::string mode = argv[1], objects = argv[2];
  srt_model* a = nullptr;
  srt_model* b = nullptr;
  if (srt_model_load((objects + "Rubik/Rubik.obj").c_str(), &a) != SRT_OK) return fail("load a");
  if (srt_model_load((objects + "Rubik/Rubik.obj").c_str(), &b) != SRT_OK) return fail("load b");
  ref::Model ma = HostModel(a), mb = HostModel(b);
  std::vector<ref::Model*> models = {&ma, &mb};
  try {
    ref::UploadModelDataToGPU({nullptr}, nullptr);
    return fail("null model accepted");
  } catch (const std::runtime_error& e) {
    if (std::string(e.what()) != "Model was null!") return fail("wrong null-model error");
  }

  if (mode == "arrays") {
    ref::UploadModelDataToGPU(models, nullptr);
    const srt_model* ms[2] = {a, b};
    srt_scene* s = nullptr;
    if (srt_scene_build(ms, 2, &s) != SRT_OK) return fail("srt_scene_build");
    uint32_t sz[5];
    srt_scene_sizes(s, sz);
    if (sz[0] != ref::g_bvhs.size() || sz[1] != ref::g_bvh_nodes.size() || sz[2] != ref::g_materials.size() ||
        sz[3] != ref::g_triangles.size() || sz[4] != ref::g_vertices.size())
      return fail("array sizes");
    std::vector<srt_bvh_record> bv(sz[0]);
    std::vector<srt_bvh_node> nd(sz[1]);
    std::vector<srt_material_obj> mt(sz[2]);
    std::vector<srt_triangle> tr(sz[3]);
    std::vector<srt_vertex> vx(sz[4]);
    srt_scene_copy(s, bv.data(), nd.data(), mt.data(), nullptr, tr.data(), vx.data());
    srt_scene_free(s);
    auto same = [](const void* x, const void* y, size_t n) { return std::memcmp(x, y, n) == 0; };
    if (!same(bv.data(), ref::g_bvhs.data(), bv.size() * sizeof(srt_bvh_record))) return fail("bvh records");
    if (!same(nd.data(), ref::g_bvh_nodes.data(), nd.size() * sizeof(srt_bvh_node))) return fail("nodes");
    if (!same(mt.data(), ref::g_materials.data(), mt.size() * sizeof(srt_material_obj))) return fail("materials");
    if (!same(tr.data(), ref::g_triangles.data(), tr.size() * sizeof(srt_triangle))) return fail("triangles");
    if (!same(vx.data(), ref::g_vertices.data(), vx.size() * sizeof(srt_vertex))) return fail("vertices");
    std::printf("OK arrays: %zu bvhs %zu nodes %zu materials %zu triangles %zu vertices\n", bv.size(), nd.size(),
                mt.size(), tr.size(), vx.size());
    return 0;
  }

  if (mode != "render") return fail("unknown mode");
  const std::string out_prefix = argc > 3 ? argv[3] : "";
  const int W = 64, H = 48;
  std::vector<float> noise(3 * W * H), noise_u(3 * W * H);
  srt_noise_generate(W * H, 1, noise.data(), noise_u.data());
  const srt_light lights[6] = {{{1, 10, 10}, 50, {1, 1, 1}, 0},       {{-5, 15, 10}, 15, {1, 0.2f, 0.2f}, 0},
                               {{5, 15, 10}, 15, {0.2f, 1, 0.2f}, 0},  {{-5, 5, 10}, 15, {0.2f, 0.2f, 1}, 0},
                               {{5, 5, 10}, 15, {1, 1, 0.1f}, 0},      {{0, 21, 17}, 50, {1, 1, 1}, 0}};
  float o[3], f[3], u[3], r[3];
  srt_camera_reset(1, o, f, u, r);
  // frame: the second model moved, the main.cpp frame loop's uniforms
  float moved[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 12, -2, -5, 1};
  std::vector<float> frames[2];
  for (int pass = 0; pass < 2; ++pass) {
    srt_context* ctx = nullptr;
    if (srt_create(0, nullptr, &ctx) != SRT_OK) return fail("srt_create");
    if (pass == 0) {  // the reference's upload path, glBufferData -> srt_upload_scene
      TexAlbedo({a, b});
      ref::UploadModelDataToGPU(models, ctx);
    } else {          // the library's own producers
      const srt_model* ms[2] = {a, b};
      srt_scene* s = nullptr;
      if (srt_scene_build(ms, 2, &s) != SRT_OK || srt_upload_scene_obj(ctx, s) != SRT_OK) return fail("obj upload");
      srt_scene_free(s);
    }
    if (srt_update_model_matrix(ctx, 1, moved) != SRT_OK) return fail("UpdateModelMatrix");
    srt_set_int(ctx, "Width", W);
    srt_set_int(ctx, "Height", H);
    srt_set_uint(ctx, "bvh_count", 2);
    srt_set_int(ctx, "lightCount", 6);
    srt_set_bool(ctx, "showModel", 1);
    srt_set_vec3(ctx, "cameraOrigin", o[0], o[1], o[2]);
    srt_set_vec3(ctx, "cameraDirection", f[0], f[1], f[2]);
    srt_set_vec3(ctx, "cameraUp", u[0], u[1], u[2]);
    srt_set_vec3(ctx, "cameraRight", r[0], r[1], r[2]);
    srt_set_lights(ctx, lights, 6);
    srt_set_noise(ctx, noise.data(), noise_u.data(), (size_t)W * H);
    if (srt_alloc_images(ctx) != SRT_OK) return fail("alloc");
    srt_set_bool(ctx, "resetAccumBuffer", 1);
    srt_set_int(ctx, "accumFrames", 1);
    if (srt_dispatch(ctx, W / 8, H / 8) != SRT_OK) return fail("reset dispatch");
    srt_set_bool(ctx, "resetAccumBuffer", 0);
    for (int k = 2; k <= 4; ++k) {
      srt_set_int(ctx, "accumFrames", k);
      if (srt_dispatch(ctx, W / 8, H / 8) != SRT_OK) return fail("dispatch");
    }
    srt_finish(ctx);
    frames[pass].resize((size_t)W * H * 4);
    if (srt_read_accum(ctx, frames[pass].data(), frames[pass].size() * sizeof(float)) != SRT_OK) return fail("read");
    srt_destroy(ctx);
  }
  if (std::memcmp(frames[0].data(), frames[1].data(), frames[0].size() * sizeof(float)) != 0)
    return fail("the reference-path upload renders a different frame");
  if (!out_prefix.empty()) {
    FILE* fp = std::fopen((out_prefix + ".accum").c_str(), "wb");
    if (!fp || std::fwrite(frames[0].data(), sizeof(float), frames[0].size(), fp) != frames[0].size())
      return fail("write");
    std::fclose(fp);
  }
  srt_model_free(a);
  srt_model_free(b);
  std::printf("OK render\n");
  return 0;
}
