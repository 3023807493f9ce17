// srt_internal.hpp -- host-side types shared by the producers, the context and
// the C ABI.  Not part of the public interface (include/srt_amd.h is).
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "../../include/srt_amd.h"

namespace srt {

struct Vec3 {
  float x = 0.f, y = 0.f, z = 0.f;
  Vec3() = default;
  Vec3(float a, float b, float c) : x(a), y(b), z(c) {}
  float& operator[](int i) { return i == 0 ? x : (i == 1 ? y : z); }
  float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
};

// glm::min / glm::max component rules (glm: min(x,y) = y < x ? y : x).
inline Vec3 vmin(const Vec3& a, const Vec3& b) {
  return {b.x < a.x ? b.x : a.x, b.y < a.y ? b.y : a.y, b.z < a.z ? b.z : a.z};
}
inline Vec3 vmax(const Vec3& a, const Vec3& b) {
  return {a.x < b.x ? b.x : a.x, a.y < b.y ? b.y : a.y, a.z < b.z ? b.z : a.z};
}

// intersection_utils/bvh.h:23-30 (host node, before GPU packing)
struct BVHNode {
  Vec3 min_bounds;
  Vec3 max_bounds;
  uint32_t first_child = 0;
  uint32_t first_prim_index = 0;
  uint32_t prim_count = 0;
};

// asset_utils/types.h:25-28
struct Triangle {
  uint32_t vertex_idxs[3];
  uint32_t material_idx;
};

// A decoded map_Kd texture in stb_image layout (gpu_texture.h:29-33)
struct Texture {
  std::string path;
  int width = 0, height = 0, channels = 0;
  std::vector<uint8_t> texels;  // rows top first, `channels` bytes per texel
};

// asset_utils/types.h:31-37
struct Material {
  Vec3 diffuse;
  Vec3 specular;
  float specular_ex = 0.f;
  bool use_texture = false;
  std::string texture_path;
  int texture = -1;  // index into Model::textures
  Vec3 tex_albedo;   // texture(sampler2D(handle), (0,0)).xyz: the albedo while every uv is (0,0)
};

// asset_utils/types.h:39-52
struct Model {
  std::vector<BVHNode> nodes;
  std::vector<Triangle> prims;         // BVH-ordered
  std::vector<uint32_t> prim_input;    // prims[i] is the loader's triangle prim_input[i] (bvh.h:66-72)
  std::vector<Material> materials;
  std::vector<srt_vertex> vertices;    // PackedVertexData, 32 B
  std::vector<Texture> textures;       // one per distinct map_Kd file
  bool texcoords = false;              // loaded with SRT_LOAD_TEXCOORDS
  uint64_t faces_dropped = 0;
  uint32_t max_depth = 0;
  uint32_t leaves = 0;
};

// Flattened scene: the five SSBO arrays of gpu_loader.cpp:44-52.
struct Scene {
  std::vector<srt_bvh_record> bvhs;
  std::vector<srt_bvh_node> nodes;
  std::vector<srt_material_obj> mats;
  std::vector<float> tex_albedo;       // 3 per material
  std::vector<srt_triangle> tris;
  std::vector<uint32_t> tri_input;       // tris[i] in loader order: model offset + Model::prim_input
  std::vector<srt_vertex> verts;
  std::vector<Texture> textures;         // material handle = index
  bool sample_textures = false;          // some model carries real uvs
};

// producers (scene.cpp)
std::unique_ptr<Model> LoadObjectFile(const std::string& obj_path, bool texcoords, std::string* err);
std::unique_ptr<Model> ModelFromTriangles(const float* xyz9, uint32_t n, const Vec3& kd, const Vec3& ks,
                                          float ns);
void BuildBVH(Model* m);  // bvh.h:40-75 over m->prims with the loader's centre/bounds functions
std::unique_ptr<Scene> FlattenModels(const std::vector<const Model*>& models, std::string* err);
bool DecodePngTexture(const std::string& path, Texture* out, std::string* err);
// texture(sampler2D, vec2(s, t)).xyz under the sampling contract
void TextureSample(const uint8_t* texels, int width, int height, int channels, float s, float t, float rgb[3]);

// noise.cpp
void GlibcRand(uint32_t n, int32_t* out);
void GenerateNoise(uint32_t texels, bool gcc_order, float* noise, float* noise_u);

// camera.cpp
void CameraReset(bool show_model, Vec3* origin, Vec3* front, Vec3* up, Vec3* right);
void CameraBasis(float yaw, float pitch, Vec3* front, Vec3* up, Vec3* right);

enum class CameraMove { kForward = 0, kBackward, kLeft, kRight, kUp, kDown };

// RayTracer::Camera's interactive state (include/raytracer/camera.h:30-96).
struct CameraState {
  Vec3 position, front, up, right;
  float yaw = -90.0f, pitch = 0.0f;
  bool show_model = true;
  int32_t frame_counter = 0;  // MoveAndRotate's static counter (camera.cpp:175)

  void Construct(bool model);  // constructor + Initialize + Reset (src/main.cpp:439-441)
  void Reset();
  void UpdateVectors();
  void Move(CameraMove dir, float delta);
  void Rotate(float yaw_offset, float pitch_offset);
  // false (state unchanged) where the reference's yaw wrap would never end
  bool MoveAndRotate(float delta_time, const Vec3& move, float rot_x, float rot_y, float speed);
};

// One frame of src/main.cpp:622-659: reset decision, MoveAndRotate, accumFrames.
bool ProgressiveFrame(CameraState* cam, const Vec3& move, float rot_x, float rot_y, bool mouse_left,
                      bool* should_reset_buffer, float delta_time, int32_t* accum_frames, bool* reset_buffer);

void SetError(const std::string& msg);

// pathtrace.hip: the multi-GPU root's assembly on a given HIP stream (group.cpp's gather stream)
int AssembleBandsOn(srt_context* c, void* stream, const void* gathered, int nranks, int rows_pad, int band_rows,
                    int frames, void* accum_full, void* out_full);
int AssembleOutputOn(srt_context* c, void* stream, const void* gathered_rgba8, int nranks, int rows_pad,
                     int band_rows, int ext_w, int ext_h, void* out_full);
// pathtrace.hip: a context leaves a device group without allocating: rank 0 of 1, no images (a
// dispatch returns SRT_ERR_STATE until it is given images again)
int DetachImages(srt_context* c);

}  // namespace srt
