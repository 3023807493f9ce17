// srt/srt.hpp -- C++ host API of the MI355X path tracer, shaped like the reference's.
//
// Header-only layer over the C ABI (include/srt_amd.h) that keeps the names,
// argument meaning and call pattern of matteobir12/simple-ray-tracer's host code
// for this path, so src/main.cpp's per-frame loop ports line for line:
//   Graphics::Compute            include/graphics/shader.h:46-55, src/graphics/Shader.cpp
//   AssetUtils::LoadObject       src/asset_utils/model_loader.cpp:20-32
//   AssetUtils::UploadModelDataToGPU / UpdateModelMatrix / UpdateRays
//                                src/asset_utils/gpu_loader.cpp:63-210
//   RayTracer::Camera / PointLight   src/raytracer/camera.cpp, include/raytracer/light.h
//   Graphics::ComputeGroup       (new) the same loop's frame tiled over several GPUs (srt_group_*)
// GL's "currently bound program" is mirrored by Compute::Use(): the upload
// functions act on the last used Compute, as they act on the bound GL state.
// Errors: std::runtime_error (the reference std::terminate()s in Init and
// throws std::runtime_error("Model was null!") in the upload).
#pragma once

#include <array>
#include <cstdint>
#include <cstdio>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../srt_amd.h"

namespace srt {

struct vec3 {
  float x = 0.f, y = 0.f, z = 0.f;
};
struct vec2 {
  float x = 0.f, y = 0.f;
};

inline void check(int code, const char* what) {
  if (code != SRT_OK) throw std::runtime_error(std::string(what) + ": " + srt_last_error());
}

namespace Graphics {

class Compute;
namespace detail {
inline Compute*& current() {
  static thread_local Compute* c = nullptr;
  return c;
}
}  // namespace detail

// Graphics::Compute(path): the program is resolved as
// Compute::CreateComputeProgram resolves it (srt_program_create: the file must
// open; raytrace_compute.glsl is the path tracer, ray_intersects.glsl the
// closest-hit test kernel); the kernels are HIP code objects for gfx950.
// Init() throws where the reference std::terminate()s (Shader.cpp:125-157).
class Compute {
 public:
  explicit Compute(const char* path, int device = 0, void* hip_stream = nullptr)
      : path_(path ? path : ""), device_(device), stream_(hip_stream) {}
  ~Compute() {
    if (detail::current() == this) detail::current() = nullptr;
    if (ctx_) srt_destroy(ctx_);
  }
  Compute(const Compute&) = delete;
  Compute& operator=(const Compute&) = delete;

  void Init() {
    if (!program_) {
      program_ = srt_program_create(path_.c_str());
      if (!program_) throw std::runtime_error("Compute::Init: no compute program for " + path_);
    }
    if (!ctx_) check(srt_create(device_, stream_, &ctx_), "Compute::Init");
  }
  uint32_t program() {
    Init();
    return program_;
  }
  void Use() {
    Init();
    detail::current() = this;
  }
  srt_context* context() {
    Init();
    return ctx_;
  }

  void SetBool(const std::string& name, bool v) {
    const int rc = srt_set_bool(context(), name.c_str(), v ? 1 : 0);
    if (rc == SRT_ERR_NOT_FOUND) {
      if (name != "resetAccumBuffer")  // Shader.cpp:170-176
        std::fprintf(stderr, "Warning: Uniform '%s' not found in compute shader\n", name.c_str());
      return;
    }
    check(rc, "SetBool");
  }
  void SetInt(const std::string& name, int v) {  // unknown names are silently ignored (Shader.cpp:190-205)
    const int rc = srt_set_int(context(), name.c_str(), v);
    if (rc != SRT_ERR_NOT_FOUND) check(rc, "SetInt");
    // images 0/3 follow Width x Height: re-allocated (cleared) only when the size changes, as a
    // GL texture keeps its contents across frames (src/main.cpp sets both every frame)
    if (rc == SRT_OK && name == "Width" && v != img_w_) img_w_ = v, images_dirty_ = true;
    if (rc == SRT_OK && name == "Height" && v != img_h_) img_h_ = v, images_dirty_ = true;
  }
  void SetUInt(const std::string& name, uint32_t v) {
    const int rc = srt_set_uint(context(), name.c_str(), v);
    if (rc != SRT_ERR_NOT_FOUND) check(rc, "SetUInt");
  }
  void SetFloat(const std::string& name, float v) {
    const int rc = srt_set_float(context(), name.c_str(), v);
    if (rc != SRT_ERR_NOT_FOUND) check(rc, "SetFloat");
  }
  void SetVec3(const std::string& name, const vec3& v) {
    const int rc = srt_set_vec3(context(), name.c_str(), v.x, v.y, v.z);
    if (rc != SRT_ERR_NOT_FOUND) check(rc, "SetVec3");
  }

  // texel buffers at units 1, 2 (src/main.cpp:269-301) and the light SSBO (binding 4)
  void BindNoise(const std::vector<float>& noise_rgb, const std::vector<float>& noise_uniform_rgb) {
    if (noise_rgb.size() != noise_uniform_rgb.size() || noise_rgb.size() % 3) throw std::runtime_error("BindNoise");
    check(srt_set_noise(context(), noise_rgb.data(), noise_uniform_rgb.data(), noise_rgb.size() / 3), "BindNoise");
  }
  void BindLights(const std::vector<srt_light>& lights) {
    check(srt_set_lights(context(), lights.data(), (uint32_t)lights.size()), "BindLights");
  }

  // glDispatchCompute(gx, gy, 1) (src/main.cpp:706); images 0/3 follow Width x Height
  void Dispatch(uint32_t gx, uint32_t gy, uint32_t gz = 1) {
    if (gz != 1) throw std::runtime_error("Dispatch: groups_z must be 1");
    if (program() != SRT_PROGRAM_RAYTRACE) throw std::runtime_error("Dispatch: " + path_ + " is not raytrace_compute");
    if (images_dirty_) {
      check(srt_alloc_images(context()), "alloc images");
      images_dirty_ = false;
    }
    check(srt_dispatch(context(), gx, gy), "Dispatch");
  }
  // glMemoryBarrier + glFinish (src/main.cpp:709-718)
  void Finish() { check(srt_finish(context()), "Finish"); }
  // Device time of the last render's sample launches, and the summed time of every sample launch since
  // the previous KernelTime call (each launch's span on the GPU clock; srt_amd.h)
  float LastKernelMs() {
    float ms = 0.0f;
    check(srt_last_kernel_ms(context(), &ms), "LastKernelMs");
    return ms;
  }
  double KernelTime(int* launches = nullptr) {
    double ms = 0.0;
    int n = 0;
    check(srt_kernel_time(context(), &ms, &n), "KernelTime");
    if (launches) *launches = n;
    return ms;
  }

  // `n` progressive frames in one launch (same accumulation as n Dispatch calls)
  void RenderFrames(int frame_first, int n, bool write_output = true) {
    if (images_dirty_) {
      check(srt_alloc_images(context()), "alloc images");
      images_dirty_ = false;
    }
    check(srt_render_frames(context(), frame_first, n, write_output ? 1 : 0, 0), "RenderFrames");
  }
  std::vector<float> ReadAccum() {
    std::vector<float> v((size_t)srt_local_rows(context()) * width() * 4);
    check(srt_read_accum(context(), v.data(), v.size() * sizeof(float)), "ReadAccum");
    return v;
  }
  std::vector<uint8_t> ReadOutput() {
    std::vector<uint8_t> v((size_t)srt_local_rows(context()) * width() * 4);
    check(srt_read_output(context(), v.data(), v.size()), "ReadOutput");
    return v;
  }
  // output stage: image0 to a PNG / PPM file, top row first (as the window shows it)
  void SaveImage(const std::string& path, bool flip_y = true) {
    check(srt_write_output(context(), path.c_str(), flip_y ? 1 : 0), "SaveImage");
  }
  void SetWidthHint(int w) { width_ = w; }
  int width() const { return width_; }

 private:
  std::string path_;
  int device_;
  void* stream_;
  srt_context* ctx_ = nullptr;
  uint32_t program_ = 0;
  bool images_dirty_ = true;
  int img_w_ = -1, img_h_ = -1;
  int width_ = 0;
};

// The frame of main.cpp's loop tiled over several GPUs of this process (srt_group_*): one
// Compute per device; uniforms and bindings go to every device; Dispatch / RenderFrames render each
// device's row bands and their sRGB8, gather those (4 B/px) to the first device over RCCL and assemble
// the full image0 there; the radiance is gathered only by ReadAccum.
//   Graphics::ComputeGroup rt("./shaders/raytrace_compute.glsl", {0, 1, 2, 3, 4, 5, 6, 7});
//   rt.ForEach([&](Graphics::Compute& c) { c.Use(); AssetUtils::UploadModelDataToGPU({model.get()}, 5); });
//   ... rt.SetInt("accumFrames", accumFrames); rt.Dispatch(W / 8, H / 8); rt.Finish(); ...
class ComputeGroup {
 public:
  ComputeGroup(const char* path, const std::vector<int>& devices, int band_rows = 8) : band_rows_(band_rows) {
    if (devices.empty()) throw std::runtime_error("ComputeGroup: no devices");
    for (int d : devices) parts_.push_back(std::make_unique<Compute>(path, d));
  }
  ~ComputeGroup() {
    if (g_) srt_group_destroy(g_);
  }
  ComputeGroup(const ComputeGroup&) = delete;
  ComputeGroup& operator=(const ComputeGroup&) = delete;

  size_t size() const { return parts_.size(); }
  Compute& operator[](size_t i) { return *parts_[i]; }
  template <class F>
  void ForEach(F f) {
    for (auto& c : parts_) f(*c);
  }
  srt_group* group() {
    if (!g_) {
      std::vector<srt_context*> ctxs;
      for (auto& c : parts_) ctxs.push_back(c->context());
      check(srt_group_create(ctxs.data(), (int)ctxs.size(), band_rows_, &g_), "ComputeGroup");
    }
    return g_;
  }
  const char* Transport() { return srt_group_transport(group()); }
  // ranks RCCL sees (or the contexts, under the copy transport), and each device's kernel time
  int Ranks() {
    int v = 0;
    check(srt_group_get_int(group(), "ranks", &v), "ComputeGroup::Ranks");
    return v;
  }
  std::vector<float> KernelMs() {
    std::vector<float> v(parts_.size());
    check(srt_group_last_kernel_ms(group(), v.data(), (int)v.size()), "ComputeGroup::KernelMs");
    return v;
  }
  // per device since the last call: sample-kernel throughput ms (back-to-back frames read once), and the
  // ms of its part of the per-frame sRGB8 exchange (device 0's includes the assembly)
  std::vector<double> KernelTime() {
    std::vector<double> v(parts_.size());
    std::vector<int> n(parts_.size());
    check(srt_group_kernel_time(group(), v.data(), n.data(), (int)v.size()), "ComputeGroup::KernelTime");
    return v;
  }
  std::vector<double> ExchangeTime() {
    std::vector<double> v(parts_.size());
    std::vector<int> n(parts_.size());
    check(srt_group_exchange_time(group(), v.data(), n.data(), (int)v.size()), "ComputeGroup::ExchangeTime");
    return v;
  }

  void SetBool(const std::string& n, bool v) { ForEach([&](Compute& c) { c.SetBool(n, v); }); }
  void SetInt(const std::string& n, int v) {
    ForEach([&](Compute& c) { c.SetInt(n, v); });
    if (n == "Width" && v != w_) w_ = v, images_dirty_ = true;
    if (n == "Height" && v != h_) h_ = v, images_dirty_ = true;
  }
  void SetUInt(const std::string& n, uint32_t v) { ForEach([&](Compute& c) { c.SetUInt(n, v); }); }
  void SetVec3(const std::string& n, const vec3& v) { ForEach([&](Compute& c) { c.SetVec3(n, v); }); }
  void BindNoise(const std::vector<float>& a, const std::vector<float>& b) {
    ForEach([&](Compute& c) { c.BindNoise(a, b); });
  }
  void BindLights(const std::vector<srt_light>& l) { ForEach([&](Compute& c) { c.BindLights(l); }); }

  // glDispatchCompute on every device, the gather and the full frame (src/main.cpp:706)
  void Dispatch(uint32_t gx, uint32_t gy, uint32_t gz = 1) {
    if (gz != 1) throw std::runtime_error("Dispatch: groups_z must be 1");
    Images();
    check(srt_group_dispatch(group(), gx, gy), "ComputeGroup::Dispatch");
  }
  void RenderFrames(int frame_first, int n) {
    Images();
    check(srt_group_render_frames(group(), frame_first, n), "ComputeGroup::RenderFrames");
  }
  void Finish() { check(srt_group_finish(group()), "ComputeGroup::Finish"); }
  std::vector<float> ReadAccum() {
    std::vector<float> v((size_t)w_ * h_ * 4);
    check(srt_group_read_accum(group(), v.data(), v.size() * sizeof(float)), "ComputeGroup::ReadAccum");
    return v;
  }
  std::vector<uint8_t> ReadOutput() {
    std::vector<uint8_t> v((size_t)w_ * h_ * 4);
    check(srt_group_read_output(group(), v.data(), v.size()), "ComputeGroup::ReadOutput");
    return v;
  }
  void SaveImage(const std::string& path, bool flip_y = true) {
    const auto img = ReadOutput();
    check(srt_image_write(path.c_str(), img.data(), w_, h_, flip_y ? 1 : 0), "ComputeGroup::SaveImage");
  }

 private:
  void Images() {
    if (images_dirty_) {
      check(srt_group_alloc_images(group()), "ComputeGroup: images");
      images_dirty_ = false;
    }
  }
  std::vector<std::unique_ptr<Compute>> parts_;
  srt_group* g_ = nullptr;
  int band_rows_;
  int w_ = 0, h_ = 0;
  bool images_dirty_ = true;
};

}  // namespace Graphics

namespace AssetUtils {

// AssetUtils::Model (asset_utils/types.h:39-52), owned on the host.
class Model {
 public:
  explicit Model(srt_model* m) : m_(m) {}
  ~Model() { srt_model_free(m_); }
  Model(const Model&) = delete;
  Model& operator=(const Model&) = delete;
  srt_model* handle() const { return m_; }
  // The BVH's primitive permutation (bvh.h:66-72): model_bvh.GetPrims()[i] is the loader's all_triangles[
  // PrimOrder()[i]] (model_loader.cpp:299-331).  A closest hit (UpdateRaysAndTrace) is a GetPrims() index, as
  // the shader's Intersects returns it; PrimOrder() maps it to the loader's order, in which
  // BVH_intergration_tests.cpp:94 states its expected triangle.
  std::vector<uint32_t> PrimOrder() const {
    uint32_t sizes[4];
    check(srt_model_sizes(m_, sizes), "Model::PrimOrder");
    std::vector<uint32_t> order(sizes[1]);
    check(srt_model_prim_order(m_, order.data()), "Model::PrimOrder");
    return order;
  }

 private:
  srt_model* m_;
};

// model_loader.cpp:20-32: objects/<name>/<name>.obj.  texcoords = true is the
// loader with has_texcoords set (vertex uvs from `vt`; the reference leaves
// them at (0,0)), and its textures are then sampled per hit.
inline std::unique_ptr<Model> LoadObject(const std::string& name, const std::string& objects_dir = "./objects/",
                                         bool texcoords = false) {
  srt_model* m = nullptr;
  check(srt_model_load_ex((objects_dir + name + "/" + name + ".obj").c_str(), texcoords ? SRT_LOAD_TEXCOORDS : 0u,
                          &m),
        "LoadObject");
  return std::make_unique<Model>(m);
}

// gpu_loader.cpp:63-183, into the last used Compute (the bound program).
inline void UploadModelDataToGPU(const std::vector<Model*>& models, const uint32_t binding_offset = 0) {
  (void)binding_offset;  // bindings are fixed by the C ABI
  Graphics::Compute* c = Graphics::detail::current();
  if (!c) throw std::runtime_error("UploadModelDataToGPU: no Compute in use");
  std::vector<const srt_model*> hs;
  for (Model* m : models) {
    if (!m) throw std::runtime_error("Model was null!");
    hs.push_back(m->handle());
  }
  srt_scene* s = nullptr;
  check(srt_scene_build(hs.data(), (uint32_t)hs.size(), &s), "UploadModelDataToGPU");
  const int rc = srt_upload_scene_obj(c->context(), s);
  srt_scene_free(s);
  check(rc, "UploadModelDataToGPU");
}

// gpu_loader.cpp:185-196 (glm::mat4 column-major, m[c * 4 + r])
inline void UpdateModelMatrix(const uint32_t index, const std::array<float, 16>& matrix) {
  Graphics::Compute* c = Graphics::detail::current();
  if (!c) throw std::runtime_error("UpdateModelMatrix: no Compute in use");
  check(srt_update_model_matrix(c->context(), index, matrix.data()), "UpdateModelMatrix");
}

// gpu_loader.cpp:198-210 + the ray_intersects.glsl test kernel: closest hit per ray
inline std::vector<uint32_t> UpdateRaysAndTrace(const std::vector<srt_ray>& rays, std::vector<float>* t_out = nullptr) {
  Graphics::Compute* c = Graphics::detail::current();
  if (!c) throw std::runtime_error("UpdateRays: no Compute in use");
  if (c->program() != SRT_PROGRAM_INTERSECT) throw std::runtime_error("UpdateRays: the program in use is not ray_intersects");
  std::vector<uint32_t> hits(rays.size());
  std::vector<float> t(rays.size());
  check(srt_trace_closest(c->context(), rays.data(), (uint32_t)rays.size(), hits.data(), t.data()), "UpdateRays");
  if (t_out) *t_out = std::move(t);
  return hits;
}

}  // namespace AssetUtils

namespace RayTracer {

// raytracer/light.h:54-63
inline srt_light PointLight(const vec3& position, const vec3& color, float intensity) {
  srt_light l{};
  l.position[0] = position.x; l.position[1] = position.y; l.position[2] = position.z;
  l.color[0] = color.x; l.color[1] = color.y; l.color[2] = color.z;
  l.intensity = intensity;
  return l;
}

// RayTracer::Camera (src/raytracer/camera.cpp, include/raytracer/camera.h) over srt_camera:
// the basis vectors src/main.cpp:672-675 uploads, Move*, Rotate, MoveAndRotate, Reset.
class Camera {
 public:
  explicit Camera(bool show_model) { check(srt_camera_init(&s_, show_model ? 1 : 0), "Camera"); }
  void Reset() { check(srt_camera_state_reset(&s_), "Camera::Reset"); }
  void Rotate(float yaw_offset, float pitch_offset) {
    check(srt_camera_rotate(&s_, yaw_offset, pitch_offset), "Camera::Rotate");
  }
  void MoveForward(float d) { check(srt_camera_move(&s_, SRT_MOVE_FORWARD, d), "Camera::MoveForward"); }
  void MoveBackward(float d) { check(srt_camera_move(&s_, SRT_MOVE_BACKWARD, d), "Camera::MoveBackward"); }
  void MoveLeft(float d) { check(srt_camera_move(&s_, SRT_MOVE_LEFT, d), "Camera::MoveLeft"); }
  void MoveRight(float d) { check(srt_camera_move(&s_, SRT_MOVE_RIGHT, d), "Camera::MoveRight"); }
  void MoveUp(float d) { check(srt_camera_move(&s_, SRT_MOVE_UP, d), "Camera::MoveUp"); }
  void MoveDown(float d) { check(srt_camera_move(&s_, SRT_MOVE_DOWN, d), "Camera::MoveDown"); }
  void MoveAndRotate(float delta_time, const vec3& movement_delta, const vec2& rotation_delta, float speed) {
    const float m[3] = {movement_delta.x, movement_delta.y, movement_delta.z};
    const float r[2] = {rotation_delta.x, rotation_delta.y};
    check(srt_camera_move_and_rotate(&s_, delta_time, m, r, speed), "Camera::MoveAndRotate");
  }
  vec3 getOrigin() const { return {s_.position[0], s_.position[1], s_.position[2]}; }
  vec3 getForward() const { return {s_.front[0], s_.front[1], s_.front[2]}; }
  vec3 getUpVector() const { return {s_.up[0], s_.up[1], s_.up[2]}; }
  vec3 getRightVector() const { return {s_.right[0], s_.right[1], s_.right[2]}; }
  srt_camera* state() { return &s_; }

 private:
  srt_camera s_{};
};

}  // namespace RayTracer

namespace Common {
// UpdateNoiseTex's buffers (src/main.cpp:269-301): W*H unit vectors, then W*H uniform vec3s
inline void GenerateNoise(uint32_t width, uint32_t height, std::vector<float>* noise, std::vector<float>* noise_uniform,
                          bool gcc_order = true) {
  const size_t n = (size_t)width * height;
  noise->resize(3 * n);
  noise_uniform->resize(3 * n);
  check(srt_noise_generate((uint32_t)n, gcc_order ? 1 : 0, noise->data(), noise_uniform->data()), "GenerateNoise");
}
}  // namespace Common

}  // namespace srt
