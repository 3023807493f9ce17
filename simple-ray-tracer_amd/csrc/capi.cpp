// capi.cpp -- C ABI of the host-side scene producers (include/srt_amd.h).
#include <cstring>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

#include "srt_internal.hpp"

struct srt_model {
  std::unique_ptr<srt::Model> m;
};
struct srt_scene {
  std::unique_ptr<srt::Scene> s;
};

extern "C" {

int srt_model_load(const char* obj_path, srt_model** out) { return srt_model_load_ex(obj_path, 0, out); }

int srt_model_load_ex(const char* obj_path, uint32_t flags, srt_model** out) {
  if (!obj_path || !out || (flags & ~SRT_LOAD_TEXCOORDS)) return SRT_ERR_INVALID;
  std::string err;
  auto m = srt::LoadObjectFile(obj_path, (flags & SRT_LOAD_TEXCOORDS) != 0, &err);
  if (!m) {
    srt::SetError(err);
    return SRT_ERR_IO;
  }
  *out = new srt_model{std::move(m)};
  return SRT_OK;
}

uint32_t srt_program_create(const char* path) {
  // create_compute_program.h:10-72: 0 with the log on stderr on failure
  if (!path) {
    std::cerr << "err opening(null)" << std::endl;
    srt::SetError("CreateComputeProgram: null path");
    return 0;
  }
  const std::string p(path);
  std::string name;
  if (p.rfind("builtin:", 0) == 0) {
    name = p.substr(8);
  } else {
    std::ifstream f(p);
    if (!f.is_open()) {  // LoadComputeShader, :13-16
      std::cerr << "err opening" << p << std::endl;
      srt::SetError("CreateComputeProgram: cannot open " + p);
      return 0;
    }
    const size_t slash = p.find_last_of('/');
    name = p.substr(slash == std::string::npos ? 0 : slash + 1);
    const size_t dot = name.rfind(".glsl");
    if (dot != std::string::npos && dot + 5 == name.size()) name.resize(dot);
  }
  if (name == "raytrace_compute") return SRT_PROGRAM_RAYTRACE;
  if (name == "ray_intersects") return SRT_PROGRAM_INTERSECT;
  std::cerr << "compile error:\nno MI355X kernel for compute program '" << name << "' (" << p << ")" << std::endl;
  srt::SetError("CreateComputeProgram: no kernel for " + p);
  return 0;
}

int srt_program_delete(uint32_t program) {
  return (program == SRT_PROGRAM_RAYTRACE || program == SRT_PROGRAM_INTERSECT) ? SRT_OK : SRT_ERR_INVALID;
}

int srt_model_from_triangles(const float* xyz9, uint32_t n_tris, const float kd[3], const float ks[3], float ns,
                             srt_model** out) {
  if (!out || (n_tris && !xyz9) || !kd || !ks) return SRT_ERR_INVALID;
  *out = new srt_model{srt::ModelFromTriangles(xyz9, n_tris, srt::Vec3(kd[0], kd[1], kd[2]),
                                               srt::Vec3(ks[0], ks[1], ks[2]), ns)};
  return SRT_OK;
}

int srt_model_free(srt_model* m) {
  delete m;
  return SRT_OK;
}

int srt_model_info(const srt_model* mm, uint64_t counts[8], float root_min[3], float root_max[3]) {
  if (!mm || !mm->m || !counts) return SRT_ERR_INVALID;
  const srt::Model& m = *mm->m;
  counts[0] = m.prims.size();
  counts[1] = m.vertices.size();
  counts[2] = m.nodes.size();
  counts[3] = m.leaves;
  counts[4] = m.max_depth;
  counts[5] = m.materials.size();
  counts[6] = m.faces_dropped;
  counts[7] = 0;
  if (!m.nodes.empty()) {
    if (root_min) {
      root_min[0] = m.nodes[0].min_bounds.x; root_min[1] = m.nodes[0].min_bounds.y; root_min[2] = m.nodes[0].min_bounds.z;
    }
    if (root_max) {
      root_max[0] = m.nodes[0].max_bounds.x; root_max[1] = m.nodes[0].max_bounds.y; root_max[2] = m.nodes[0].max_bounds.z;
    }
  }
  return SRT_OK;
}

int srt_model_sizes(const srt_model* mm, uint32_t sizes[4]) {
  if (!mm || !mm->m || !sizes) return SRT_ERR_INVALID;
  const srt::Model& m = *mm->m;
  sizes[0] = (uint32_t)m.nodes.size();
  sizes[1] = (uint32_t)m.prims.size();
  sizes[2] = (uint32_t)m.materials.size();
  sizes[3] = (uint32_t)m.vertices.size();
  return SRT_OK;
}

int srt_model_copy(const srt_model* mm, srt_host_bvh_node* nodes, srt_triangle* prims, srt_host_material* mats,
                   srt_vertex* verts) {
  if (!mm || !mm->m) return SRT_ERR_INVALID;
  const srt::Model& m = *mm->m;
  if (nodes)
    for (size_t i = 0; i < m.nodes.size(); ++i) {
      const srt::BVHNode& n = m.nodes[i];
      srt_host_bvh_node& o = nodes[i];
      for (int k = 0; k < 3; ++k) {
        o.min_bounds[k] = n.min_bounds[k];
        o.max_bounds[k] = n.max_bounds[k];
      }
      o.first_child = n.first_child;
      o.first_prim_index = n.first_prim_index;
      o.prim_count = n.prim_count;
    }
  if (prims)
    for (size_t i = 0; i < m.prims.size(); ++i)
      prims[i] = srt_triangle{m.prims[i].vertex_idxs[0], m.prims[i].vertex_idxs[1], m.prims[i].vertex_idxs[2],
                              m.prims[i].material_idx};
  if (mats)
    for (size_t i = 0; i < m.materials.size(); ++i) {
      const srt::Material& a = m.materials[i];
      srt_host_material& o = mats[i];
      for (int k = 0; k < 3; ++k) {
        o.diffuse[k] = a.diffuse[k];
        o.specular[k] = a.specular[k];
        o.tex_albedo[k] = a.tex_albedo[k];
      }
      o.specular_ex = a.specular_ex;
      o.use_texture = a.use_texture ? 1u : 0u;
    }
  if (verts) std::memcpy(verts, m.vertices.data(), m.vertices.size() * sizeof(srt_vertex));
  return SRT_OK;
}

int srt_model_prim_order(const srt_model* mm, uint32_t* input_index) {
  if (!mm || !mm->m || !input_index) return SRT_ERR_INVALID;
  const srt::Model& m = *mm->m;
  for (size_t i = 0; i < m.prims.size(); ++i)
    input_index[i] = i < m.prim_input.size() ? m.prim_input[i] : (uint32_t)i;
  return SRT_OK;
}

int srt_scene_build(const srt_model* const* models, uint32_t n_models, srt_scene** out) {
  if (!out || (n_models && !models)) return SRT_ERR_INVALID;
  std::vector<const srt::Model*> ms;
  for (uint32_t i = 0; i < n_models; ++i) ms.push_back(models[i] ? models[i]->m.get() : nullptr);
  std::string err;
  auto s = srt::FlattenModels(ms, &err);
  if (!s) {
    srt::SetError(err);
    return SRT_ERR_INVALID;
  }
  *out = new srt_scene{std::move(s)};
  return SRT_OK;
}

int srt_scene_free(srt_scene* s) {
  delete s;
  return SRT_OK;
}

int srt_scene_sizes(const srt_scene* s, uint32_t sizes[5]) {
  if (!s || !sizes) return SRT_ERR_INVALID;
  sizes[0] = (uint32_t)s->s->bvhs.size();
  sizes[1] = (uint32_t)s->s->nodes.size();
  sizes[2] = (uint32_t)s->s->mats.size();
  sizes[3] = (uint32_t)s->s->tris.size();
  sizes[4] = (uint32_t)s->s->verts.size();
  return SRT_OK;
}

int srt_scene_tri_order(const srt_scene* s, uint32_t* input_index) {
  if (!s || !input_index) return SRT_ERR_INVALID;
  std::memcpy(input_index, s->s->tri_input.data(), s->s->tri_input.size() * sizeof(uint32_t));
  return SRT_OK;
}

int srt_scene_copy(const srt_scene* s, srt_bvh_record* bvhs, srt_bvh_node* nodes, srt_material_obj* mats,
                   float* tex_albedo, srt_triangle* tris, srt_vertex* verts) {
  if (!s) return SRT_ERR_INVALID;
  const srt::Scene& sc = *s->s;
  if (bvhs) std::memcpy(bvhs, sc.bvhs.data(), sc.bvhs.size() * sizeof(srt_bvh_record));
  if (nodes) std::memcpy(nodes, sc.nodes.data(), sc.nodes.size() * sizeof(srt_bvh_node));
  if (mats) std::memcpy(mats, sc.mats.data(), sc.mats.size() * sizeof(srt_material_obj));
  if (tex_albedo) std::memcpy(tex_albedo, sc.tex_albedo.data(), sc.tex_albedo.size() * sizeof(float));
  if (tris) std::memcpy(tris, sc.tris.data(), sc.tris.size() * sizeof(srt_triangle));
  if (verts) std::memcpy(verts, sc.verts.data(), sc.verts.size() * sizeof(srt_vertex));
  return SRT_OK;
}

int srt_scene_texture_count(const srt_scene* s, uint32_t* n, int* sample_textures) {
  if (!s) return SRT_ERR_INVALID;
  if (n) *n = (uint32_t)s->s->textures.size();
  if (sample_textures) *sample_textures = s->s->sample_textures ? 1 : 0;
  return SRT_OK;
}

int srt_scene_texture(const srt_scene* s, uint32_t i, srt_texture* out) {
  if (!s || !out || i >= s->s->textures.size()) return SRT_ERR_INVALID;
  const srt::Texture& t = s->s->textures[i];
  *out = srt_texture{t.texels.data(), t.width, t.height, t.channels};
  return SRT_OK;
}

int srt_texture_sample(const srt_texture* tex, float s, float t, float rgb[3]) {
  if (!tex || !tex->texels || !rgb || tex->width <= 0 || tex->height <= 0 || tex->channels < 1 || tex->channels > 4)
    return SRT_ERR_INVALID;
  srt::TextureSample(tex->texels, tex->width, tex->height, tex->channels, s, t, rgb);
  return SRT_OK;
}

int srt_upload_scene_obj(srt_context* ctx, const srt_scene* s) {
  if (!ctx || !s) return SRT_ERR_INVALID;
  const srt::Scene& sc = *s->s;
  if (sc.sample_textures) {
    std::vector<srt_texture> tx;
    for (const auto& t : sc.textures) tx.push_back(srt_texture{t.texels.data(), t.width, t.height, t.channels});
    const int rc = srt_upload_textures(ctx, tx.data(), (uint32_t)tx.size());
    if (rc) return rc;
  }
  return srt_upload_scene(ctx, sc.bvhs.data(), (uint32_t)sc.bvhs.size(), sc.nodes.data(), (uint32_t)sc.nodes.size(),
                          sc.mats.data(), sc.sample_textures ? nullptr : sc.tex_albedo.data(),
                          (uint32_t)sc.mats.size(), sc.tris.data(), (uint32_t)sc.tris.size(), sc.verts.data(),
                          (uint32_t)sc.verts.size());
}

int srt_noise_generate(uint32_t texels, int gcc_order, float* noise_rgb, float* noise_uniform_rgb) {
  if (!noise_rgb || !noise_uniform_rgb) return SRT_ERR_INVALID;
  srt::GenerateNoise(texels, gcc_order != 0, noise_rgb, noise_uniform_rgb);
  return SRT_OK;
}

int srt_glibc_rand(uint32_t n, int32_t* out) {
  if (n && !out) return SRT_ERR_INVALID;
  srt::GlibcRand(n, out);
  return SRT_OK;
}

int srt_camera_reset(int show_model, float origin[3], float front[3], float up[3], float right[3]) {
  srt::Vec3 o, f, u, r;
  srt::CameraReset(show_model != 0, &o, &f, &u, &r);
  if (origin) { origin[0] = o.x; origin[1] = o.y; origin[2] = o.z; }
  if (front) { front[0] = f.x; front[1] = f.y; front[2] = f.z; }
  if (up) { up[0] = u.x; up[1] = u.y; up[2] = u.z; }
  if (right) { right[0] = r.x; right[1] = r.y; right[2] = r.z; }
  return SRT_OK;
}

int srt_camera_basis(float yaw_deg, float pitch_deg, float front[3], float up[3], float right[3]) {
  srt::Vec3 f, u, r;
  srt::CameraBasis(yaw_deg, pitch_deg, &f, &u, &r);
  if (front) { front[0] = f.x; front[1] = f.y; front[2] = f.z; }
  if (up) { up[0] = u.x; up[1] = u.y; up[2] = u.z; }
  if (right) { right[0] = r.x; right[1] = r.y; right[2] = r.z; }
  return SRT_OK;
}

namespace {
void ToState(const srt_camera* c, srt::CameraState* s) {
  s->position = srt::Vec3(c->position[0], c->position[1], c->position[2]);
  s->front = srt::Vec3(c->front[0], c->front[1], c->front[2]);
  s->up = srt::Vec3(c->up[0], c->up[1], c->up[2]);
  s->right = srt::Vec3(c->right[0], c->right[1], c->right[2]);
  s->yaw = c->yaw;
  s->pitch = c->pitch;
  s->show_model = c->show_model != 0;
  s->frame_counter = c->frame_counter;
}
void FromState(const srt::CameraState& s, srt_camera* c) {
  const srt::Vec3* v[4] = {&s.position, &s.front, &s.up, &s.right};
  float* d[4] = {c->position, c->front, c->up, c->right};
  for (int i = 0; i < 4; ++i) { d[i][0] = v[i]->x; d[i][1] = v[i]->y; d[i][2] = v[i]->z; }
  c->yaw = s.yaw;
  c->pitch = s.pitch;
  c->show_model = s.show_model ? 1 : 0;
  c->frame_counter = s.frame_counter;
}
}  // namespace

int srt_camera_init(srt_camera* cam, int show_model) {
  if (!cam) return SRT_ERR_INVALID;
  srt::CameraState s;
  s.Construct(show_model != 0);
  FromState(s, cam);
  return SRT_OK;
}

int srt_camera_state_reset(srt_camera* cam) {
  if (!cam) return SRT_ERR_INVALID;
  srt::CameraState s;
  ToState(cam, &s);
  s.Reset();
  FromState(s, cam);
  return SRT_OK;
}

int srt_camera_move(srt_camera* cam, int direction, float delta) {
  if (!cam || direction < SRT_MOVE_FORWARD || direction > SRT_MOVE_DOWN) return SRT_ERR_INVALID;
  srt::CameraState s;
  ToState(cam, &s);
  s.Move(static_cast<srt::CameraMove>(direction), delta);
  FromState(s, cam);
  return SRT_OK;
}

int srt_camera_rotate(srt_camera* cam, float yaw_offset, float pitch_offset) {
  if (!cam) return SRT_ERR_INVALID;
  srt::CameraState s;
  ToState(cam, &s);
  s.Rotate(yaw_offset, pitch_offset);
  FromState(s, cam);
  return SRT_OK;
}

int srt_camera_move_and_rotate(srt_camera* cam, float delta_time, const float movement_delta[3],
                               const float rotation_delta[2], float movement_speed) {
  if (!cam || !movement_delta || !rotation_delta) return SRT_ERR_INVALID;
  srt::CameraState s;
  ToState(cam, &s);
  const srt::Vec3 mv(movement_delta[0], movement_delta[1], movement_delta[2]);
  if (!s.MoveAndRotate(delta_time, mv, rotation_delta[0], rotation_delta[1], movement_speed)) {
    srt::SetError("srt_camera_move_and_rotate: yaw cannot be wrapped into [-180, 180]");
    return SRT_ERR_INVALID;
  }
  FromState(s, cam);
  return SRT_OK;
}

int srt_progressive_frame(srt_camera* cam, const float movement_delta[3], const float rotation_delta[2],
                          int mouse_left, int32_t* should_reset_buffer, float delta_time, int32_t* accum_frames,
                          int32_t* reset_buffer) {
  if (!cam || !movement_delta || !rotation_delta || !should_reset_buffer || !accum_frames || !reset_buffer)
    return SRT_ERR_INVALID;
  srt::CameraState s;
  ToState(cam, &s);
  const srt::Vec3 mv(movement_delta[0], movement_delta[1], movement_delta[2]);
  bool flag = *should_reset_buffer != 0, reset = false;
  int32_t frames = *accum_frames;
  if (!srt::ProgressiveFrame(&s, mv, rotation_delta[0], rotation_delta[1], mouse_left != 0, &flag, delta_time,
                             &frames, &reset)) {
    srt::SetError("srt_progressive_frame: yaw cannot be wrapped into [-180, 180]");
    return SRT_ERR_INVALID;
  }
  FromState(s, cam);
  *should_reset_buffer = flag ? 1 : 0;
  *accum_frames = frames;
  *reset_buffer = reset ? 1 : 0;
  return SRT_OK;
}

}  // extern "C"
