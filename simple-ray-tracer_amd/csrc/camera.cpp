// camera.cpp -- the camera the kernel receives as uniforms, and the interactive
// mode's host side.
//
// Restates RayTracer::Camera (src/raytracer/camera.cpp, include/raytracer/camera.h):
//   * UpdateCameraVectors (:120-136): yaw/pitch in degrees ->
//     front = normalize(cos(y)cos(p), sin(p), sin(y)cos(p)); right =
//     normalize(cross(front, +Y)); up = normalize(cross(right, front)).
//   * Reset (:187-212), the constructor (camera.h:34-37), Move* (:71-105),
//     Rotate (:107-118) and MoveAndRotate (:138-185) with its yaw wrap and the
//     every-120th-call re-orthonormalisation.
// and the frame loop's accumulation-reset schedule (src/main.cpp:622-659).
// glm::normalize(v) = v * (1 / sqrt(dot(v, v))); dot is ((x*x + y*y) + z*z);
// glm::radians multiplies by the float constant pi/180; cos/sin are evaluated in
// double and rounded (the reference's unqualified cos(float) resolves to the
// double overload).  The library is built with -ffp-contract=off, as the
// reference's x86-64 gcc build has no FMA.
#include <cmath>

#include "srt_internal.hpp"

namespace srt {

namespace {

inline float Dot(const Vec3& a, const Vec3& b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline Vec3 Normalize(const Vec3& v) {
  const float inv = 1.0f / std::sqrt(Dot(v, v));
  return Vec3(v.x * inv, v.y * inv, v.z * inv);
}
// glm::cross: (x.y*y.z - y.y*x.z, x.z*y.x - y.z*x.x, x.x*y.y - y.x*x.y)
inline Vec3 Cross(const Vec3& x, const Vec3& y) {
  return Vec3(x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y);
}
inline float Radians(float deg) { return deg * static_cast<float>(0.01745329251994329576923690768489); }
// glm::clamp(x, lo, hi) = min(max(x, lo), hi) with glm's scalar min/max rules
inline float Clamp(float x, float lo, float hi) {
  const float m = (x < lo) ? lo : x;
  return (hi < m) ? hi : m;
}
// position += a * s * k  (glm: vec3 * float, then * float, then +=)
inline void AddScaled(Vec3* p, const Vec3& a, float s, float k) {
  p->x = p->x + (a.x * s) * k;
  p->y = p->y + (a.y * s) * k;
  p->z = p->z + (a.z * s) * k;
}

}  // namespace

void CameraBasis(float yaw, float pitch, Vec3* front, Vec3* up, Vec3* right) {
  Vec3 nf;
  const double cy = std::cos(static_cast<double>(Radians(yaw)));
  const double cp = std::cos(static_cast<double>(Radians(pitch)));
  const double sy = std::sin(static_cast<double>(Radians(yaw)));
  const double sp = std::sin(static_cast<double>(Radians(pitch)));
  nf.x = static_cast<float>(cy * cp);
  nf.y = static_cast<float>(sp);
  nf.z = static_cast<float>(sy * cp);
  *front = Normalize(nf);
  const Vec3 world_up(0.0f, 1.0f, 0.0f);
  *right = Normalize(Cross(*front, world_up));
  *up = Normalize(Cross(*right, *front));
}

void CameraReset(bool show_model, Vec3* origin, Vec3* front, Vec3* up, Vec3* right) {
  *origin = show_model ? Vec3(0.0f, 9.0f, 40.0f) : Vec3(0.0f, 1.0f, 4.0f);
  CameraBasis(-90.0f, 0.0f, front, up, right);
}

void CameraState::UpdateVectors() { CameraBasis(yaw, pitch, &front, &up, &right); }

void CameraState::Construct(bool model) {
  // camera.h:34-37 with a default CameraSettings (origin 0, lookAt (0,0,-1), vUp +Y)
  const Vec3 origin(0.0f, 0.0f, 0.0f), look_at(0.0f, 0.0f, -1.0f), v_up(0.0f, 1.0f, 0.0f);
  position = origin;
  front = Normalize(Vec3(look_at.x - origin.x, look_at.y - origin.y, look_at.z - origin.z));
  up = v_up;
  right = Normalize(Cross(front, up));
  yaw = -90.0f;
  pitch = 0.0f;
  show_model = model;
  frame_counter = 0;
  UpdateVectors();  // Camera::Initialize (camera.cpp:8-18)
  Reset();          // src/main.cpp:441
}

void CameraState::Reset() {
  position = show_model ? Vec3(0.0f, 9.0f, 40.0f) : Vec3(0.0f, 1.0f, 4.0f);
  yaw = -90.0f;
  pitch = 0.0f;
  front = Vec3(0.0f, 0.0f, -1.0f);
  right = Vec3(1.0f, 0.0f, 0.0f);
  up = Vec3(0.0f, 1.0f, 0.0f);
  UpdateVectors();
  UpdateVectors();  // Initialize(showModel) calls it again; idempotent
}

void CameraState::Move(CameraMove dir, float delta) {
  switch (dir) {
    case CameraMove::kForward: AddScaled(&position, front, delta, 1.0f); break;
    case CameraMove::kBackward:
      position = Vec3(position.x - front.x * delta, position.y - front.y * delta, position.z - front.z * delta);
      break;
    case CameraMove::kLeft:
      position = Vec3(position.x - right.x * delta, position.y - right.y * delta, position.z - right.z * delta);
      break;
    case CameraMove::kRight: AddScaled(&position, right, delta, 1.0f); break;
    case CameraMove::kUp: AddScaled(&position, up, delta, 1.0f); break;
    case CameraMove::kDown:
      position = Vec3(position.x - up.x * delta, position.y - up.y * delta, position.z - up.z * delta);
      break;
  }
  UpdateVectors();
}

void CameraState::Rotate(float yaw_offset, float pitch_offset) {
  yaw += yaw_offset;
  pitch += pitch_offset;
  if (pitch > 89.0f) pitch = 89.0f;
  if (pitch < -89.0f) pitch = -89.0f;
  UpdateVectors();
}

bool CameraState::MoveAndRotate(float delta_time, const Vec3& move, float rot_x, float rot_y, float speed) {
  if (std::fabs(rot_x) > 0.0001f || std::fabs(rot_y) > 0.0001f) {
    float y = yaw + rot_x;
    // The reference's `while (yaw > 180) yaw -= 360` never ends for a non-finite
    // yaw, or one so large that subtracting 360 leaves it unchanged: refuse those.
    while (y > 180.0f) {
      const float n = y - 360.0f;
      if (n == y) return false;
      y = n;
    }
    while (y < -180.0f) {
      const float n = y + 360.0f;
      if (n == y) return false;
      y = n;
    }
    yaw = y;
    pitch = Clamp(pitch + rot_y, -89.0f, 89.0f);
    UpdateVectors();
  }
  if (std::sqrt(Dot(move, move)) > 0.0001f) {
    const float adjusted = speed * delta_time;
    AddScaled(&position, front, move.z, adjusted);
    AddScaled(&position, right, move.x, adjusted);
    AddScaled(&position, up, move.y, adjusted);
  }
  // the reference's function-static counter (camera.cpp:175): one per camera here
  if (++frame_counter % 120 == 0) {
    front = Normalize(front);
    const Vec3 world_up(0.0f, 1.0f, 0.0f);
    right = Normalize(Cross(front, world_up));
    up = Normalize(Cross(right, front));
  }
  return true;
}

bool ProgressiveFrame(CameraState* cam, const Vec3& move, float rot_x, float rot_y, bool mouse_left,
                      bool* should_reset_buffer, float delta_time, int32_t* accum_frames, bool* reset_buffer) {
  // src/main.cpp:622-659
  bool reset = false;
  const bool any_input = std::sqrt(Dot(move, move)) > 0.0001f ||
                         std::sqrt(rot_x * rot_x + rot_y * rot_y) > 0.0001f || mouse_left;
  if (any_input) {
    reset = true;
    *accum_frames = 0;
  }
  if (*should_reset_buffer) {  // InputHandler::ShouldResetBuffer / ClearResetFlag (input_handler.cpp:160-168)
    reset = true;
    *accum_frames = 0;
    *should_reset_buffer = false;
  }
  const float movement_speed = 1.0f;
  if (!cam->MoveAndRotate(delta_time, move, rot_x, rot_y, movement_speed)) return false;
  *accum_frames += 1;  // RUN_COMPUTE_RT (main.cpp:657-659)
  *reset_buffer = reset;
  return true;
}

}  // namespace srt
