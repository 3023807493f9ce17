// camera.cpp -- the camera basis the kernel receives as uniforms.
//
// Restates Camera::UpdateCameraVectors and Camera::Reset
// (src/raytracer/camera.cpp:120-136, 187-212): yaw/pitch in degrees ->
// front = normalize(cos(y)cos(p), sin(p), sin(y)cos(p)); right =
// normalize(cross(front, +Y)); up = normalize(cross(right, front)).
// glm::normalize(v) = v * (1 / sqrt(dot(v, v))); glm::radians multiplies by the
// float constant pi/180; cos/sin are evaluated in double and rounded (the
// reference's unqualified cos(float) resolves to the double overload).
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

}  // namespace srt
