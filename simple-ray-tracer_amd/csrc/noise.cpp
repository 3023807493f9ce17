// noise.cpp -- the two noise texel buffers of UpdateNoiseTex (src/main.cpp:269-301).
//
// The reference fills them from glibc rand(), never seeded (no srand anywhere,
// so seed 1), through Common::randomUnitVector / randomVec3
// (include/common/utils.h:22-51).  glibc's rand() is random_r's TYPE_3
// additive feedback generator; it is restated here so the stream is the same
// on any host:  r[0] = 1; r[i] = 16807 * r[i-1] mod (2^31 - 1) for i < 31
// (Schrage); r[i] = r[i-31] for 31 <= i < 34; r[i] = r[i-31] + r[i-3] (mod 2^32)
// afterwards; output k is r[k + 344] >> 1.
#include <cmath>
#include <cstring>
#include <vector>

#include "srt_internal.hpp"

namespace srt {

namespace {

class GlibcRandom {
 public:
  GlibcRandom() {
    int32_t r[34];
    r[0] = 1;
    for (int i = 1; i < 31; ++i) {
      const int32_t hi = r[i - 1] / 127773;
      const int32_t lo = r[i - 1] % 127773;
      int32_t word = 16807 * lo - 2836 * hi;
      if (word < 0) word += 2147483647;
      r[i] = word;
    }
    for (int i = 31; i < 34; ++i) r[i] = r[i - 31];
    for (int i = 0; i < 34; ++i) ring_[i] = static_cast<uint32_t>(r[i]);
    pos_ = 34;
    for (int i = 34; i < 344; ++i) Step();
  }
  int32_t Next() { return static_cast<int32_t>(Step() >> 1); }

 private:
  uint32_t Step() {
    // ring of the last 34 values: r[i] = r[i-31] + r[i-3]
    const uint32_t v = ring_[(pos_ - 31) % 34] + ring_[(pos_ - 3) % 34];
    ring_[pos_ % 34] = v;
    ++pos_;
    return v;
  }
  uint32_t ring_[34];
  uint64_t pos_;
};

// utils.h:22-24: std::rand() / (RAND_MAX + 1.0f); RAND_MAX + 1.0f == 2^31
inline float RandomFloat(GlibcRandom& g) { return static_cast<float>(g.Next()) / 2147483648.0f; }
// utils.h:26-28
inline float RandomFloat(GlibcRandom& g, float mn, float mx) { return mn + (mx - mn) * RandomFloat(g); }
// utils.h:30-32: glm::vec3(a(), b(), c()); g++ evaluates the arguments right to left
inline Vec3 RandomVec3(GlibcRandom& g, float mn, float mx, bool gcc_order) {
  Vec3 v;
  if (gcc_order) {
    v.z = RandomFloat(g, mn, mx);
    v.y = RandomFloat(g, mn, mx);
    v.x = RandomFloat(g, mn, mx);
  } else {
    v.x = RandomFloat(g, mn, mx);
    v.y = RandomFloat(g, mn, mx);
    v.z = RandomFloat(g, mn, mx);
  }
  return v;
}

}  // namespace

void GlibcRand(uint32_t n, int32_t* out) {
  GlibcRandom g;
  for (uint32_t i = 0; i < n; ++i) out[i] = g.Next();
}

void GenerateNoise(uint32_t texels, bool gcc_order, float* noise, float* noise_u) {
  GlibcRandom g;
  // utils.h:43-51 randomUnitVector: rejection from the cube, 1e-160 < |p|^2 <= 1
  for (uint32_t i = 0; i < texels; ++i) {
    for (;;) {
      const Vec3 p = RandomVec3(g, -1.0f, 1.0f, gcc_order);
      const float lensq = p.x * p.x + p.y * p.y + p.z * p.z;  // glm::length2
      if (1e-160 < static_cast<double>(lensq) && lensq <= 1.0f) {
        const float s = std::sqrt(lensq);
        noise[size_t(i) * 3 + 0] = p.x / s;
        noise[size_t(i) * 3 + 1] = p.y / s;
        noise[size_t(i) * 3 + 2] = p.z / s;
        break;
      }
    }
  }
  // main.cpp:277-280: randomVec3(0, 1)
  for (uint32_t i = 0; i < texels; ++i) {
    const Vec3 p = RandomVec3(g, 0.0f, 1.0f, gcc_order);
    noise_u[size_t(i) * 3 + 0] = p.x;
    noise_u[size_t(i) * 3 + 1] = p.y;
    noise_u[size_t(i) * 3 + 2] = p.z;
  }
}

}  // namespace srt
