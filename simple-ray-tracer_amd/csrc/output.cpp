// output.cpp -- the output stage: RGBA8 frames to PNG / PPM files.
//
// Replaces the reference's display path (src/main.cpp:303-349: image0 bound to
// a texture and drawn on a full-screen quad).  The kernel's image has row 0 at
// the bottom (GetRay's j = 0 is the bottom row, raytrace_compute.glsl:78-90, as
// GL textures are stored); files are written top row first, so `flip_y` = 1
// reproduces what the window shows.
#include <zlib.h>

#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/srt_amd.h"
#include "srt_internal.hpp"

namespace {

void PutBe32(std::vector<unsigned char>& v, uint32_t x) {
  v.push_back((unsigned char)(x >> 24));
  v.push_back((unsigned char)(x >> 16));
  v.push_back((unsigned char)(x >> 8));
  v.push_back((unsigned char)x);
}

void PngChunk(std::vector<unsigned char>& out, const char type[4], const unsigned char* data, size_t n) {
  PutBe32(out, (uint32_t)n);
  const size_t at = out.size();
  out.insert(out.end(), type, type + 4);
  if (n) out.insert(out.end(), data, data + n);
  uLong crc = crc32(0L, Z_NULL, 0);
  crc = crc32(crc, out.data() + at, (uInt)(n + 4));
  PutBe32(out, (uint32_t)crc);
}

const uint8_t* Row(const uint8_t* rgba8, int width, int height, int y, int flip_y) {
  const int src = flip_y ? height - 1 - y : y;
  return rgba8 + (size_t)src * width * 4;
}

// 8-bit RGBA, non-interlaced, filter 0 on every scanline, zlib level 6
int WritePng(const std::string& path, const uint8_t* rgba8, int width, int height, int flip_y) {
  std::vector<unsigned char> raw;
  raw.reserve((size_t)height * (1 + (size_t)width * 4));
  for (int y = 0; y < height; ++y) {
    raw.push_back(0);
    const uint8_t* r = Row(rgba8, width, height, y, flip_y);
    raw.insert(raw.end(), r, r + (size_t)width * 4);
  }
  uLongf zlen = compressBound((uLong)raw.size());
  std::vector<unsigned char> z(zlen);
  if (compress2(z.data(), &zlen, raw.data(), (uLong)raw.size(), 6) != Z_OK) return SRT_ERR_IO;
  std::vector<unsigned char> out = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1A, '\n'};
  std::vector<unsigned char> ihdr;
  PutBe32(ihdr, (uint32_t)width);
  PutBe32(ihdr, (uint32_t)height);
  ihdr.insert(ihdr.end(), {8, 6, 0, 0, 0});  // bit depth 8, colour type 6 (RGBA), deflate, filter 0, no interlace
  PngChunk(out, "IHDR", ihdr.data(), ihdr.size());
  PngChunk(out, "IDAT", z.data(), zlen);
  PngChunk(out, "IEND", nullptr, 0);
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) return SRT_ERR_IO;
  const bool ok = std::fwrite(out.data(), 1, out.size(), f) == out.size();
  return (std::fclose(f) == 0 && ok) ? SRT_OK : SRT_ERR_IO;
}

// binary PPM (P6): RGB, alpha dropped
int WritePpm(const std::string& path, const uint8_t* rgba8, int width, int height, int flip_y) {
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) return SRT_ERR_IO;
  bool ok = std::fprintf(f, "P6\n%d %d\n255\n", width, height) > 0;
  std::vector<unsigned char> line((size_t)width * 3);
  for (int y = 0; y < height && ok; ++y) {
    const uint8_t* r = Row(rgba8, width, height, y, flip_y);
    for (int x = 0; x < width; ++x) std::memcpy(&line[(size_t)x * 3], r + (size_t)x * 4, 3);
    ok = std::fwrite(line.data(), 1, line.size(), f) == line.size();
  }
  return (std::fclose(f) == 0 && ok) ? SRT_OK : SRT_ERR_IO;
}

bool EndsWith(const std::string& s, const char* suf) {
  const size_t n = std::strlen(suf);
  if (s.size() < n) return false;
  for (size_t i = 0; i < n; ++i) {
    char c = s[s.size() - n + i];
    if (c >= 'A' && c <= 'Z') c = (char)(c - 'A' + 'a');
    if (c != suf[i]) return false;
  }
  return true;
}

}  // namespace

extern "C" int srt_image_write(const char* path, const uint8_t* rgba8, int width, int height, int flip_y) {
  if (!path || !rgba8 || width <= 0 || height <= 0) return SRT_ERR_INVALID;
  const std::string p(path);
  if (EndsWith(p, ".png")) return WritePng(p, rgba8, width, height, flip_y);
  if (EndsWith(p, ".ppm")) return WritePpm(p, rgba8, width, height, flip_y);
  return SRT_ERR_INVALID;
}
