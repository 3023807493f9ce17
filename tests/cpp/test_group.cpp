// test_group.cpp -- src/main.cpp's progressive loop over a Graphics::ComputeGroup (include/srt/srt.hpp):
// the frame tiled over the devices named on the command line (a device may repeat), one gather to the
// first.  ./test_group <objects_dir> <shader_dir> <out_prefix> <band_rows> <device>...; prints "OK
// <transport>" and writes <out_prefix>.accum / .rgba8 (the full frame) for tests/test_gpu_group.py.
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "srt/srt.hpp"

using namespace srt;

int main(int argc, char** argv) {
  if (argc < 6) {
    std::printf("FAIL usage\n");
    return 1;
  }
  const std::string objects = argv[1], shaders = argv[2], out_prefix = argv[3];
  const int band_rows = std::atoi(argv[4]);
  std::vector<int> devices;
  for (int i = 5; i < argc; ++i) devices.push_back(std::atoi(argv[i]));
  const int W = 64, H = 48;
  Graphics::ComputeGroup rt((shaders + "raytrace_compute.glsl").c_str(), devices, band_rows);
  auto model = AssetUtils::LoadObject("Rubik", objects);
  rt.ForEach([&](Graphics::Compute& c) {
    c.Use();
    AssetUtils::UploadModelDataToGPU({model.get()}, 5);
  });
  RayTracer::Camera camera(true);
  std::vector<srt_light> lights = {
      RayTracer::PointLight({1, 10, 10}, {1, 1, 1}, 50), RayTracer::PointLight({-5, 15, 10}, {1, 0.2f, 0.2f}, 15),
      RayTracer::PointLight({5, 15, 10}, {0.2f, 1, 0.2f}, 15), RayTracer::PointLight({-5, 5, 10}, {0.2f, 0.2f, 1}, 15),
      RayTracer::PointLight({5, 5, 10}, {1, 1, 0.1f}, 15), RayTracer::PointLight({0, 21, 17}, {1, 1, 1}, 50)};
  std::vector<float> noise, noise_u;
  Common::GenerateNoise(W, H, &noise, &noise_u);
  rt.BindNoise(noise, noise_u);
  rt.BindLights(lights);
  // main.cpp:657-725 for 4 frames: the reset frame (EnableMouseCapture(false) raised the flag), then 3
  // sampled frames from the reset camera
  for (int accumFrames = 1; accumFrames <= 4; ++accumFrames) {
    rt.SetBool("resetAccumBuffer", accumFrames == 1);
    rt.SetVec3("cameraOrigin", camera.getOrigin());
    rt.SetVec3("cameraDirection", camera.getForward());
    rt.SetVec3("cameraUp", camera.getUpVector());
    rt.SetVec3("cameraRight", camera.getRightVector());
    rt.SetInt("accumFrames", accumFrames);
    rt.SetInt("Width", W);
    rt.SetInt("Height", H);
    rt.SetUInt("bvh_count", 1);
    rt.SetInt("lightCount", (int)lights.size());
    rt.SetBool("showModel", true);
    rt.Dispatch(W / 8, H / 8, 1);
    rt.Finish();
  }
  const auto acc = rt.ReadAccum();
  const auto out = rt.ReadOutput();
  FILE* f = std::fopen((out_prefix + ".accum").c_str(), "wb");
  if (!f || std::fwrite(acc.data(), sizeof(float), acc.size(), f) != acc.size()) return 1;
  std::fclose(f);
  f = std::fopen((out_prefix + ".rgba8").c_str(), "wb");
  if (!f || std::fwrite(out.data(), 1, out.size(), f) != out.size()) return 1;
  std::fclose(f);
  const auto ms = rt.KernelMs();
  for (float m : ms)
    if (!(m > 0.0f)) return 2;  // every device ran its launch (HIP events around it)
  std::printf("OK %s %d\n", rt.Transport(), rt.Ranks());
  return 0;
}
