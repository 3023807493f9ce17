// group.cpp -- the multi-GPU frame of one host process (include/srt_amd.h, srt_group_*).
//
// The reference renders one frame per glDispatchCompute on one GL context (src/main.cpp:657-725).
// Here n contexts, one per device, render interleaved row bands of the same frame (srt_set_tiling),
// and the only exchange is one gather of every context's radiance rows to context 0: ncclGather
// over xGMI (RCCL) when the devices are distinct, device-to-device copies when a device repeats
// (RCCL takes one rank per device; this lets one GPU run the group's whole path for tests).
// Context 0 then de-interleaves the bands and writes the sRGB8 image (srt_assemble_bands).
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <set>
#include <string>
#include <vector>

#include "srt_internal.hpp"

struct srt_group {
  std::vector<srt_context*> ctx;
  std::vector<int> dev;
  std::vector<hipStream_t> stream;
  std::vector<ncclComm_t> comm;  // empty: copy transport
  std::vector<hipEvent_t> done;  // per context: its bands are rendered (copy transport)
  int band_rows = 8;
  int W = 0, H = 0, rows_pad = 0;
  std::vector<void*> band_accum, band_out;  // per context, rows_pad rows (the gather's send buffers)
  void* recv = nullptr;                      // context 0: n * rows_pad rows
  void* full_accum = nullptr;                // context 0: the assembled frame
  void* full_out = nullptr;
};

namespace {

#define GHIP(x)                                                               \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      srt::SetError(std::string("group: " #x ": ") + hipGetErrorString(e_)); \
      return SRT_ERR_HIP;                                                     \
    }                                                                         \
  } while (0)
#define GNCCL(x)                                                                \
  do {                                                                          \
    ncclResult_t r_ = (x);                                                      \
    if (r_ != ncclSuccess) {                                                    \
      srt::SetError(std::string("group: " #x ": ") + ncclGetErrorString(r_)); \
      return SRT_ERR_HIP;                                                       \
    }                                                                           \
  } while (0)

void FreeImages(srt_group* g) {
  for (size_t i = 0; i < g->ctx.size(); ++i) {
    (void)hipSetDevice(g->dev[i]);
    if (i < g->band_accum.size() && g->band_accum[i]) (void)hipFree(g->band_accum[i]);
    if (i < g->band_out.size() && g->band_out[i]) (void)hipFree(g->band_out[i]);
  }
  g->band_accum.clear();
  g->band_out.clear();
  if (!g->dev.empty()) (void)hipSetDevice(g->dev[0]);
  for (void* p : {g->recv, g->full_accum, g->full_out})
    if (p) (void)hipFree(p);
  g->recv = g->full_accum = g->full_out = nullptr;
}

// The gather of every context's band rows into context 0's receive buffer, then the assembly of the
// full frame for accumFrames = `frames` (sRGB8 image too when write_out).
int GatherAssemble(srt_group* g, int frames, bool write_out) {
  const size_t floats = (size_t)g->rows_pad * g->W * 4;
  const int n = (int)g->ctx.size();
  if (!g->comm.empty()) {
    GNCCL(ncclGroupStart());
    for (int i = 0; i < n; ++i) {
      GHIP(hipSetDevice(g->dev[i]));
      GNCCL(ncclGather(g->band_accum[i], i == 0 ? g->recv : nullptr, floats, ncclFloat32, 0, g->comm[i],
                       g->stream[i]));
    }
    GNCCL(ncclGroupEnd());
  } else {
    for (int i = 0; i < n; ++i) {
      GHIP(hipSetDevice(g->dev[i]));
      GHIP(hipEventRecord(g->done[i], g->stream[i]));
    }
    GHIP(hipSetDevice(g->dev[0]));
    for (int i = 0; i < n; ++i) {
      GHIP(hipStreamWaitEvent(g->stream[0], g->done[i], 0));
      char* dst = static_cast<char*>(g->recv) + (size_t)i * floats * sizeof(float);
      GHIP(hipMemcpyPeerAsync(dst, g->dev[0], g->band_accum[i], g->dev[i], floats * sizeof(float), g->stream[0]));
    }
  }
  GHIP(hipSetDevice(g->dev[0]));
  return srt_assemble_bands(g->ctx[0], g->recv, n, g->rows_pad, g->band_rows, std::max(frames, 1), g->full_accum,
                            write_out ? g->full_out : nullptr);
}

}  // namespace

extern "C" {

int srt_group_create(srt_context* const* ctxs, int n, int band_rows, srt_group** out) {
  if (!ctxs || n < 1 || band_rows < 1 || !out) return SRT_ERR_INVALID;
  auto* g = new srt_group();
  g->band_rows = band_rows;
  std::set<int> seen;
  bool repeated = false;
  for (int i = 0; i < n; ++i) {
    if (!ctxs[i]) {
      delete g;
      return SRT_ERR_INVALID;
    }
    g->ctx.push_back(ctxs[i]);
    g->dev.push_back(srt_device(ctxs[i]));
    g->stream.push_back(static_cast<hipStream_t>(srt_stream(ctxs[i])));
    repeated |= !seen.insert(g->dev.back()).second;
  }
  const char* tr = std::getenv("SRT_GROUP_TRANSPORT");
  const bool copy = repeated || (tr && std::string(tr) == "copy");
  if (!copy) {
    g->comm.resize(n);
    const ncclResult_t r = ncclCommInitAll(g->comm.data(), n, g->dev.data());
    if (r != ncclSuccess) {
      srt::SetError(std::string("group: ncclCommInitAll: ") + ncclGetErrorString(r));
      delete g;
      return SRT_ERR_HIP;
    }
  } else {
    g->done.resize(n, nullptr);
    for (int i = 0; i < n; ++i) {
      if (hipSetDevice(g->dev[i]) != hipSuccess ||
          hipEventCreateWithFlags(&g->done[i], hipEventDisableTiming) != hipSuccess) {
        srt::SetError("group: hipEventCreate failed");
        srt_group_destroy(g);
        return SRT_ERR_HIP;
      }
    }
  }
  *out = g;
  return SRT_OK;
}

int srt_group_destroy(srt_group* g) {
  if (!g) return SRT_ERR_INVALID;
  (void)srt_group_finish(g);
  FreeImages(g);
  for (ncclComm_t c : g->comm) (void)ncclCommDestroy(c);
  for (size_t i = 0; i < g->done.size(); ++i) {
    if (!g->done[i]) continue;
    (void)hipSetDevice(g->dev[i]);
    (void)hipEventDestroy(g->done[i]);
  }
  delete g;
  return SRT_OK;
}

const char* srt_group_transport(srt_group* g) { return !g ? "" : g->comm.empty() ? "copy" : "rccl"; }

int srt_group_set_bool(srt_group* g, const char* name, int v) {
  if (!g) return SRT_ERR_INVALID;
  for (srt_context* c : g->ctx)
    if (int rc = srt_set_bool(c, name, v)) return rc;
  return SRT_OK;
}
int srt_group_set_int(srt_group* g, const char* name, int v) {
  if (!g) return SRT_ERR_INVALID;
  for (srt_context* c : g->ctx)
    if (int rc = srt_set_int(c, name, v)) return rc;
  return SRT_OK;
}
int srt_group_set_uint(srt_group* g, const char* name, uint32_t v) {
  if (!g) return SRT_ERR_INVALID;
  for (srt_context* c : g->ctx)
    if (int rc = srt_set_uint(c, name, v)) return rc;
  return SRT_OK;
}
int srt_group_set_vec3(srt_group* g, const char* name, float x, float y, float z) {
  if (!g) return SRT_ERR_INVALID;
  for (srt_context* c : g->ctx)
    if (int rc = srt_set_vec3(c, name, x, y, z)) return rc;
  return SRT_OK;
}

int srt_group_alloc_images(srt_group* g) {
  if (!g) return SRT_ERR_INVALID;
  int W = 0, H = 0;
  if (srt_get_int(g->ctx[0], "Width", &W) || srt_get_int(g->ctx[0], "Height", &H) || W <= 0 || H <= 0)
    return SRT_ERR_STATE;
  const int n = (int)g->ctx.size();
  for (int i = 0; i < n; ++i) {
    int w = 0, h = 0;
    srt_get_int(g->ctx[i], "Width", &w);
    srt_get_int(g->ctx[i], "Height", &h);
    if (w != W || h != H) {
      srt::SetError("group: every context needs the same Width and Height");
      return SRT_ERR_INVALID;
    }
  }
  FreeImages(g);
  g->W = W;
  g->H = H;
  const int bands = (H + g->band_rows - 1) / g->band_rows;
  g->rows_pad = ((bands + n - 1) / n) * g->band_rows;  // every context's local rows fit, padded equal
  const size_t band_px = (size_t)g->rows_pad * W, full_px = (size_t)W * H;
  g->band_accum.assign(n, nullptr);
  g->band_out.assign(n, nullptr);
  for (int i = 0; i < n; ++i) {
    if (int rc = srt_set_tiling(g->ctx[i], i, n, g->band_rows)) return rc;
    GHIP(hipSetDevice(g->dev[i]));
    GHIP(hipMalloc(&g->band_accum[i], band_px * 16));
    GHIP(hipMalloc(&g->band_out[i], band_px * 4));
    GHIP(hipMemset(g->band_accum[i], 0, band_px * 16));
    GHIP(hipMemset(g->band_out[i], 0, band_px * 4));
    if (int rc = srt_set_image_buffers(g->ctx[i], g->band_accum[i], g->band_out[i])) return rc;
  }
  GHIP(hipSetDevice(g->dev[0]));
  GHIP(hipMalloc(&g->recv, (size_t)n * band_px * 16));
  GHIP(hipMalloc(&g->full_accum, full_px * 16));
  GHIP(hipMalloc(&g->full_out, full_px * 4));
  GHIP(hipMemset(g->full_accum, 0, full_px * 16));
  GHIP(hipMemset(g->full_out, 0, full_px * 4));
  return SRT_OK;
}

int srt_group_dispatch(srt_group* g, uint32_t gx, uint32_t gy) {
  if (!g || !g->recv) return SRT_ERR_STATE;
  for (srt_context* c : g->ctx)
    if (int rc = srt_dispatch(c, gx, gy)) return rc;
  int frames = 0, reset = 0;
  srt_get_int(g->ctx[0], "accumFrames", &frames);
  srt_get_int(g->ctx[0], "resetAccumBuffer", &reset);
  return GatherAssemble(g, frames, !reset);
}

int srt_group_render_frames(srt_group* g, int frame_first, int nframes) {
  if (!g || !g->recv) return SRT_ERR_STATE;
  for (srt_context* c : g->ctx)
    if (int rc = srt_render_frames(c, frame_first, nframes, 0, 0)) return rc;
  if (nframes == 0) return SRT_OK;
  return GatherAssemble(g, frame_first + nframes - 1, true);
}

int srt_group_finish(srt_group* g) {
  if (!g) return SRT_ERR_INVALID;
  for (srt_context* c : g->ctx)
    if (int rc = srt_finish(c)) return rc;
  return SRT_OK;
}

int srt_group_read_accum(srt_group* g, float* host, size_t bytes) {
  if (!g || !host || !g->full_accum) return SRT_ERR_INVALID;
  const size_t need = (size_t)g->W * g->H * 16;
  if (bytes < need) return SRT_ERR_INVALID;
  if (int rc = srt_group_finish(g)) return rc;
  GHIP(hipSetDevice(g->dev[0]));
  GHIP(hipMemcpy(host, g->full_accum, need, hipMemcpyDeviceToHost));
  return SRT_OK;
}

int srt_group_read_output(srt_group* g, uint8_t* host, size_t bytes) {
  if (!g || !host || !g->full_out) return SRT_ERR_INVALID;
  const size_t need = (size_t)g->W * g->H * 4;
  if (bytes < need) return SRT_ERR_INVALID;
  if (int rc = srt_group_finish(g)) return rc;
  GHIP(hipSetDevice(g->dev[0]));
  GHIP(hipMemcpy(host, g->full_out, need, hipMemcpyDeviceToHost));
  return SRT_OK;
}

int srt_group_image_pointers(srt_group* g, void** accum_dev, void** out_dev) {
  if (!g) return SRT_ERR_INVALID;
  if (accum_dev) *accum_dev = g->full_accum;
  if (out_dev) *out_dev = g->full_out;
  return SRT_OK;
}

}  // extern "C"
