// group.cpp -- the multi-GPU frame of one host process (include/srt_amd.h, srt_group_*).
//
// The reference renders one frame per glDispatchCompute on one GL context (src/main.cpp:657-725).
// Here n contexts, one per device, render interleaved row bands of the same frame (srt_set_tiling)
// and each encodes its own rows' sRGB8 (accumFrames is one uniform for all).  Per frame, the only
// exchange is one gather of those 4-B pixels to context 0: ncclGather over xGMI (RCCL) when the
// devices are distinct, device-to-device copies when a device repeats (RCCL takes one rank per
// device; this lets one GPU run the group's whole path for tests).  Context 0 then de-interleaves
// the bands.  The radiance (16 B/px) stays where it was rendered -- the next frame adds to it there
// -- and is gathered only when the full accumulation image is asked for.
//
// Streams.  A context renders on its own stream; each device also has a gather stream, so frame
// k's gather and assembly run beside frame k+1's render.  The sRGB8 band images are
// double-buffered for that: frame k writes buffer k % 2, and a render waits (hipStreamWaitEvent)
// for the gather that last read the buffer it is about to write, and for the last radiance
// gather.  Under the copy transport a context's copy into context 0's receive buffer waits for
// the previous assembly, which read that buffer.
#include <dlfcn.h>
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "srt_internal.hpp"

namespace {

// RCCL, loaded when the first group that needs it is created: the library itself does not depend on
// it, so an embedder that never tiles a frame over devices needs no librccl.  (When PyTorch has
// loaded its own librccl.so.1 first, dlopen returns that one: both carry the soname.)
struct Rccl {
  bool ok = false;
  std::string err;
  decltype(&ncclCommInitAll) CommInitAll = nullptr;
  decltype(&ncclCommDestroy) CommDestroy = nullptr;
  decltype(&ncclCommCount) CommCount = nullptr;
  decltype(&ncclGather) Gather = nullptr;
  decltype(&ncclGroupStart) GroupStart = nullptr;
  decltype(&ncclGroupEnd) GroupEnd = nullptr;
  decltype(&ncclGetErrorString) GetErrorString = nullptr;
};

const Rccl& rccl() {
  static const Rccl r = [] {
    Rccl x;
    void* h = nullptr;
    for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
      if ((h = dlopen(name, RTLD_NOW | RTLD_GLOBAL)) != nullptr) break;
    if (!h) {
      const char* e = dlerror();
      x.err = std::string("cannot load librccl.so.1: ") + (e ? e : "");
      return x;
    }
    auto sym = [&](auto* fn, const char* name) {
      *fn = reinterpret_cast<std::remove_pointer_t<decltype(fn)>>(dlsym(h, name));
      if (!*fn && x.err.empty()) x.err = std::string("librccl: no symbol ") + name;
    };
    sym(&x.CommInitAll, "ncclCommInitAll");
    sym(&x.CommDestroy, "ncclCommDestroy");
    sym(&x.CommCount, "ncclCommCount");
    sym(&x.Gather, "ncclGather");
    sym(&x.GroupStart, "ncclGroupStart");
    sym(&x.GroupEnd, "ncclGroupEnd");
    sym(&x.GetErrorString, "ncclGetErrorString");
    x.ok = x.err.empty();
    return x;
  }();
  return r;
}

// One host thread per context beyond the first: every device's launches of a frame are enqueued at
// once rather than one device after another (a launch costs tens of microseconds of host API calls,
// so with 8 devices the last would start a good fraction of a millisecond after the first).
// Run(job) calls job(i) for every context i, job(0) on the calling thread, and returns the first
// non-zero status.  SRT_GROUP_THREADS=0 enqueues serially on the calling thread.
class Workers {
 public:
  Workers(int n, bool threads) : rc_(n, 0) {
    if (threads)
      for (int i = 1; i < n; ++i) threads_.emplace_back([this, i] { Loop(i); });
  }
  ~Workers() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : threads_) t.join();
  }
  int Run(const std::function<int(int)>& job) {
    const int n = (int)rc_.size();
    if (threads_.empty()) {
      for (int i = 0; i < n; ++i)
        if (int rc = job(i)) return rc;
      return 0;
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      job_ = &job;
      pending_ = n - 1;
      ++gen_;
    }
    cv_.notify_all();
    rc_[0] = job(0);
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [this] { return pending_ == 0; });
    job_ = nullptr;
    for (int r : rc_)
      if (r) return r;
    return 0;
  }

 private:
  void Loop(int i) {
    long long seen = 0;
    for (;;) {
      const std::function<int(int)>* job = nullptr;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        job = job_;
      }
      const int r = (*job)(i);
      std::lock_guard<std::mutex> lk(mu_);
      rc_[i] = r;
      if (--pending_ == 0) done_cv_.notify_one();
    }
  }
  std::vector<std::thread> threads_;
  std::vector<int> rc_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<int(int)>* job_ = nullptr;
  long long gen_ = 0;
  int pending_ = 0;
  bool stop_ = false;
};

}  // namespace

struct srt_group {
  std::unique_ptr<Workers> workers;  // per-context launch threads
  std::vector<srt_context*> ctx;
  std::vector<int> dev;
  std::vector<hipStream_t> stream;  // each context's render stream (srt_stream)
  std::vector<hipStream_t> xfer;    // per context: its gather stream (on its device)
  std::vector<ncclComm_t> comm;     // empty: copy transport
  std::vector<hipEvent_t> rendered;  // per context: its launches so far (render stream)
  std::vector<hipEvent_t> sent[2];   // per context and sRGB8 buffer: the gather that read it (gather stream)
  std::vector<hipEvent_t> acc_sent;  // per context: the radiance gather that read its accumulation image
  std::vector<hipEvent_t> arrived;   // per context, copy transport: its rows are in context 0's buffer
  hipEvent_t assembled = nullptr;    // context 0's gather stream: the last assembly (it read recv_*)
  // per context: timing events around its part of each frame's exchange (srt_group_exchange_time), a
  // ring of kExCap pairs created as they are first used; ex_seq frames recorded, ex_read summed
  static constexpr int kExCap = 4096;
  std::vector<std::vector<hipEvent_t>> ex_ev;
  long long ex_seq = 0, ex_read = 0;
  int band_rows = 8;
  int W = 0, H = 0, rows_pad = 0;
  int cur = 0;               // the sRGB8 buffer the next frame writes
  bool accum_stale = false;  // full_accum is older than the contexts' radiance
  long long gathers_out = 0, gathers_acc = 0;
  std::vector<void*> band_accum;  // per context, rows_pad rows RGBA32F (its accumulation image)
  std::vector<void*> band_out[2];  // per context, rows_pad rows RGBA8 (its image0, double-buffered)
  void* recv_out = nullptr;        // context 0: n * rows_pad rows RGBA8
  void* recv_acc = nullptr;        // context 0: n * rows_pad rows RGBA32F (allocated on first use)
  void* full_accum = nullptr;      // context 0: the assembled frame
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
#define GNCCL(x)                                                                        \
  do {                                                                                  \
    ncclResult_t r_ = (x);                                                              \
    if (r_ != ncclSuccess) {                                                            \
      srt::SetError(std::string("group: " #x ": ") + rccl().GetErrorString(r_));      \
      return SRT_ERR_HIP;                                                               \
    }                                                                                   \
  } while (0)

void FreeImages(srt_group* g) {
  for (size_t i = 0; i < g->ctx.size(); ++i) {
    (void)hipSetDevice(g->dev[i]);
    if (i < g->band_accum.size() && g->band_accum[i]) (void)hipFree(g->band_accum[i]);
    for (auto& bo : g->band_out)
      if (i < bo.size() && bo[i]) (void)hipFree(bo[i]);
  }
  g->band_accum.clear();
  for (auto& bo : g->band_out) bo.clear();
  if (!g->dev.empty()) (void)hipSetDevice(g->dev[0]);
  for (void* p : {g->recv_out, g->recv_acc, g->full_accum, g->full_out})
    if (p) (void)hipFree(p);
  g->recv_out = g->recv_acc = g->full_accum = g->full_out = nullptr;
}

void DestroyStreamsEvents(srt_group* g) {
  auto destroy = [&](std::vector<hipEvent_t>& v) {
    for (size_t i = 0; i < v.size(); ++i) {
      if (!v[i]) continue;
      (void)hipSetDevice(g->dev[i]);
      (void)hipEventDestroy(v[i]);
    }
    v.clear();
  };
  for (size_t i = 0; i < g->ex_ev.size(); ++i) {  // context i's exchange timing events, on its device
    (void)hipSetDevice(g->dev[i]);
    for (hipEvent_t e : g->ex_ev[i])
      if (e) (void)hipEventDestroy(e);
  }
  g->ex_ev.clear();
  destroy(g->rendered);
  destroy(g->sent[0]);
  destroy(g->sent[1]);
  destroy(g->acc_sent);
  destroy(g->arrived);
  if (g->assembled) {
    (void)hipSetDevice(g->dev[0]);
    (void)hipEventDestroy(g->assembled);
    g->assembled = nullptr;
  }
  for (size_t i = 0; i < g->xfer.size(); ++i) {
    if (!g->xfer[i]) continue;
    (void)hipSetDevice(g->dev[i]);
    (void)hipStreamDestroy(g->xfer[i]);
  }
  g->xfer.clear();
}

int CreateStreamsEvents(srt_group* g) {
  const int n = (int)g->ctx.size();
  g->xfer.assign(n, nullptr);
  for (auto* v : {&g->rendered, &g->sent[0], &g->sent[1], &g->acc_sent, &g->arrived}) v->assign(n, nullptr);
  for (int i = 0; i < n; ++i) {
    GHIP(hipSetDevice(g->dev[i]));
    GHIP(hipStreamCreateWithFlags(&g->xfer[i], hipStreamNonBlocking));
    for (auto* v : {&g->rendered, &g->sent[0], &g->sent[1], &g->acc_sent, &g->arrived}) {
      GHIP(hipEventCreateWithFlags(&(*v)[i], hipEventDisableTiming));
      GHIP(hipEventRecord((*v)[i], g->xfer[i]));  // recorded once: every wait below has a completed event
    }
  }
  GHIP(hipSetDevice(g->dev[0]));
  GHIP(hipEventCreateWithFlags(&g->assembled, hipEventDisableTiming));
  GHIP(hipEventRecord(g->assembled, g->xfer[0]));
  return SRT_OK;
}

// Before a launch that writes sRGB8 buffer `b`: context i's image buffers point at its band images,
// and its render stream waits for the gathers that last read them.
int PrepareLaunch(srt_group* g, int i, int b) {
  if (int rc = srt_set_image_buffers(g->ctx[i], g->band_accum[i], g->band_out[b][i])) return rc;
  GHIP(hipSetDevice(g->dev[i]));
  GHIP(hipStreamWaitEvent(g->stream[i], g->sent[b][i], 0));
  GHIP(hipStreamWaitEvent(g->stream[i], g->acc_sent[i], 0));
  return SRT_OK;
}

// One gather of every context's `bytes` at send[i] into context 0's `recv` (rank order), on the
// gather streams, behind each context's launches so far; `sent_ev[i]` marks the end of context i's
// part (its send buffer may be written again after it).
// Timing event `k` (0: start, 1: end) of context i's part of exchange frame g->ex_seq, created on first use.
int ExEvent(srt_group* g, int i, int k, hipEvent_t* out) {
  auto& v = g->ex_ev[i];
  const size_t at = 2 * (size_t)(g->ex_seq % srt_group::kExCap) + k;
  if (v.size() <= at) v.resize(at + 1, nullptr);
  if (!v[at]) GHIP(hipEventCreate(&v[at]));  // (the caller has set context i's device)
  *out = v[at];
  return SRT_OK;
}

// `timed`: the per-frame exchange, whose parts srt_group_exchange_time reports.
int Gather(srt_group* g, const std::vector<void*>& send, void* recv, size_t bytes, std::vector<hipEvent_t>& sent_ev,
           bool timed) {
  const int n = (int)g->ctx.size();
  if (timed && g->ex_ev.size() != (size_t)n) g->ex_ev.resize(n);
  for (int i = 0; i < n; ++i) {
    GHIP(hipSetDevice(g->dev[i]));
    GHIP(hipEventRecord(g->rendered[i], g->stream[i]));
    GHIP(hipStreamWaitEvent(g->xfer[i], g->rendered[i], 0));
    if (timed) {
      hipEvent_t e;
      if (int rc = ExEvent(g, i, 0, &e)) return rc;
      GHIP(hipEventRecord(e, g->xfer[i]));
    }
  }
  if (!g->comm.empty()) {
    const Rccl& R = rccl();
    GNCCL(R.GroupStart());
    for (int i = 0; i < n; ++i) {
      GHIP(hipSetDevice(g->dev[i]));
      GNCCL(R.Gather(send[i], i == 0 ? recv : nullptr, bytes, ncclUint8, 0, g->comm[i], g->xfer[i]));
    }
    GNCCL(R.GroupEnd());
  } else {
    for (int i = 0; i < n; ++i) {
      GHIP(hipSetDevice(g->dev[i]));
      // context 0's buffer is free once the last assembly (on context 0's gather stream) has read it
      if (i > 0) GHIP(hipStreamWaitEvent(g->xfer[i], g->assembled, 0));
      char* dst = static_cast<char*>(recv) + (size_t)i * bytes;
      GHIP(hipMemcpyPeerAsync(dst, g->dev[0], send[i], g->dev[i], bytes, g->xfer[i]));
      GHIP(hipEventRecord(g->arrived[i], g->xfer[i]));
    }
    GHIP(hipSetDevice(g->dev[0]));
    for (int i = 1; i < n; ++i) GHIP(hipStreamWaitEvent(g->xfer[0], g->arrived[i], 0));
  }
  for (int i = 0; i < n; ++i) {
    GHIP(hipSetDevice(g->dev[i]));
    GHIP(hipEventRecord(sent_ev[i], g->xfer[i]));
    if (timed && i > 0) {  // (context 0's part ends after the assembly, GatherOutput)
      hipEvent_t e;
      if (int rc = ExEvent(g, i, 1, &e)) return rc;
      GHIP(hipEventRecord(e, g->xfer[i]));
    }
  }
  GHIP(hipSetDevice(g->dev[0]));
  return SRT_OK;
}

// Frame's end: the sRGB8 rows of buffer `b` to context 0, de-interleaved into full_out over the
// dispatch extent.
int GatherOutput(srt_group* g, int b, int ext_w, int ext_h) {
  const size_t bytes = (size_t)g->rows_pad * g->W * 4;
  if (int rc = Gather(g, g->band_out[b], g->recv_out, bytes, g->sent[b], true)) return rc;
  if (int rc = srt::AssembleOutputOn(g->ctx[0], g->xfer[0], g->recv_out, (int)g->ctx.size(), g->rows_pad,
                                     g->band_rows, ext_w, ext_h, g->full_out))
    return rc;
  GHIP(hipEventRecord(g->assembled, g->xfer[0]));
  hipEvent_t e;
  if (int rc = ExEvent(g, 0, 1, &e)) return rc;
  GHIP(hipEventRecord(e, g->xfer[0]));
  ++g->ex_seq;
  ++g->gathers_out;
  return SRT_OK;
}

// The radiance rows to context 0 (only when the full accumulation image is asked for).
int GatherAccum(srt_group* g) {
  if (!g->accum_stale) return SRT_OK;
  const int n = (int)g->ctx.size();
  const size_t bytes = (size_t)g->rows_pad * g->W * 16;
  if (!g->recv_acc) {
    GHIP(hipSetDevice(g->dev[0]));
    GHIP(hipMalloc(&g->recv_acc, (size_t)n * bytes));
  }
  if (int rc = Gather(g, g->band_accum, g->recv_acc, bytes, g->acc_sent, false)) return rc;
  if (int rc = srt::AssembleBandsOn(g->ctx[0], g->xfer[0], g->recv_acc, n, g->rows_pad, g->band_rows, 1,
                                    g->full_accum, nullptr))
    return rc;
  GHIP(hipEventRecord(g->assembled, g->xfer[0]));
  ++g->gathers_acc;
  g->accum_stale = false;
  return SRT_OK;
}

// A frame some contexts enqueued and others failed to: the contexts' radiance may have moved, so the
// assembled copy is stale, and everything in flight is drained (no gather may still read a buffer the
// next frame writes).  Returns the frame's error.
int Abandon(srt_group* g, int rc) {
  g->accum_stale = true;
  (void)srt_group_finish(g);
  return rc;
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
    const Rccl& R = rccl();
    if (!R.ok) {
      srt::SetError("group: " + R.err);
      delete g;
      return SRT_ERR_HIP;
    }
    g->comm.resize(n);
    const ncclResult_t r = R.CommInitAll(g->comm.data(), n, g->dev.data());
    if (r != ncclSuccess) {
      srt::SetError(std::string("group: ncclCommInitAll: ") + R.GetErrorString(r));
      g->comm.clear();
      delete g;
      return SRT_ERR_HIP;
    }
    for (int i = 0; i < n; ++i) {  // every communicator must see all n ranks, or the gather is not the frame
      int count = 0;
      const ncclResult_t rc = R.CommCount(g->comm[i], &count);
      if (rc != ncclSuccess || count != n) {
        srt::SetError("group: ncclCommCount of communicator " + std::to_string(i) + " is " + std::to_string(count) +
                      ", not the group's " + std::to_string(n) + " ranks");
        for (ncclComm_t cm : g->comm) (void)R.CommDestroy(cm);
        g->comm.clear();
        delete g;
        return SRT_ERR_HIP;
      }
    }
  }
  if (int rc = CreateStreamsEvents(g)) {
    srt_group_destroy(g);
    return rc;
  }
  const char* th = std::getenv("SRT_GROUP_THREADS");
  g->workers = std::make_unique<Workers>(n, !(th && th[0] == '0'));
  *out = g;
  return SRT_OK;
}

int srt_group_destroy(srt_group* g) {
  if (!g) return SRT_ERR_INVALID;
  g->workers.reset();
  (void)srt_group_finish(g);
  // the contexts outlive the group: detach each from the band images freed below (rank 0 of 1, no
  // images; nothing is allocated here -- the caller gives a context images again before dispatching it)
  if (!g->band_accum.empty())
    for (srt_context* c : g->ctx) (void)srt::DetachImages(c);
  FreeImages(g);
  if (!g->comm.empty())
    for (ncclComm_t c : g->comm) (void)rccl().CommDestroy(c);
  DestroyStreamsEvents(g);
  delete g;
  return SRT_OK;
}

const char* srt_group_transport(srt_group* g) { return !g ? "" : g->comm.empty() ? "copy" : "rccl"; }

int srt_group_get_int(srt_group* g, const char* name, int* v) {
  if (!g || !name || !v) return SRT_ERR_INVALID;
  const std::string k(name);
  const int n = (int)g->ctx.size();
  if (k == "contexts") {
    *v = n;
  } else if (k == "ranks") {
    *v = n;
    if (!g->comm.empty()) {
      int count = 0;
      GNCCL(rccl().CommCount(g->comm[0], &count));
      *v = count;
    }
  } else if (k == "gathers.output") {
    *v = (int)std::min<long long>(g->gathers_out, 0x7FFFFFFF);
  } else if (k == "gathers.accum") {
    *v = (int)std::min<long long>(g->gathers_acc, 0x7FFFFFFF);
  } else if (k == "bytes.output") {
    *v = (int)((size_t)n * g->rows_pad * g->W * 4 / 1024);
  } else if (k == "bytes.accum") {
    *v = (int)((size_t)n * g->rows_pad * g->W * 16 / 1024);
  } else {
    return SRT_ERR_NOT_FOUND;
  }
  return SRT_OK;
}

int srt_group_last_kernel_ms(srt_group* g, float* ms, int n) {
  if (!g || !ms || n < 0) return SRT_ERR_INVALID;
  for (int i = 0; i < n && i < (int)g->ctx.size(); ++i)
    if (int rc = srt_last_kernel_ms(g->ctx[i], ms + i)) return rc;
  return SRT_OK;
}

int srt_group_kernel_time(srt_group* g, double* total_ms, int* launches, int n) {
  if (!g || !total_ms || !launches || n < 0) return SRT_ERR_INVALID;
  int first = SRT_OK;
  for (int i = 0; i < n && i < (int)g->ctx.size(); ++i) {  // (every context's records are consumed)
    const int rc = srt_kernel_time(g->ctx[i], total_ms + i, launches + i);
    if (rc && !first) first = rc;
  }
  return first;
}

int srt_group_exchange_time(srt_group* g, double* total_ms, int* frames, int n) {
  if (!g || !total_ms || !frames || n < 0) return SRT_ERR_INVALID;
  const int m = std::min(n, (int)g->ctx.size());
  for (int i = 0; i < m; ++i) total_ms[i] = 0.0, frames[i] = 0;
  for (size_t i = 0; i < g->xfer.size(); ++i) {
    GHIP(hipSetDevice(g->dev[i]));
    GHIP(hipStreamSynchronize(g->xfer[i]));
  }
  const long long from = g->ex_read;
  g->ex_read = g->ex_seq;
  if (g->ex_seq - from > srt_group::kExCap) {
    srt::SetError("srt_group_exchange_time: more than 4096 frames since the last call (timing events reused)");
    return SRT_ERR_LIMIT;
  }
  for (int i = 0; i < m && i < (int)g->ex_ev.size(); ++i) {
    GHIP(hipSetDevice(g->dev[i]));
    for (long long q = from; q < g->ex_seq; ++q) {
      const size_t at = 2 * (size_t)(q % srt_group::kExCap);
      float t = 0.0f;
      GHIP(hipEventElapsedTime(&t, g->ex_ev[i][at], g->ex_ev[i][at + 1]));
      total_ms[i] += t;
      ++frames[i];
    }
  }
  GHIP(hipSetDevice(g->dev[0]));
  return SRT_OK;
}

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
  if (int rc = srt_group_finish(g)) return rc;
  FreeImages(g);
  g->W = W;
  g->H = H;
  g->cur = 0;
  g->accum_stale = false;
  const int bands = (H + g->band_rows - 1) / g->band_rows;
  g->rows_pad = ((bands + n - 1) / n) * g->band_rows;  // every context's local rows fit, padded equal
  const size_t band_px = (size_t)g->rows_pad * W, full_px = (size_t)W * H;
  g->band_accum.assign(n, nullptr);
  for (auto& bo : g->band_out) bo.assign(n, nullptr);
  for (int i = 0; i < n; ++i) {
    if (int rc = srt_set_tiling(g->ctx[i], i, n, g->band_rows)) return rc;
    GHIP(hipSetDevice(g->dev[i]));
    GHIP(hipMalloc(&g->band_accum[i], band_px * 16));
    GHIP(hipMemset(g->band_accum[i], 0, band_px * 16));
    for (auto& bo : g->band_out) {
      GHIP(hipMalloc(&bo[i], band_px * 4));
      GHIP(hipMemset(bo[i], 0, band_px * 4));
    }
    if (int rc = srt_set_image_buffers(g->ctx[i], g->band_accum[i], g->band_out[0][i])) return rc;
  }
  GHIP(hipSetDevice(g->dev[0]));
  GHIP(hipMalloc(&g->recv_out, (size_t)n * band_px * 4));
  GHIP(hipMalloc(&g->full_accum, full_px * 16));
  GHIP(hipMalloc(&g->full_out, full_px * 4));
  GHIP(hipMemset(g->full_accum, 0, full_px * 16));
  GHIP(hipMemset(g->full_out, 0, full_px * 4));
  return SRT_OK;
}

int srt_group_dispatch(srt_group* g, uint32_t gx, uint32_t gy) {
  if (!g || !g->recv_out) return SRT_ERR_STATE;
  const int b = g->cur;
  if (int rc = g->workers->Run([&](int i) {
        if (int r = PrepareLaunch(g, i, b)) return r;
        return srt_dispatch(g->ctx[i], gx, gy);
      }))
    return Abandon(g, rc);
  g->accum_stale = true;
  int reset = 0;
  srt_get_int(g->ctx[0], "resetAccumBuffer", &reset);
  if (reset) return SRT_OK;  // the reset dispatch stores no image0 pixel
  const int ext_w = (int)std::min<uint64_t>((uint64_t)gx * 8, (uint64_t)g->W);
  const int ext_h = (int)std::min<uint64_t>((uint64_t)gy * 8, (uint64_t)g->H);
  const int rc = GatherOutput(g, g->cur, ext_w, ext_h);
  g->cur ^= 1;
  return rc;
}

int srt_group_render_frames(srt_group* g, int frame_first, int nframes) {
  if (!g || !g->recv_out) return SRT_ERR_STATE;
  if (nframes < 0 || frame_first < 1) return SRT_ERR_INVALID;
  if (nframes == 0) return SRT_OK;
  const int b = g->cur;
  if (int rc = g->workers->Run([&](int i) {
        if (int r = PrepareLaunch(g, i, b)) return r;
        return srt_render_frames(g->ctx[i], frame_first, nframes, 1, 0);
      }))
    return Abandon(g, rc);
  g->accum_stale = true;
  const int rc = GatherOutput(g, g->cur, g->W, g->H);
  g->cur ^= 1;
  return rc;
}

int srt_group_finish(srt_group* g) {
  if (!g) return SRT_ERR_INVALID;
  for (size_t i = 0; i < g->xfer.size(); ++i) {
    if (!g->xfer[i]) continue;
    GHIP(hipSetDevice(g->dev[i]));
    GHIP(hipStreamSynchronize(g->xfer[i]));
  }
  for (srt_context* c : g->ctx)
    if (int rc = srt_finish(c)) return rc;
  return SRT_OK;
}

int srt_group_read_accum(srt_group* g, float* host, size_t bytes) {
  if (!g || !host || !g->full_accum) return SRT_ERR_INVALID;
  const size_t need = (size_t)g->W * g->H * 16;
  if (bytes < need) return SRT_ERR_INVALID;
  if (int rc = GatherAccum(g)) return rc;
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
  if (accum_dev && g->full_accum)
    if (int rc = GatherAccum(g)) return rc;
  if (accum_dev) *accum_dev = g->full_accum;
  if (out_dev) *out_dev = g->full_out;
  return SRT_OK;
}

}  // extern "C"
