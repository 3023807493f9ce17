// coop_quad.hip -- does a quad-cooperative gather pay once the exchange is counted?  Probe for the global-
// scene kernels; not product code.
//
// Each lane of a wave needs, per step, one random 64-B record (4 x float4, as a traversal sub-step needs a
// node pair) with probability P (else it idles that step), and does W dependent FMAs on it.
//   div   each lane loads its own record: 4 divergent dwordx4 gathers (one 16-B piece per lane each);
//   quad  the 4 lanes of a quad load the 4 records of its members together: in instruction k every lane
//         reads piece (lane & 3) of member k's record (one contiguous 64-B segment per quad), then a 4 x 4
//         transpose across the quad (DPP quad_perm moves + selects) gives each lane its own 4 pieces.
// 256-lane blocks at 5 waves per SIMD (__launch_bounds__(256, 5)); time per step per CU.
//
// build: hipcc -O3 --offload-arch=gfx950 -o tools/probes/coop_quad tools/probes/coop_quad.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                 \
    }                                                                               \
  } while (0)

__device__ __forceinline__ uint32_t mix32(uint32_t z) {
  z = (z ^ (z >> 16)) * 0x7feb352du;
  z = (z ^ (z >> 15)) * 0x846ca68bu;
  return z ^ (z >> 16);
}

// quad_perm DPP control: lane j of each quad reads lane p[j]
constexpr int qp(int a, int b, int c, int d) { return a | (b << 2) | (c << 4) | (d << 6); }
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
template <int CTRL>
__device__ __forceinline__ uint32_t dppu(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true);
}
template <int CTRL>
__device__ __forceinline__ float4 dpp4(float4 v) {
  return make_float4(dppf<CTRL>(v.x), dppf<CTRL>(v.y), dppf<CTRL>(v.z), dppf<CTRL>(v.w));
}
__device__ __forceinline__ float4 sel4(bool c, float4 a, float4 b) {
  return make_float4(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z, c ? a.w : b.w);
}

// r_k = piece (lane & 3) of member k's record  ->  r_m = piece m of this lane's record
__device__ __forceinline__ void quad_transpose(float4& r0, float4& r1, float4& r2, float4& r3, int j) {
  const bool b0 = (j & 1) != 0, b1 = (j & 2) != 0;
  {  // stage 1 (bit 0): across lanes j ^ 1, the odd lanes send r0 / r2, the even ones r1 / r3
    const float4 y01 = dpp4<qp(1, 0, 3, 2)>(sel4(b0, r0, r1)), y23 = dpp4<qp(1, 0, 3, 2)>(sel4(b0, r2, r3));
    r0 = sel4(b0, y01, r0);
    r1 = sel4(b0, r1, y01);
    r2 = sel4(b0, y23, r2);
    r3 = sel4(b0, r3, y23);
  }
  {  // stage 2 (bit 1): across lanes j ^ 2, lanes 2-3 send r0 / r1, lanes 0-1 r2 / r3
    const float4 y02 = dpp4<qp(2, 3, 0, 1)>(sel4(b1, r0, r2)), y13 = dpp4<qp(2, 3, 0, 1)>(sel4(b1, r1, r3));
    r0 = sel4(b1, y02, r0);
    r2 = sel4(b1, r2, y02);
    r1 = sel4(b1, y13, r1);
    r3 = sel4(b1, r3, y13);
  }
}

// the quad's cooperative load: every lane loads piece j of each member's record (masked where that member
// needs none), then the transpose
__device__ __forceinline__ void quad_load(const float4* __restrict__ t, uint32_t rec, bool need, int j, float4& r0,
                                          float4& r1, float4& r2, float4& r3) {
  const uint32_t nd = need ? 1u : 0u;
  const uint32_t a0 = dppu<qp(0, 0, 0, 0)>(rec), a1 = dppu<qp(1, 1, 1, 1)>(rec), a2 = dppu<qp(2, 2, 2, 2)>(rec),
                 a3 = dppu<qp(3, 3, 3, 3)>(rec);
  const uint32_t n0 = dppu<qp(0, 0, 0, 0)>(nd), n1 = dppu<qp(1, 1, 1, 1)>(nd), n2 = dppu<qp(2, 2, 2, 2)>(nd),
                 n3 = dppu<qp(3, 3, 3, 3)>(nd);
  typedef float v4f __attribute__((ext_vector_type(4)));
  const v4f* tv = reinterpret_cast<const v4f*>(t);
  v4f v0 = {0.f, 0.f, 0.f, 0.f}, v1 = v0, v2 = v0, v3 = v0;
  if (n0) v0 = tv[(size_t)a0 * 4 + j];
  if (n1) v1 = tv[(size_t)a1 * 4 + j];
  if (n2) v2 = tv[(size_t)a2 * 4 + j];
  if (n3) v3 = tv[(size_t)a3 * 4 + j];
  r0 = make_float4(v0.x, v0.y, v0.z, v0.w);
  r1 = make_float4(v1.x, v1.y, v1.z, v1.w);
  r2 = make_float4(v2.x, v2.y, v2.z, v2.w);
  r3 = make_float4(v3.x, v3.y, v3.z, v3.w);
  quad_transpose(r0, r1, r2, r3, j);
}

// W rounds of 8 independent FMAs on the record (as a node pair's two box tests are ~50 VALU)
template <int W>
__device__ __forceinline__ float work(const float4 r[4], float acc) {
  float a0 = acc, a1 = r[0].x, a2 = r[1].y, a3 = r[2].z;
#pragma unroll
  for (int i = 0; i < W; ++i) {
    a0 = __builtin_fmaf(a0, r[0].x, r[1].y);
    a1 = __builtin_fmaf(a1, r[0].y, r[2].z);
    a2 = __builtin_fmaf(a2, r[1].z, r[3].w);
    a3 = __builtin_fmaf(a3, r[2].w, r[3].x);
    a0 = __builtin_fmaf(a0, r[3].y, r[0].z);
    a1 = __builtin_fmaf(a1, r[1].x, r[2].y);
    a2 = __builtin_fmaf(a2, r[2].x, r[1].w);
    a3 = __builtin_fmaf(a3, r[3].z, r[0].w);
  }
  return (a0 + a1) + (a2 + a3);
}

template <bool QUAD, int W>
__global__ __launch_bounds__(256, 5) void step_kernel(const float4* __restrict__ t, uint32_t n_rec, int iters,
                                                      uint32_t p_thresh, float* out) {
  const int lane = threadIdx.x & 63, j = lane & 3;
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  float acc = 0.0f;
  for (int it = 0; it < iters; ++it) {
    const uint32_t h = mix32(gid * 0x9E3779B9u + (uint32_t)it * 0x85EBCA6Bu);
    const bool need = (h >> 8) < p_thresh;
    const uint32_t rec = mix32(h) % n_rec;
    float4 r[4];
    if constexpr (!QUAD) {
      if (need) {
        const float4* p = t + (size_t)rec * 4;
        r[0] = p[0]; r[1] = p[1]; r[2] = p[2]; r[3] = p[3];
        acc = work<W>(r, acc);
      }
    } else {
      quad_load(t, rec, need, j, r[0], r[1], r[2], r[3]);
      if (need) acc = work<W>(r, acc);
    }
  }
  if (acc == 1234.5f) out[0] = acc;
}

// checks the transpose: every lane's pieces equal the record it asked for
__global__ void check_kernel(const float4* __restrict__ t, uint32_t n_rec, uint32_t* bad) {
  const int lane = threadIdx.x & 63, j = lane & 3;
  const uint32_t rec = mix32(blockIdx.x * blockDim.x + threadIdx.x) % n_rec;
  float4 r0, r1, r2, r3;
  quad_load(t, rec, true, j, r0, r1, r2, r3);
  const float4* w = t + (size_t)rec * 4;
  auto ne = [](float4 a, float4 b) { return a.x != b.x || a.y != b.y || a.z != b.z || a.w != b.w; };
  const uint32_t nbad = (ne(r0, w[0]) ? 1u : 0u) + (ne(r1, w[1]) ? 1u : 0u) + (ne(r2, w[2]) ? 1u : 0u) +
                        (ne(r3, w[3]) ? 1u : 0u);
  if (nbad) atomicAdd(bad, nbad);
  (void)lane;
}

__global__ void fill_kernel(float4* t, uint32_t n) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    t[i] = make_float4((float)i, (float)(i ^ 1u), (float)(i * 3u), (float)(i + 7u));
}

int main() {
  const uint32_t n_rec = (2u << 20) / 64;  // 2 MiB: L2-resident
  float4* t;
  float* out;
  uint32_t* bad;
  CK(hipMalloc(&t, (size_t)n_rec * 64));
  CK(hipMalloc(&out, 4));
  CK(hipMalloc(&bad, 4));
  CK(hipMemset(bad, 0, 4));
  hipLaunchKernelGGL(fill_kernel, dim3(1024), dim3(256), 0, 0, t, n_rec * 4);
  hipLaunchKernelGGL(check_kernel, dim3(1024), dim3(256), 0, 0, t, n_rec, bad);
  uint32_t hbad = 0;
  CK(hipMemcpy(&hbad, bad, 4, hipMemcpyDeviceToHost));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int blocks = cus * 5, iters = 4000;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::printf("{\"probe\": \"coop_quad\", \"transpose_errors\": %u, \"rows\": [\n", hbad);
  const double Ps[] = {1.0, 0.75, 0.5, 0.3};
  const int Ws[] = {2, 6, 12};
  bool first = true;
  for (double P : Ps)
    for (int W : Ws)
      for (int quad = 0; quad < 2; ++quad) {
        const uint32_t th = (uint32_t)(P * 16777216.0);
        float best = 1e30f;
        for (int rep = 0; rep < 3; ++rep) {
          CK(hipEventRecord(e0));
#define LAUNCH(Q, WW) hipLaunchKernelGGL((step_kernel<Q, WW>), dim3(blocks), dim3(256), 0, 0, t, n_rec, iters, th, out)
          if (quad) { if (W == 2) LAUNCH(true, 2); else if (W == 6) LAUNCH(true, 6); else LAUNCH(true, 12); }
          else { if (W == 2) LAUNCH(false, 2); else if (W == 6) LAUNCH(false, 6); else LAUNCH(false, 12); }
          CK(hipEventRecord(e1));
          CK(hipEventSynchronize(e1));
          float ms = 0;
          CK(hipEventElapsedTime(&ms, e0, e1));
          best = ms < best ? ms : best;
        }
        const double steps_per_cu = (double)blocks * 4 * iters / cus;  // wave-steps
        std::printf("%s  {\"mode\": \"%s\", \"need_prob\": %.2f, \"fmas_per_step\": %d, \"ms\": %.3f, \"cycles_per_wave_step_per_cu\": %.2f}",
                    first ? "" : ",\n", quad ? "quad" : "div", P, 8 * W, best, best * 1e-3 * 2.4e9 / steps_per_cu);
        first = false;
      }
  std::printf("\n]}\n");
  return 0;
}
