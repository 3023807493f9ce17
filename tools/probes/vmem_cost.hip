// vmem_cost.hip -- what a divergent dwordx4 gather costs the vector-memory pipeline (TA / TD / L1) on
// gfx950, as a function of the instruction's active lanes and of the distinct 128-B lines they touch.
// Measurement probe for DESIGN.md section 5 (the global-scene kernels wait on TA/TD); not product code.
//
// Every lane of a wave reads 64-B records (4 x dwordx4, as a traversal step reads a node pair) from an
// L2-resident table (2 MiB, so L1 misses and L2 hits, as the surface legs' loads mostly are).  Per case:
//   A  lanes active (lane < A; the rest masked off by the branch),
//   D  distinct lines per instruction (lane l reads line h(l % D), record (l / D) & 1 of its two),
// and the time per load instruction per CU (all CUs busy: 8 waves per SIMD).  Grouped cases (G > 1): the
// lanes of each group of G read G consecutive 16-B pieces of one random record per instruction (a
// cooperative load: G lanes fetch one lane's record together, then exchange within the group).
//
// build: hipcc -O3 --offload-arch=gfx950 -o tools/probes/vmem_cost tools/probes/vmem_cost.hip
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

__global__ __launch_bounds__(256) void gather_kernel(const uint4* __restrict__ t, uint32_t n_lines, int iters,
                                                     int A, int D, uint32_t* out) {
  const int lane = threadIdx.x & 63;
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  uint32_t acc = 0;
  if (D < 0 && lane < A) {  // grouped: G = -D lanes read one record's consecutive pieces per instruction
    const int G = -D;
    const uint32_t grp = (uint32_t)(lane / G), piece = (uint32_t)(lane % G);
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {  // 4 instructions, each a different record of the group
        const uint32_t line = mix32(wave * 0x9E3779B9u + (uint32_t)(4 * it + k) * 0x85EBCA6Bu + grp * 0xC2B2AE35u) % n_lines;
        const uint4 a = t[(size_t)line * 8 + piece];
        acc ^= a.x ^ (a.y + a.z + a.w);
      }
    }
  } else if (lane < A) {
    const uint32_t grp = (uint32_t)(lane % D), rec = (uint32_t)((lane / D) & 1);
    for (int it = 0; it < iters; ++it) {
      const uint32_t line = mix32(wave * 0x9E3779B9u + (uint32_t)it * 0x85EBCA6Bu + grp * 0xC2B2AE35u) % n_lines;
      const uint4* p = t + (size_t)line * 8 + rec * 4;  // 128-B line = 8 uint4, two 64-B records
      const uint4 a = p[0], b = p[1], c = p[2], d = p[3];
      acc ^= a.x ^ b.y ^ c.z ^ d.w ^ (a.w + b.x + c.y + d.z);
    }
  }
  if (acc == 0x12345678u) out[0] = acc;  // keeps the loads live
}

// per lane one random 16-B, 8-B or 4-B piece per instruction (W = 4, 2 or 1 dwords), all 64 lanes divergent
template <int W>
__global__ __launch_bounds__(256) void width_kernel(const uint32_t* __restrict__ t, uint32_t n_lines, int iters,
                                                    uint32_t* out) {
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc = 0;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t line = mix32(gid * 0x9E3779B9u + (uint32_t)(4 * it + k) * 0x85EBCA6Bu) % n_lines;
      const uint32_t* p = t + (size_t)line * 32;
      if constexpr (W == 4) {
        const uint4 v = *reinterpret_cast<const uint4*>(p);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
      } else if constexpr (W == 2) {
        const uint2 v = *reinterpret_cast<const uint2*>(p);
        acc ^= v.x ^ v.y;
      } else {
        acc ^= *p;
      }
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main(int argc, char** argv) {
  const size_t bytes = 2u << 20;
  const uint32_t n_lines = (uint32_t)(bytes / 128);
  uint4* t;
  uint32_t* out;
  CK(hipMalloc(&t, bytes));
  CK(hipMalloc(&out, 4));
  CK(hipMemset(t, 1, bytes));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int blocks = cus * 8;  // 256-lane blocks: 8 waves per SIMD
  const int iters = 2000;
  const int cases[][2] = {{64, 64}, {48, 48}, {32, 32}, {16, 16}, {8, 8}, {64, 32}, {64, 16}, {64, 8}, {32, 16}, {32, 8},
                          {64, -2}, {64, -4}, {64, -8}, {32, -4}, {32, -8}};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL(gather_kernel, dim3(blocks), dim3(256), 0, 0, t, n_lines, 50, 64, 64, out);  // warm-up
  CK(hipDeviceSynchronize());
  std::printf("{\"probe\": \"vmem_cost\", \"table_bytes\": %zu, \"cus\": %d, \"waves_per_simd\": 8, \"rows\": [\n", bytes, cus);
  const int n = (int)(sizeof(cases) / sizeof(cases[0]));
  for (int k = 0; k < n; ++k) {
    const int A = cases[k][0], D = cases[k][1];
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(gather_kernel, dim3(blocks), dim3(256), 0, 0, t, n_lines, iters, A, D, out);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    const double instr_per_cu = (double)blocks * 4 * iters * 4 / cus;  // waves x iterations x 4 loads
    const double ns = best * 1e6 / instr_per_cu;
    std::printf("  {\"active_lanes\": %d, \"%s\": %d, \"ms\": %.3f, \"ns_per_load_instr_per_cu\": %.4f, "
                "\"cycles_at_2p4GHz\": %.2f}%s\n", A, D < 0 ? "lanes_per_record_group" : "lines_per_instr",
                D < 0 ? -D : D, best, ns, ns * 2.4, k + 1 < n ? "," : "");
  }
  std::printf("], \"widths\": [\n");
  for (int W : {4, 2, 1}) {
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipEventRecord(e0));
      if (W == 4) hipLaunchKernelGGL(width_kernel<4>, dim3(blocks), dim3(256), 0, 0, (const uint32_t*)t, n_lines, iters, out);
      else if (W == 2) hipLaunchKernelGGL(width_kernel<2>, dim3(blocks), dim3(256), 0, 0, (const uint32_t*)t, n_lines, iters, out);
      else hipLaunchKernelGGL(width_kernel<1>, dim3(blocks), dim3(256), 0, 0, (const uint32_t*)t, n_lines, iters, out);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    const double instr_per_cu = (double)blocks * 4 * iters * 4 / cus;
    const double ns = best * 1e6 / instr_per_cu;
    std::printf("  {\"dwords_per_lane\": %d, \"active_lanes\": 64, \"ms\": %.3f, \"cycles_at_2p4GHz\": %.2f}%s\n", W, best,
                ns * 2.4, W != 1 ? "," : "");
  }
  std::printf("]}\n");
  return 0;
}
