// gather_calib.hip -- calibration of the memory-side byte counters for the path tracer's access
// patterns (MI355X_MICROARCH.md 'HBM': FETCH_SIZE is calibrated only for 16-B/lane
// streaming reads).  Measurement tool, not part of the product.
//
// Each launch reads a KNOWN number of bytes from a table:
//   stream    16 B per lane, consecutive lanes consecutive (1 KiB per wave-instruction), each byte once
//   rec<R>    every lane reads whole random R-byte records (R/16 dwordx4 loads from one lane, as a
//             traversal step reads a 64-B node pair or a 48-B triangle record), R = 32, 48, 64, 128
// from a table of T bytes (64 MiB: L2 misses served by the Infinity Cache; 4 GiB: past it, HBM).
// Printed per case: the algorithmic bytes and the time (HIP events).  Under rocprofv3 --pmc the per-
// dispatch counters give FETCH_SIZE (and TCC_EA0_RDREQ_*) for the same launches; tools/gather_calib.py
// joins them into profiles/r03_gather_calibration.json.
//
// build: hipcc -O3 --offload-arch=gfx950 -o tools/gather_calib tools/gather_calib.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                 \
    }                                                                               \
  } while (0)

__device__ __forceinline__ uint64_t mix64(uint64_t z) {  // splitmix64 finaliser
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void fill_kernel(uint4* t, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint64_t h = mix64(i);
    t[i] = make_uint4((uint32_t)h, (uint32_t)(h >> 32), (uint32_t)(h * 3), (uint32_t)(h * 5));
  }
}

// each lane: `iters` random whole records of R bytes (R / 16 loads of 16 B), XOR-folded; one dword out
template <int R>
__global__ __launch_bounds__(256) void rec_kernel(const uint4* __restrict__ t, uint64_t n_rec, int iters,
                                                  uint32_t* out) {
  constexpr int L = R / 16;
  const uint64_t gid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint32_t acc = 0;
  uint64_t h = gid * 0x9E3779B97F4A7C15ull + 0x5EED;
  for (int it = 0; it < iters; ++it) {
    h = mix64(h + it);
    const uint64_t idx = __umul64hi(h, n_rec);  // uniform in [0, n_rec)
    const uint4* p = t + idx * L;
    uint4 v[L];
#pragma unroll
    for (int k = 0; k < L; ++k) v[k] = p[k];
#pragma unroll
    for (int k = 0; k < L; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
  }
  out[gid] = acc;
}

// 48-B records at a 48-B stride (the device triangle record: three dwordx4 loads)
__global__ __launch_bounds__(256) void rec48_kernel(const uint4* __restrict__ t, uint64_t n_rec, int iters,
                                                    uint32_t* out) {
  const uint64_t gid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint32_t acc = 0;
  uint64_t h = gid * 0x9E3779B97F4A7C15ull + 0x5EED;
  for (int it = 0; it < iters; ++it) {
    h = mix64(h + it);
    const uint64_t idx = __umul64hi(h, n_rec);
    const uint4* p = t + idx * 3;
    const uint4 a = p[0], b = p[1], c = p[2];
    acc ^= a.x ^ a.w ^ b.y ^ b.z ^ c.x ^ c.w;
  }
  out[gid] = acc;
}

// 16 B per lane, the whole table once (grid-stride, coalesced)
__global__ __launch_bounds__(256) void stream_kernel(const uint4* __restrict__ t, size_t n, uint32_t* out) {
  const size_t gid = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  uint32_t acc = 0;
  for (size_t i = gid; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = t[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  out[gid] = acc;
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 3;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const int block = 256, blocks = cus * 16;  // 16 waves per CU
  const size_t lanes = (size_t)blocks * block;
  const size_t sizes[2] = {64ull << 20, 4ull << 30};
  uint4* tab = nullptr;
  uint32_t* out = nullptr;
  CK(hipMalloc(&tab, sizes[1]));
  CK(hipMalloc(&out, lanes * sizeof(uint32_t)));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::printf("# case table_bytes rep algorithmic_read_bytes write_bytes ms GBps\n");
  for (size_t T : sizes) {
    hipLaunchKernelGGL(fill_kernel, dim3(blocks), dim3(block), 0, 0, tab, T / 16);
    CK(hipDeviceSynchronize());
    struct Case { const char* name; int rec; };
    const Case cases[] = {{"stream", 0}, {"rec32", 32}, {"rec48", 48}, {"rec64", 64}, {"rec128", 128}};
    for (const Case& cs : cases) {
      for (int r = 0; r < reps; ++r) {
        // about 1 GiB of algorithmic reads per launch (the 64-MiB table is read ~16 times over)
        const int iters = cs.rec ? (int)((1ull << 30) / (lanes * (size_t)cs.rec)) : 0;
        size_t bytes = 0;
        CK(hipEventRecord(e0));
        if (cs.rec == 0) {
          hipLaunchKernelGGL(stream_kernel, dim3(blocks), dim3(block), 0, 0, tab, T / 16, out);
          bytes = T;
        } else if (cs.rec == 48) {
          hipLaunchKernelGGL(rec48_kernel, dim3(blocks), dim3(block), 0, 0, tab, (uint64_t)(T / 48), iters, out);
          bytes = lanes * (size_t)iters * 48;
        } else {
          const uint64_t n_rec = T / cs.rec;
          if (cs.rec == 32) hipLaunchKernelGGL(rec_kernel<32>, dim3(blocks), dim3(block), 0, 0, tab, n_rec, iters, out);
          if (cs.rec == 64) hipLaunchKernelGGL(rec_kernel<64>, dim3(blocks), dim3(block), 0, 0, tab, n_rec, iters, out);
          if (cs.rec == 128) hipLaunchKernelGGL(rec_kernel<128>, dim3(blocks), dim3(block), 0, 0, tab, n_rec, iters, out);
          bytes = lanes * (size_t)iters * cs.rec;
        }
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0.0f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("%s %zu %d %zu %zu %.4f %.1f\n", cs.name, T, r, bytes, lanes * sizeof(uint32_t), ms,
                    bytes / (ms * 1e-3) / 1e9);
        std::fflush(stdout);
      }
    }
  }
  CK(hipFree(tab));
  CK(hipFree(out));
  return 0;
}
