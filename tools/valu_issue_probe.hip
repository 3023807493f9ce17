// valu_issue_probe.hip -- diagnostic: VALU issue rate on gfx950 for encodings the kernels use.
// Each lane runs 8 independent accumulator chains of one instruction form; 4 waves per SIMD
// (1024-thread blocks, one per CU) or 1 wave per SIMD.  Prints wave-instructions per SIMD per cycle
// (a single wave issues at most 1 per 4 cycles; two VALU instructions from different waves may issue in
// one quad-cycle: SQ_ACTIVE_INST_VALU2).
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/valu_issue_probe tools/valu_issue_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHAIN8(INSN)                                                                   \
  asm volatile(INSN : "+v"(a0) : "v"(x), "v"(y)); asm volatile(INSN : "+v"(a1) : "v"(x), "v"(y)); \
  asm volatile(INSN : "+v"(a2) : "v"(x), "v"(y)); asm volatile(INSN : "+v"(a3) : "v"(x), "v"(y)); \
  asm volatile(INSN : "+v"(a4) : "v"(x), "v"(y)); asm volatile(INSN : "+v"(a5) : "v"(x), "v"(y)); \
  asm volatile(INSN : "+v"(a6) : "v"(x), "v"(y)); asm volatile(INSN : "+v"(a7) : "v"(x), "v"(y));

template <int FORM>
__global__ void probe(float* out, float x, float y, int iters) {
  float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  unsigned long long m0 = 0, m1 = 0, m2 = 0, m3 = 0;  // FORM 10's compare results (SGPR pairs)
  const unsigned long long msk = __ballot(threadIdx.x & 1);  // FORM 11's select mask (an SGPR pair)
  if constexpr (FORM >= 12 && FORM <= 16) asm volatile("v_cmp_gt_f32_e32 vcc, %0, %1" ::"v"(a0), "v"(a1) : "vcc");
  for (int i = 0; i < iters; i += 4) {  // four copies of the chains per loop pass (the loop's SALU is 3 per 32 VALU)
    if constexpr (FORM == 0) { CHAIN8("v_fmac_f32_e32 %0, %1, %2") CHAIN8("v_fmac_f32_e32 %0, %1, %2") CHAIN8("v_fmac_f32_e32 %0, %1, %2") CHAIN8("v_fmac_f32_e32 %0, %1, %2") }           // VOP2
    else if constexpr (FORM == 1) { CHAIN8("v_fma_f32 %0, %1, %2, %0") CHAIN8("v_fma_f32 %0, %1, %2, %0") CHAIN8("v_fma_f32 %0, %1, %2, %0") CHAIN8("v_fma_f32 %0, %1, %2, %0") }       // VOP3, 3 VGPR sources
    else if constexpr (FORM == 2) { CHAIN8("v_mul_f32_e64 %0, %1, -%2") CHAIN8("v_mul_f32_e64 %0, %1, -%2") CHAIN8("v_mul_f32_e64 %0, %1, -%2") CHAIN8("v_mul_f32_e64 %0, %1, -%2") }      // VOP3 with a neg modifier
    else if constexpr (FORM == 3) { CHAIN8("v_mul_f32_e32 %0, %1, %2") CHAIN8("v_mul_f32_e32 %0, %1, %2") CHAIN8("v_mul_f32_e32 %0, %1, %2") CHAIN8("v_mul_f32_e32 %0, %1, %2") }       // VOP2, 2 sources
    else if constexpr (FORM == 4) { CHAIN8("v_max3_f32 %0, %1, %2, %0") CHAIN8("v_max3_f32 %0, %1, %2, %0") CHAIN8("v_max3_f32 %0, %1, %2, %0") CHAIN8("v_max3_f32 %0, %1, %2, %0") }      // VOP3 min/max3
    else if constexpr (FORM == 5) { CHAIN8("v_max_f32_e32 %0, %1, %0") CHAIN8("v_max_f32_e32 %0, %1, %0") CHAIN8("v_max_f32_e32 %0, %1, %0") CHAIN8("v_max_f32_e32 %0, %1, %0") }       // VOP2 max
    else if constexpr (FORM == 6) { CHAIN8("v_cndmask_b32_e32 %0, %1, %0, vcc") CHAIN8("v_cndmask_b32_e32 %0, %1, %0, vcc") CHAIN8("v_cndmask_b32_e32 %0, %1, %0, vcc") CHAIN8("v_cndmask_b32_e32 %0, %1, %0, vcc") }  // VOP2 select on VCC
    else if constexpr (FORM == 7) { CHAIN8("v_add_u32_e32 %0, %1, %0") CHAIN8("v_add_u32_e32 %0, %1, %0") CHAIN8("v_add_u32_e32 %0, %1, %0") CHAIN8("v_add_u32_e32 %0, %1, %0") }       // VOP2 integer add
    else if constexpr (FORM == 8) { CHAIN8("v_lshl_add_u32 %0, %1, 2, %0") CHAIN8("v_lshl_add_u32 %0, %1, 2, %0") CHAIN8("v_lshl_add_u32 %0, %1, 2, %0") CHAIN8("v_lshl_add_u32 %0, %1, 2, %0") }   // VOP3 integer
    else if constexpr (FORM == 10) {  // VOPC to an SGPR pair (the triangle tests' compares), 8 per 8 chains
#define CMP4 asm volatile("v_cmp_lt_f32_e64 %0, %1, %2" : "=s"(m0) : "v"(a0), "v"(y)); \
             asm volatile("v_cmp_lt_f32_e64 %0, %1, %2" : "=s"(m1) : "v"(a1), "v"(y)); \
             asm volatile("v_cmp_lt_f32_e64 %0, %1, %2" : "=s"(m2) : "v"(a2), "v"(y)); \
             asm volatile("v_cmp_lt_f32_e64 %0, %1, %2" : "=s"(m3) : "v"(a3), "v"(y));
      CMP4 CMP4 CMP4 CMP4 CMP4 CMP4 CMP4 CMP4
    }
    else if constexpr (FORM == 11) {
#define SEL8 asm volatile("v_cndmask_b32_e64 %0, %1, %0, %2" : "+v"(a0) : "v"(x), "s"(msk)); \
             asm volatile("v_cndmask_b32_e64 %0, %1, %0, %2" : "+v"(a1) : "v"(x), "s"(msk)); \
             asm volatile("v_cndmask_b32_e64 %0, %1, %0, %2" : "+v"(a2) : "v"(x), "s"(msk)); \
             asm volatile("v_cndmask_b32_e64 %0, %1, %0, %2" : "+v"(a3) : "v"(x), "s"(msk)); \
             asm volatile("v_cndmask_b32_e64 %0, %1, %0, %2" : "+v"(a4) : "v"(x), "s"(msk)); \
             asm volatile("v_cndmask_b32_e64 %0, %1, %0, %2" : "+v"(a5) : "v"(x), "s"(msk)); \
             asm volatile("v_cndmask_b32_e64 %0, %1, %0, %2" : "+v"(a6) : "v"(x), "s"(msk)); \
             asm volatile("v_cndmask_b32_e64 %0, %1, %0, %2" : "+v"(a7) : "v"(x), "s"(msk));
      SEL8 SEL8 SEL8 SEL8
    }
    else if constexpr (FORM == 12) { CHAIN8("v_cndmask_b32_e32 %0, %1, %0, vcc") CHAIN8("v_cndmask_b32_e32 %0, %1, %0, vcc") CHAIN8("v_cndmask_b32_e32 %0, %1, %0, vcc") CHAIN8("v_cndmask_b32_e32 %0, %1, %0, vcc") }
    else if constexpr (FORM == 13) { CHAIN8("v_cndmask_b32_e64 %0, %1, %0, vcc") CHAIN8("v_cndmask_b32_e64 %0, %1, %0, vcc") CHAIN8("v_cndmask_b32_e64 %0, %1, %0, vcc") CHAIN8("v_cndmask_b32_e64 %0, %1, %0, vcc") }
    else if constexpr (FORM == 14) { CHAIN8("v_cndmask_b32_e32 %0, 0, %0, vcc") CHAIN8("v_cndmask_b32_e32 %0, 0, %0, vcc") CHAIN8("v_cndmask_b32_e32 %0, 0, %0, vcc") CHAIN8("v_cndmask_b32_e32 %0, 0, %0, vcc") }
    else if constexpr (FORM == 15 || FORM == 16) {  // 7 FMAs and one select per 8 (the select in its own chain)
#define MIX(SEL) asm volatile("v_fmac_f32_e32 %0, %1, %2" : "+v"(a0) : "v"(x), "v"(y)); \
                 asm volatile("v_fmac_f32_e32 %0, %1, %2" : "+v"(a1) : "v"(x), "v"(y)); \
                 asm volatile("v_fmac_f32_e32 %0, %1, %2" : "+v"(a2) : "v"(x), "v"(y)); \
                 asm volatile(SEL : "+v"(a3) : "v"(x), "v"(y)); \
                 asm volatile("v_fmac_f32_e32 %0, %1, %2" : "+v"(a4) : "v"(x), "v"(y)); \
                 asm volatile("v_fmac_f32_e32 %0, %1, %2" : "+v"(a5) : "v"(x), "v"(y)); \
                 asm volatile("v_fmac_f32_e32 %0, %1, %2" : "+v"(a6) : "v"(x), "v"(y)); \
                 asm volatile("v_fmac_f32_e32 %0, %1, %2" : "+v"(a7) : "v"(x), "v"(y));
      if constexpr (FORM == 15) { MIX("v_cndmask_b32_e32 %0, %1, %0, vcc") MIX("v_cndmask_b32_e32 %0, %1, %0, vcc") MIX("v_cndmask_b32_e32 %0, %1, %0, vcc") MIX("v_cndmask_b32_e32 %0, %1, %0, vcc") }
      else { MIX("v_cndmask_b32_e64 %0, %1, %0, vcc") MIX("v_cndmask_b32_e64 %0, %1, %0, vcc") MIX("v_cndmask_b32_e64 %0, %1, %0, vcc") MIX("v_cndmask_b32_e64 %0, %1, %0, vcc") }
    }
    else if constexpr (FORM == 9) { CHAIN8("v_sub_f32_e32 %0, %1, %0") CHAIN8("v_sub_f32_e32 %0, %1, %0") CHAIN8("v_sub_f32_e32 %0, %1, %0") CHAIN8("v_sub_f32_e32 %0, %1, %0") }       // VOP2 sub
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + (float)((m0 ^ m1 ^ m2 ^ m3) & 1);
}

template <int FORM>
float run(int block, int iters, float* d, int grid = 256) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(probe<FORM>, dim3(grid), dim3(block), 0, 0, d, 1.0f, 1.0f, 16);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(probe<FORM>, dim3(grid), dim3(block), 0, 0, d, 1.0f, 1.0f, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

int main() {
  float* d;
  if (hipMalloc(&d, 512 * 1024 * sizeof(float)) != hipSuccess) return 1;
  const int iters = 20000;
  const char* names[] = {"v_fmac_f32_e32 (VOP2)", "v_fma_f32 (VOP3)", "v_mul_f32_e64 neg (VOP3)", "v_mul_f32_e32 (VOP2)",
                         "v_max3_f32 (VOP3)", "v_max_f32_e32 (VOP2)", "v_cndmask_b32_e32 (VOP2)", "v_add_u32_e32 (VOP2)",
                         "v_lshl_add_u32 (VOP3)", "v_sub_f32_e32 (VOP2)", "v_cmp_lt_f32_e64 -> SGPRs", "v_cndmask_b32_e64 SGPR mask",
                         "v_cndmask_b32_e32, vcc set", "v_cndmask_b32_e64 vcc", "v_cndmask_b32_e32 0, vcc",
                         "7 fmac + cndmask_e32 vcc", "7 fmac + cndmask_e64 vcc"};
  for (int wps : {1, 2, 4, 8}) {  // waves per SIMD: 256 threads per SIMD-wave row, 1024-thread blocks past 4
    const int block = wps <= 4 ? 256 * wps : 1024, grid = wps <= 4 ? 256 : 256 * wps / 4;
    float ms[17] = {run<0>(block, iters, d, grid), run<1>(block, iters, d, grid), run<2>(block, iters, d, grid),
                    run<3>(block, iters, d, grid), run<4>(block, iters, d, grid), run<5>(block, iters, d, grid),
                    run<6>(block, iters, d, grid), run<7>(block, iters, d, grid), run<8>(block, iters, d, grid),
                    run<9>(block, iters, d, grid), run<10>(block, iters, d, grid), run<11>(block, iters, d, grid),
                    run<12>(block, iters, d, grid), run<13>(block, iters, d, grid), run<14>(block, iters, d, grid),
                    run<15>(block, iters, d, grid), run<16>(block, iters, d, grid)};
    for (int f = 0; f < 17; ++f) {
      const double winst = (double)grid * (block / 64) * 8.0 * iters;  // wave-instructions
      const double cyc = ms[f] * 1e-3 * 2.4e9;                  // at 2.4 GHz
      printf("%d waves/SIMD  %-26s %8.3f ms  %.3f wave-instr per SIMD per cycle\n", wps, names[f], ms[f],
             winst / (1024.0 * cyc));
    }
  }
  return 0;
}
