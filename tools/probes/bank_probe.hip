// bank_probe.hip -- VGPR bank sensitivity of VALU issue on gfx950 (DESIGN
// EVIDENCE): the same instruction with its two VGPR sources in the same
// bank (register numbers equal mod 4) or in different banks, 8 waves/SIMD.
#include <hip/hip_runtime.h>

#include <cstdio>

template <int K>
__global__ void __launch_bounds__(256) rate(float *out, int iters) {
  float r = threadIdx.x * 1e-3f;
  for (int it = 0; it < iters; ++it) {
    if (K == 0)  // cvt_pk, sources v40/v44 (same bank)
      asm volatile(
          "v_cvt_pk_f16_f32 v60, v40, v44\n v_cvt_pk_f16_f32 v61, v41, v45\n"
          "v_cvt_pk_f16_f32 v62, v42, v46\n v_cvt_pk_f16_f32 v63, v43, v47\n"
          "v_cvt_pk_f16_f32 v64, v40, v48\n v_cvt_pk_f16_f32 v65, v41, v49\n"
          "v_cvt_pk_f16_f32 v66, v42, v50\n v_cvt_pk_f16_f32 v67, v43, v51\n"
          ::: "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48",
          "v49", "v50", "v51", "v60", "v61", "v62", "v63", "v64", "v65", "v66",
          "v67");
    if (K == 1)  // cvt_pk, sources in different banks
      asm volatile(
          "v_cvt_pk_f16_f32 v60, v40, v45\n v_cvt_pk_f16_f32 v61, v41, v46\n"
          "v_cvt_pk_f16_f32 v62, v42, v47\n v_cvt_pk_f16_f32 v63, v43, v44\n"
          "v_cvt_pk_f16_f32 v64, v40, v49\n v_cvt_pk_f16_f32 v65, v41, v50\n"
          "v_cvt_pk_f16_f32 v66, v42, v51\n v_cvt_pk_f16_f32 v67, v43, v48\n"
          ::: "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48",
          "v49", "v50", "v51", "v60", "v61", "v62", "v63", "v64", "v65", "v66",
          "v67");
    if (K == 2)  // fma_mix_f32 same bank (src0 v60, src2 v44)
      asm volatile(
          "v_fma_mix_f32 v70, v60, -1.0, v40 op_sel_hi:[1,0,0]\n"
          "v_fma_mix_f32 v71, v61, -1.0, v41 op_sel_hi:[1,0,0]\n"
          "v_fma_mix_f32 v72, v62, -1.0, v42 op_sel_hi:[1,0,0]\n"
          "v_fma_mix_f32 v73, v63, -1.0, v43 op_sel_hi:[1,0,0]\n"
          "v_fma_mix_f32 v74, v64, -1.0, v44 op_sel_hi:[1,0,0]\n"
          "v_fma_mix_f32 v75, v65, -1.0, v45 op_sel_hi:[1,0,0]\n"
          "v_fma_mix_f32 v76, v66, -1.0, v46 op_sel_hi:[1,0,0]\n"
          "v_fma_mix_f32 v77, v67, -1.0, v47 op_sel_hi:[1,0,0]\n"
          ::: "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v60",
          "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v70", "v71", "v72",
          "v73", "v74", "v75", "v76", "v77");
    if (K == 3)  // fma_mix_f32 different banks
      asm volatile(
          "v_fma_mix_f32 v70, v60, -1.0, v41 op_sel_hi:[1,0,0]\n"
          "v_fma_mix_f32 v71, v61, -1.0, v42 op_sel_hi:[1,0,0]\n"
          "v_fma_mix_f32 v72, v62, -1.0, v43 op_sel_hi:[1,0,0]\n"
          "v_fma_mix_f32 v73, v63, -1.0, v40 op_sel_hi:[1,0,0]\n"
          "v_fma_mix_f32 v74, v64, -1.0, v45 op_sel_hi:[1,0,0]\n"
          "v_fma_mix_f32 v75, v65, -1.0, v46 op_sel_hi:[1,0,0]\n"
          "v_fma_mix_f32 v76, v66, -1.0, v47 op_sel_hi:[1,0,0]\n"
          "v_fma_mix_f32 v77, v67, -1.0, v44 op_sel_hi:[1,0,0]\n"
          ::: "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v60",
          "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v70", "v71", "v72",
          "v73", "v74", "v75", "v76", "v77");
    if (K == 4)  // v_fma_f32 3 sources same bank
      asm volatile(
          "v_fma_f32 v60, v40, v44, v48\n v_fma_f32 v61, v41, v45, v49\n"
          "v_fma_f32 v62, v42, v46, v50\n v_fma_f32 v63, v43, v47, v51\n"
          "v_fma_f32 v64, v40, v44, v48\n v_fma_f32 v65, v41, v45, v49\n"
          "v_fma_f32 v66, v42, v46, v50\n v_fma_f32 v67, v43, v47, v51\n"
          ::: "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48",
          "v49", "v50", "v51", "v60", "v61", "v62", "v63", "v64", "v65", "v66",
          "v67");
    if (K == 5)  // v_fma_f32 3 sources in 3 banks
      asm volatile(
          "v_fma_f32 v60, v40, v45, v50\n v_fma_f32 v61, v41, v46, v51\n"
          "v_fma_f32 v62, v42, v47, v48\n v_fma_f32 v63, v43, v44, v49\n"
          "v_fma_f32 v64, v40, v45, v50\n v_fma_f32 v65, v41, v46, v51\n"
          "v_fma_f32 v66, v42, v47, v48\n v_fma_f32 v67, v43, v44, v49\n"
          ::: "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48",
          "v49", "v50", "v51", "v60", "v61", "v62", "v63", "v64", "v65", "v66",
          "v67");
    r += 1.0f;
  }
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

template <int K>
void run(const char *name, float *out) {
  const int grid = 256 * 8, iters = 20000;
  hipLaunchKernelGGL(rate<K>, dim3(grid), dim3(256), 0, 0, out, 100);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, 0);
  hipLaunchKernelGGL(rate<K>, dim3(grid), dim3(256), 0, 0, out, iters);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  std::printf("%-44s %7.3f ms %6.2f cyc/instr\n", name, ms,
              ms * 1e-3 * 2.4e9 / (iters * 8.0) / 8);
}

int main() {
  float *out;
  (void)hipMalloc(&out, 256 * 8 * 256 * sizeof(float));
  run<0>("v_cvt_pk_f16_f32, sources same bank", out);
  run<1>("v_cvt_pk_f16_f32, sources 2 banks", out);
  run<2>("v_fma_mix_f32, VGPR sources same bank", out);
  run<3>("v_fma_mix_f32, VGPR sources 2 banks", out);
  run<4>("v_fma_f32, 3 sources same bank", out);
  run<5>("v_fma_f32, 3 sources 3 banks", out);
  (void)hipDeviceSynchronize();
  return 0;
}
