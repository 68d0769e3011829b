// split_rates_probe.hip -- issue cost of the f16 split instructions and of
// the split + MFMA pattern of the MFMA loops (DESIGN EVIDENCE, §4.3/§5.1).
// Same harness as rates_probe.hip (inline asm on independent registers,
// full chip, 4 or 8 waves per SIMD): cycles per instruction per SIMD.
#include <hip/hip_runtime.h>

#include <cstdio>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// KIND 0: 8 v_cvt_pk_f16_f32; 1: 8 v_fma_mixlo_f16; 2: 8 v_fma_mixhi_f16;
// 3: 8 v_fma_f32 (reference); 4: split_oct pattern (4 cvt + 8 mix) with its
// pads; 5: split_oct + 2 MFMA consuming it (the loop's unit, x2 per tile
// pair); 6: 2 MFMA on constant operands + 12 independent v_fma_f32;
// 7: split_oct without pads + 2 MFMA on other registers (no dependency)
template <int KIND>
__global__ void __launch_bounds__(256) rate(float *out, int iters, float b) {
  float a[8];
  unsigned h[8];
  for (int i = 0; i < 8; ++i) {
    a[i] = threadIdx.x * 1e-3f + i * 0.1f;
    h[i] = 0x3c003c00u + i;
  }
  floatx4 acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
  half8 bf;
  for (int i = 0; i < 8; ++i) bf[i] = (_Float16)(i * 0.5f);
  u32x4 ac = {h[0], h[1], h[2], h[3]}, as = {h[4], h[5], h[6], h[7]};
  for (int it = 0; it < iters; ++it) {
    if (KIND == 0)
      asm volatile(
          "v_cvt_pk_f16_f32 %0, %8, %9\n v_cvt_pk_f16_f32 %1, %8, %9\n"
          "v_cvt_pk_f16_f32 %2, %8, %9\n v_cvt_pk_f16_f32 %3, %8, %9\n"
          "v_cvt_pk_f16_f32 %4, %8, %9\n v_cvt_pk_f16_f32 %5, %8, %9\n"
          "v_cvt_pk_f16_f32 %6, %8, %9\n v_cvt_pk_f16_f32 %7, %8, %9\n"
          : "+v"(h[0]), "+v"(h[1]), "+v"(h[2]), "+v"(h[3]), "+v"(h[4]),
            "+v"(h[5]), "+v"(h[6]), "+v"(h[7])
          : "v"(a[0]), "v"(a[1]));
    if (KIND == 1)
      asm volatile(
          "v_fma_mixlo_f16 %0, %8, -1.0, %9 op_sel_hi:[1,0,0]\n"
          "v_fma_mixlo_f16 %1, %8, -1.0, %9 op_sel_hi:[1,0,0]\n"
          "v_fma_mixlo_f16 %2, %8, -1.0, %9 op_sel_hi:[1,0,0]\n"
          "v_fma_mixlo_f16 %3, %8, -1.0, %9 op_sel_hi:[1,0,0]\n"
          "v_fma_mixlo_f16 %4, %8, -1.0, %9 op_sel_hi:[1,0,0]\n"
          "v_fma_mixlo_f16 %5, %8, -1.0, %9 op_sel_hi:[1,0,0]\n"
          "v_fma_mixlo_f16 %6, %8, -1.0, %9 op_sel_hi:[1,0,0]\n"
          "v_fma_mixlo_f16 %7, %8, -1.0, %9 op_sel_hi:[1,0,0]\n"
          : "+v"(h[0]), "+v"(h[1]), "+v"(h[2]), "+v"(h[3]), "+v"(h[4]),
            "+v"(h[5]), "+v"(h[6]), "+v"(h[7])
          : "v"(a[2]), "v"(a[3]));
    if (KIND == 2)
      asm volatile(
          "v_fma_mixhi_f16 %0, %8, -1.0, %9 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n"
          "v_fma_mixhi_f16 %1, %8, -1.0, %9 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n"
          "v_fma_mixhi_f16 %2, %8, -1.0, %9 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n"
          "v_fma_mixhi_f16 %3, %8, -1.0, %9 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n"
          "v_fma_mixhi_f16 %4, %8, -1.0, %9 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n"
          "v_fma_mixhi_f16 %5, %8, -1.0, %9 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n"
          "v_fma_mixhi_f16 %6, %8, -1.0, %9 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n"
          "v_fma_mixhi_f16 %7, %8, -1.0, %9 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n"
          : "+v"(h[0]), "+v"(h[1]), "+v"(h[2]), "+v"(h[3]), "+v"(h[4]),
            "+v"(h[5]), "+v"(h[6]), "+v"(h[7])
          : "v"(a[2]), "v"(a[3]));
    if (KIND == 3)
      asm volatile(
          "v_fma_f32 %0, %8, %9, %0\n v_fma_f32 %1, %8, %9, %1\n"
          "v_fma_f32 %2, %8, %9, %2\n v_fma_f32 %3, %8, %9, %3\n"
          "v_fma_f32 %4, %8, %9, %4\n v_fma_f32 %5, %8, %9, %5\n"
          "v_fma_f32 %6, %8, %9, %6\n v_fma_f32 %7, %8, %9, %7\n"
          : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]),
            "+v"(a[5]), "+v"(a[6]), "+v"(a[7])
          : "v"(b), "v"(b));
    if (KIND == 4 || KIND == 5 || KIND == 7) {
      unsigned h0, l0, h1, l1, h2, l2, h3, l3;
      if (KIND == 7)
        asm volatile(
            "v_cvt_pk_f16_f32 %0, %8, %9\n\t"
            "v_cvt_pk_f16_f32 %2, %10, %11\n\t"
            "v_cvt_pk_f16_f32 %4, %12, %13\n\t"
            "v_cvt_pk_f16_f32 %6, %14, %15\n\t"
            "v_fma_mixlo_f16 %1, %0, -1.0, %8 op_sel_hi:[1,0,0]\n\t"
            "v_fma_mixlo_f16 %3, %2, -1.0, %10 op_sel_hi:[1,0,0]\n\t"
            "v_fma_mixlo_f16 %5, %4, -1.0, %12 op_sel_hi:[1,0,0]\n\t"
            "v_fma_mixlo_f16 %7, %6, -1.0, %14 op_sel_hi:[1,0,0]\n\t"
            "v_fma_mixhi_f16 %1, %0, -1.0, %9 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
            "v_fma_mixhi_f16 %3, %2, -1.0, %11 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
            "v_fma_mixhi_f16 %5, %4, -1.0, %13 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
            "v_fma_mixhi_f16 %7, %6, -1.0, %15 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
            : "=&v"(h0), "=&v"(l0), "=&v"(h1), "=&v"(l1), "=&v"(h2), "=&v"(l2),
              "=&v"(h3), "=&v"(l3)
            : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]),
              "v"(a[6]), "v"(a[7]));
      else
        asm volatile(
            "s_nop 0\n\t"
            "v_cvt_pk_f16_f32 %0, %8, %9\n\t"
            "v_cvt_pk_f16_f32 %2, %10, %11\n\t"
            "v_cvt_pk_f16_f32 %4, %12, %13\n\t"
            "v_cvt_pk_f16_f32 %6, %14, %15\n\t"
            "v_fma_mixlo_f16 %1, %0, -1.0, %8 op_sel_hi:[1,0,0]\n\t"
            "v_fma_mixlo_f16 %3, %2, -1.0, %10 op_sel_hi:[1,0,0]\n\t"
            "v_fma_mixlo_f16 %5, %4, -1.0, %12 op_sel_hi:[1,0,0]\n\t"
            "v_fma_mixlo_f16 %7, %6, -1.0, %14 op_sel_hi:[1,0,0]\n\t"
            "v_fma_mixhi_f16 %1, %0, -1.0, %9 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
            "v_fma_mixhi_f16 %3, %2, -1.0, %11 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
            "v_fma_mixhi_f16 %5, %4, -1.0, %13 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
            "v_fma_mixhi_f16 %7, %6, -1.0, %15 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
            "s_nop 1"
            : "=&v"(h0), "=&v"(l0), "=&v"(h1), "=&v"(l1), "=&v"(h2), "=&v"(l2),
              "=&v"(h3), "=&v"(l3)
            : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]),
              "v"(a[6]), "v"(a[7]));
      u32x4 A = {h0, l0, h1, l1}, B = {h2, l2, h3, l3};
      if (KIND == 5) {
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(
            __builtin_bit_cast(half8, A), bf, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(
            __builtin_bit_cast(half8, B), bf, acc1, 0, 0, 0);
      } else if (KIND == 7) {
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(
            __builtin_bit_cast(half8, ac), bf, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(
            __builtin_bit_cast(half8, as), bf, acc1, 0, 0, 0);
        ac = A;  // next iteration's operands (one iteration of slack)
        as = B;
      } else {
        a[0] += __uint_as_float(h0 ^ l1) * 1e-30f;  // keep the results live
        a[1] += __uint_as_float(h2 ^ l3) * 1e-30f;
      }
    }
    if (KIND == 8 || KIND == 9) {
      unsigned h0, l0, h1, l1, h2, l2, h3, l3;
      float r0, r1, r2, r3, r4, r5, r6, r7;
      asm volatile(
          "s_nop 0\n\t"
          "v_cvt_pk_f16_f32 %0, %16, %17\n\t"
          "v_cvt_pk_f16_f32 %2, %18, %19\n\t"
          "v_cvt_pk_f16_f32 %4, %20, %21\n\t"
          "v_cvt_pk_f16_f32 %6, %22, %23\n\t"
          "v_fma_mix_f32 %8, %0, -1.0, %16 op_sel_hi:[1,0,0]\n\t"
          "v_fma_mix_f32 %9, %0, -1.0, %17 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
          "v_fma_mix_f32 %10, %2, -1.0, %18 op_sel_hi:[1,0,0]\n\t"
          "v_fma_mix_f32 %11, %2, -1.0, %19 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
          "v_fma_mix_f32 %12, %4, -1.0, %20 op_sel_hi:[1,0,0]\n\t"
          "v_fma_mix_f32 %13, %4, -1.0, %21 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
          "v_fma_mix_f32 %14, %6, -1.0, %22 op_sel_hi:[1,0,0]\n\t"
          "v_fma_mix_f32 %15, %6, -1.0, %23 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n\t"
          "v_cvt_pk_f16_f32 %1, %8, %9\n\t"
          "v_cvt_pk_f16_f32 %3, %10, %11\n\t"
          "v_cvt_pk_f16_f32 %5, %12, %13\n\t"
          "v_cvt_pk_f16_f32 %7, %14, %15\n\t"
          "s_nop 1"
          : "=&v"(h0), "=&v"(l0), "=&v"(h1), "=&v"(l1), "=&v"(h2), "=&v"(l2),
            "=&v"(h3), "=&v"(l3), "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3),
            "=&v"(r4), "=&v"(r5), "=&v"(r6), "=&v"(r7)
          : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]),
            "v"(a[6]), "v"(a[7]));
      u32x4 A = {h0, l0, h1, l1}, B = {h2, l2, h3, l3};
      if (KIND == 9) {
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(
            __builtin_bit_cast(half8, A), bf, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(
            __builtin_bit_cast(half8, B), bf, acc1, 0, 0, 0);
      } else {
        a[0] += __uint_as_float(h0 ^ l1) * 1e-30f;
        a[1] += __uint_as_float(h2 ^ l3) * 1e-30f;
      }
    }
    if (KIND == 6) {
      acc0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(
          __builtin_bit_cast(half8, ac), bf, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(
          __builtin_bit_cast(half8, as), bf, acc1, 0, 0, 0);
      asm volatile(
          "v_fma_f32 %0, %8, %9, %0\n v_fma_f32 %1, %8, %9, %1\n"
          "v_fma_f32 %2, %8, %9, %2\n v_fma_f32 %3, %8, %9, %3\n"
          "v_fma_f32 %4, %8, %9, %4\n v_fma_f32 %5, %8, %9, %5\n"
          "v_fma_f32 %6, %8, %9, %6\n v_fma_f32 %7, %8, %9, %7\n"
          "v_fma_f32 %0, %8, %9, %0\n v_fma_f32 %1, %8, %9, %1\n"
          "v_fma_f32 %2, %8, %9, %2\n v_fma_f32 %3, %8, %9, %3\n"
          : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]),
            "+v"(a[5]), "+v"(a[6]), "+v"(a[7])
          : "v"(b), "v"(b));
    }
  }
  float r = 0;
  for (int i = 0; i < 8; ++i) r += a[i] + __uint_as_float(h[i]);
  r += acc0[0] + acc0[3] + acc1[1] + acc1[2];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

template <int KIND>
void run(const char *name, float *out, int grid, double instr_per_iter) {
  const int iters = 20000;
  hipLaunchKernelGGL(rate<KIND>, dim3(grid), dim3(256), 0, 0, out, 100,
                     1.0001f);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, 0);
  hipLaunchKernelGGL(rate<KIND>, dim3(grid), dim3(256), 0, 0, out, iters,
                     1.0001f);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double waves_per_simd = grid * 4.0 / 1024.0;
  const double cyc = ms * 1e-3 * 2.4e9 / (iters * waves_per_simd);
  std::printf("%-44s w/SIMD %2.0f %8.3f ms %7.2f cyc/iter/wave %6.2f cyc/instr\n",
              name, waves_per_simd, ms, cyc, cyc / instr_per_iter);
}

int main() {
  float *out;
  (void)hipMalloc(&out, 256 * 8 * 256 * sizeof(float));
  for (int wpc : {4, 8}) {  // 4 or 8 workgroups of 4 waves per CU
    const int grid = 256 * wpc;
    run<0>("8 v_cvt_pk_f16_f32", out, grid, 8);
    run<1>("8 v_fma_mixlo_f16", out, grid, 8);
    run<2>("8 v_fma_mixhi_f16", out, grid, 8);
    run<3>("8 v_fma_f32", out, grid, 8);
    run<4>("split_oct (12 VALU + pads)", out, grid, 12);
    run<5>("split_oct + 2 dependent MFMA", out, grid, 14);
    run<6>("2 MFMA + 12 independent v_fma_f32", out, grid, 14);
    run<7>("split_oct no pads + 2 MFMA (1 iter slack)", out, grid, 14);
    run<8>("split via mix_f32 + cvt_pk (16 VALU + pads)", out, grid, 16);
    run<9>("split via mix_f32 + cvt_pk + 2 dep. MFMA", out, grid, 18);
  }
  (void)hipDeviceSynchronize();
  return 0;
}
