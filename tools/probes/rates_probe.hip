// rates_probe.hip -- issue-rate microbenchmarks on gfx950 (DESIGN EVIDENCE).
//
// Full-chip grid (256 CUs x 8 workgroups x 256 threads), each lane runs
// `iters` iterations of a fixed instruction mix on independent registers
// (inline asm, so the compiler cannot fold or reorder it).  Prints ns per
// iteration and the implied cycles per instruction per SIMD at 2.4 GHz,
// which fixes the cost model used in DESIGN.md (v_fma vs v_pk_fma vs
// v_sin/v_cos vs their mix vs f16 MFMA beside VALU).
#include <hip/hip_runtime.h>

#include <cstdio>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

#define FMA8(a, b, c)                                                   \
  asm volatile(                                                         \
      "v_fma_f32 %0, %8, %9, %0\n v_fma_f32 %1, %8, %9, %1\n"            \
      "v_fma_f32 %2, %8, %9, %2\n v_fma_f32 %3, %8, %9, %3\n"            \
      "v_fma_f32 %4, %8, %9, %4\n v_fma_f32 %5, %8, %9, %5\n"            \
      "v_fma_f32 %6, %8, %9, %6\n v_fma_f32 %7, %8, %9, %7\n"            \
      : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]),      \
        "+v"(a[5]), "+v"(a[6]), "+v"(a[7])                               \
      : "v"(b), "v"(c))

#define SIN8(a)                                                          \
  asm volatile(                                                          \
      "v_sin_f32 %0, %0\n v_cos_f32 %1, %1\n v_sin_f32 %2, %2\n"          \
      "v_cos_f32 %3, %3\n v_sin_f32 %4, %4\n v_cos_f32 %5, %5\n"          \
      "v_sin_f32 %6, %6\n v_cos_f32 %7, %7\n"                             \
      : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]),       \
        "+v"(a[5]), "+v"(a[6]), "+v"(a[7]))

// KIND 0: 8 v_fma; 1: 4 v_pk_fma (8 FMAs); 2: 8 trans; 3: 8 fma + 2 trans
// (IDG-like 4:1); 4: 8 fma + 8 trans; 5: f16 MFMA 16x16x32 alone;
// 6: 8 fma beside one f16 MFMA; 7: 16 fma + 4 trans beside 2 MFMA
template <int KIND>
__global__ void __launch_bounds__(256) rate(float *out, int iters, float b,
                                            float c) {
  float a[8], s[8];
  for (int i = 0; i < 8; ++i) {
    a[i] = threadIdx.x * 1e-3f + i;
    s[i] = threadIdx.x * 1e-4f + i * 0.01f;
  }
  double pk[4];
  for (int i = 0; i < 4; ++i) pk[i] = a[2 * i] * 1e-3;
  half8 ha, hb;
  for (int i = 0; i < 8; ++i) {
    ha[i] = (_Float16)(threadIdx.x * 1e-3f + i);
    hb[i] = (_Float16)(i * 0.5f);
  }
  floatx4 acc = {0, 0, 0, 0}, acc2 = {0, 0, 0, 0};
  for (int it = 0; it < iters; ++it) {
    if (KIND == 0) FMA8(a, b, c);
    if (KIND == 1) {
      asm volatile(
          "v_pk_fma_f32 %0, %4, %5, %0\n v_pk_fma_f32 %1, %4, %5, %1\n"
          "v_pk_fma_f32 %2, %4, %5, %2\n v_pk_fma_f32 %3, %4, %5, %3\n"
          : "+v"(pk[0]), "+v"(pk[1]), "+v"(pk[2]), "+v"(pk[3])
          : "v"(pk[0]), "v"(pk[1]));
    }
    if (KIND == 2) SIN8(s);
    if (KIND == 3) {
      FMA8(a, b, c);
      asm volatile("v_sin_f32 %0, %0\n v_cos_f32 %1, %1\n"
                   : "+v"(s[0]), "+v"(s[1]));
    }
    if (KIND == 4) {
      FMA8(a, b, c);
      SIN8(s);
    }
    if (KIND == 5) {
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ha, hb, acc, 0, 0, 0);
      acc2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(hb, ha, acc2, 0, 0, 0);
    }
    if (KIND == 6) {
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ha, hb, acc, 0, 0, 0);
      FMA8(a, b, c);
    }
    if (KIND == 7) {
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ha, hb, acc, 0, 0, 0);
      FMA8(a, b, c);
      asm volatile("v_sin_f32 %0, %0\n v_cos_f32 %1, %1\n"
                   : "+v"(s[0]), "+v"(s[1]));
      acc2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(hb, ha, acc2, 0, 0, 0);
      FMA8(a, b, c);
      asm volatile("v_sin_f32 %0, %0\n v_cos_f32 %1, %1\n"
                   : "+v"(s[2]), "+v"(s[3]));
    }
  }
  float r = 0;
  for (int i = 0; i < 8; ++i) r += a[i] + s[i];
  for (int i = 0; i < 4; ++i) r += (float)pk[i];
  r += acc[0] + acc[1] + acc[2] + acc[3] + acc2[0] + acc2[3];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

template <int KIND>
void run(const char *name, float *out, int grid, double instr_per_iter) {
  const int iters = 20000;
  hipLaunchKernelGGL(rate<KIND>, dim3(grid), dim3(256), 0, 0, out, 100,
                     1.0001f, 1e-7f);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, 0);
  hipLaunchKernelGGL(rate<KIND>, dim3(grid), dim3(256), 0, 0, out, iters,
                     1.0001f, 1e-7f);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  // waves per SIMD = grid*4 waves / 1024 SIMDs
  const double waves_per_simd = grid * 4.0 / 1024.0;
  const double cycles = ms * 1e-3 * 2.4e9;
  const double per_iter_wave = cycles / (iters * waves_per_simd);
  std::printf("%-34s %9.3f ms  %7.2f cyc/iter/wave  %6.2f cyc/instr\n", name,
              ms, per_iter_wave, per_iter_wave / instr_per_iter);
}

int main() {
  float *out;
  const int grid = 256 * 8;
  (void)hipMalloc(&out, grid * 256 * sizeof(float));
  run<0>("8 v_fma_f32", out, grid, 8);
  run<1>("4 v_pk_fma_f32 (8 FMA)", out, grid, 4);
  run<2>("8 v_sin/v_cos", out, grid, 8);
  run<3>("8 v_fma + 2 trans", out, grid, 10);
  run<4>("8 v_fma + 8 trans", out, grid, 16);
  run<5>("2 mfma_f32_16x16x32_f16", out, grid, 2);
  run<6>("1 mfma16x16x32_f16 + 8 v_fma", out, grid, 9);
  run<7>("2 mfma + 16 v_fma + 4 trans", out, grid, 22);
  (void)hipDeviceSynchronize();
  return 0;
}
