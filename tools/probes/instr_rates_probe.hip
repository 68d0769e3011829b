// instr_rates_probe.hip -- issue cost of single VALU instruction kinds on
// gfx950 (DESIGN EVIDENCE): 8 independent instructions of one kind per loop
// iteration (inline asm, read-modify-write of 8 registers), full chip at 8
// waves per SIMD; cycles per instruction per SIMD at 2.4 GHz.
#include <hip/hip_runtime.h>

#include <cstdio>

#define R8(INS)                                                            \
  asm volatile(INS(0) INS(1) INS(2) INS(3) INS(4) INS(5) INS(6) INS(7)     \
               : "+v"(h[0]), "+v"(h[1]), "+v"(h[2]), "+v"(h[3]), "+v"(h[4]), \
                 "+v"(h[5]), "+v"(h[6]), "+v"(h[7])                        \
               : "v"(x), "v"(y))
#define R8P(INS)                                                           \
  asm volatile(INS(0) INS(1) INS(2) INS(3) INS(4) INS(5) INS(6) INS(7)     \
               : "+v"(d[0]), "+v"(d[1]), "+v"(d[2]), "+v"(d[3]), "+v"(d[4]), \
                 "+v"(d[5]), "+v"(d[6]), "+v"(d[7])                        \
               : "v"(dx), "v"(dy))

#define CVT_PK(i) "v_cvt_pk_f16_f32 %" #i ", %8, %9\n"
#define MIXLO(i) "v_fma_mixlo_f16 %" #i ", %8, -1.0, %9 op_sel_hi:[1,0,0]\n"
#define MIXLO32(i) "v_fma_mixlo_f16 %" #i ", %8, %9, %9\n"
#define MIX32(i) "v_fma_mix_f32 %" #i ", %8, -1.0, %9 op_sel_hi:[1,0,0]\n"
#define CVT32(i) "v_cvt_f32_f16 %" #i ", %8\n"
#define CVT32H(i) "v_cvt_f32_f16_sdwa %" #i ", %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1\n"
#define SUB(i) "v_sub_f32 %" #i ", %8, %9\n"
#define FMA(i) "v_fma_f32 %" #i ", %8, %9, %" #i "\n"
#define PKADD(i) "v_pk_add_f32 %" #i ", %8, %9\n"
#define PKFMA(i) "v_pk_fma_f32 %" #i ", %8, %9, %" #i "\n"
#define PKFMAH(i) "v_pk_fma_f16 %" #i ", %8, %9, %" #i "\n"
#define PERM(i) "v_perm_b32 %" #i ", %8, %9, %" #i "\n"
#define MADMIX(i) "v_fma_mixlo_f16 %" #i ", %8, %9, %" #i " op_sel_hi:[0,0,1]\n"
#define CVTPKRTZ(i) "v_cvt_pkrtz_f16_f32 %" #i ", %8, %9\n"
#define SIN(i) "v_sin_f32 %" #i ", %" #i "\n"
#define COS(i) "v_cos_f32 %" #i ", %" #i "\n"
#define RNDNE(i) "v_rndne_f32 %" #i ", %" #i "\n"
#define PKMUL(i) "v_pk_mul_f32 %" #i ", %8, %9\n"
#define MOV(i) "v_mov_b32 %" #i ", %8\n"
#define XORL(i) "v_xor_b32 %" #i ", 0x808080, %" #i "\n"
#define XORV(i) "v_xor_b32 %" #i ", %8, %" #i "\n"
#define ADDF(i) "v_add_f32 %" #i ", %8, %" #i "\n"
#define DOT2C(i) "v_dot2c_f32_f16 %" #i ", %8, %9\n"
#define DOT2(i) "v_dot2_f32_f16 %" #i ", %8, %9, %" #i "\n"
#define CVTPK_DEP(i) "v_cvt_pk_f16_f32 %" #i ", %" #i ", %9\n"

template <int K>
__global__ void __launch_bounds__(256) rate(float *out, int iters) {
  unsigned h[8];
  double d[8];
  const unsigned x = 0x3c003c01u + threadIdx.x, y = 0x3f800000u + threadIdx.x;
  const double dx = 1.0 + threadIdx.x, dy = 2.0;
  for (int i = 0; i < 8; ++i) {
    h[i] = 0x3c003c00u + i;
    d[i] = i * 0.5;
  }
  for (int it = 0; it < iters; ++it) {
    if (K == 0) R8(CVT_PK);
    if (K == 1) R8(MIXLO);
    if (K == 2) R8(MIXLO32);
    if (K == 3) R8(MIX32);
    if (K == 4) R8(CVT32);
    if (K == 5) R8(CVT32H);
    if (K == 6) R8(SUB);
    if (K == 7) R8(FMA);
    if (K == 8) R8P(PKADD);
    if (K == 9) R8P(PKFMA);
    if (K == 10) R8(PKFMAH);
    if (K == 11) R8(PERM);
    if (K == 12) R8(MADMIX);
    if (K == 13) R8(CVTPKRTZ);
    if (K == 14) R8(SIN);
    if (K == 15) R8(COS);
    if (K == 16) R8(RNDNE);
    if (K == 17) R8P(PKMUL);
    if (K == 18) R8(MOV);
    if (K == 19) R8(XORL);
    if (K == 20) R8(XORV);
    if (K == 21) R8(ADDF);
    if (K == 22) R8(DOT2C);
    if (K == 23) R8(DOT2);
  }
  float r = 0;
  for (int i = 0; i < 8; ++i) r += __uint_as_float(h[i]) + (float)d[i];
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
  const double cyc = ms * 1e-3 * 2.4e9 / (iters * 8.0);
  std::printf("%-36s %7.3f ms %6.2f cyc/instr\n", name, ms, cyc / 8);
}

int main() {
  float *out;
  (void)hipMalloc(&out, 256 * 8 * 256 * sizeof(float));
  run<0>("v_cvt_pk_f16_f32", out);
  run<13>("v_cvt_pkrtz_f16_f32", out);
  run<1>("v_fma_mixlo_f16 (f16,-1,f32)", out);
  run<2>("v_fma_mixlo_f16 (all f32 srcs)", out);
  run<12>("v_fma_mixlo_f16 (f32,f32,f16 src2)", out);
  run<3>("v_fma_mix_f32 (f16,-1,f32)", out);
  run<4>("v_cvt_f32_f16", out);
  run<5>("v_cvt_f32_f16 op_sel (high half)", out);
  run<6>("v_sub_f32", out);
  run<7>("v_fma_f32", out);
  run<8>("v_pk_add_f32", out);
  run<9>("v_pk_fma_f32", out);
  run<10>("v_pk_fma_f16", out);
  run<11>("v_perm_b32", out);
  run<14>("v_sin_f32", out);
  run<15>("v_cos_f32", out);
  run<16>("v_rndne_f32", out);
  run<17>("v_pk_mul_f32", out);
  run<18>("v_mov_b32", out);
  run<19>("v_xor_b32 (32-bit literal)", out);
  run<20>("v_xor_b32 (VGPR)", out);
  run<21>("v_add_f32", out);
  run<22>("v_dot2c_f32_f16 (VOP2)", out);
  run<23>("v_dot2_f32_f16 (VOP3P)", out);
  (void)hipDeviceSynchronize();
  return 0;
}
