// seq_rates_probe.hip -- issue cost of the instruction kinds the bit-exact
// ("sequential") kernels spend their time in (DESIGN EVIDENCE, round 6):
// glibc sincosf's f64 polynomial, its Payne-Hanek integer products and the
// f64 <-> int / f32 converts.  Same method as instr_rates_probe.hip: 8
// independent instructions of one kind per loop iteration (inline asm,
// read-modify-write of 8 registers), full chip at 8 waves per SIMD; cycles
// per wave64 instruction per SIMD at 2.4 GHz.
#include <hip/hip_runtime.h>

#include <cstdio>

#define R8(INS)                                                            \
  asm volatile(INS(0) INS(1) INS(2) INS(3) INS(4) INS(5) INS(6) INS(7)     \
               : "+v"(h[0]), "+v"(h[1]), "+v"(h[2]), "+v"(h[3]), "+v"(h[4]), \
                 "+v"(h[5]), "+v"(h[6]), "+v"(h[7])                        \
               : "v"(x), "v"(y))
#define R8D(INS)                                                           \
  asm volatile(INS(0) INS(1) INS(2) INS(3) INS(4) INS(5) INS(6) INS(7)     \
               : "+v"(d[0]), "+v"(d[1]), "+v"(d[2]), "+v"(d[3]), "+v"(d[4]), \
                 "+v"(d[5]), "+v"(d[6]), "+v"(d[7])                        \
               : "v"(dx), "v"(dy))
#define R8Q(INS)                                                           \
  asm volatile(INS(0) INS(1) INS(2) INS(3) INS(4) INS(5) INS(6) INS(7)     \
               : "+v"(q[0]), "+v"(q[1]), "+v"(q[2]), "+v"(q[3]), "+v"(q[4]), \
                 "+v"(q[5]), "+v"(q[6]), "+v"(q[7])                        \
               : "v"(x), "v"(y)                                            \
               : "vcc")
// f64 result from 32-bit sources / 32-bit result from an f64 source
#define R8DX(INS)                                                          \
  asm volatile(INS(0) INS(1) INS(2) INS(3) INS(4) INS(5) INS(6) INS(7)     \
               : "+v"(d[0]), "+v"(d[1]), "+v"(d[2]), "+v"(d[3]), "+v"(d[4]), \
                 "+v"(d[5]), "+v"(d[6]), "+v"(d[7])                        \
               : "v"(x), "v"(y))
#define R8HD(INS)                                                          \
  asm volatile(INS(0) INS(1) INS(2) INS(3) INS(4) INS(5) INS(6) INS(7)     \
               : "+v"(h[0]), "+v"(h[1]), "+v"(h[2]), "+v"(h[3]), "+v"(h[4]), \
                 "+v"(h[5]), "+v"(h[6]), "+v"(h[7])                        \
               : "v"(dx), "v"(dy))

#define R8DT(INS)                                                          \
  asm volatile(INS(0) INS(1) INS(2) INS(3) INS(4) INS(5) INS(6) INS(7)     \
               : "+v"(d[0]), "+v"(d[1]), "+v"(d[2]), "+v"(d[3]), "+v"(d[4]), \
                 "+v"(d[5]), "+v"(d[6]), "+v"(d[7])                        \
               : "v"(dx), "v"(y))

#define FMA64(i) "v_fma_f64 %" #i ", %8, %9, %" #i "\n"
#define MUL64(i) "v_mul_f64 %" #i ", %8, %" #i "\n"
#define ADD64(i) "v_add_f64 %" #i ", %8, %" #i "\n"
#define CVT64I(i) "v_cvt_f64_i32 %" #i ", %8\n"
#define CVT64U(i) "v_cvt_f64_u32 %" #i ", %8\n"
#define CVT64F(i) "v_cvt_f64_f32 %" #i ", %8\n"
#define CVT32F64(i) "v_cvt_f32_f64 %" #i ", %8\n"
#define CVTI32F64(i) "v_cvt_i32_f64 %" #i ", %8\n"
#define MULLO(i) "v_mul_lo_u32 %" #i ", %8, %" #i "\n"
#define MULHI(i) "v_mul_hi_u32 %" #i ", %8, %" #i "\n"
#define MAD64(i) "v_mad_u64_u32 %" #i ", vcc, %8, %9, %" #i "\n"
#define MUL24(i) "v_mul_u32_u24 %" #i ", %8, %" #i "\n"
#define MULHI24(i) "v_mul_hi_u32_u24 %" #i ", %8, %" #i "\n"
#define CND(i) "v_cndmask_b32 %" #i ", %8, %" #i ", vcc\n"
#define BFE(i) "v_bfe_u32 %" #i ", %" #i ", %8, 3\n"
#define LSHL64(i) "v_lshlrev_b64 %" #i ", 3, %" #i "\n"
#define FMAF32(i) "v_fma_f32 %" #i ", %8, %9, %" #i "\n"
#define TRIGPRE(i) "v_trig_preop_f64 %" #i ", %8, %9\n"
#define FRACT64(i) "v_fract_f64 %" #i ", %" #i "\n"
#define LDEXP64(i) "v_ldexp_f64 %" #i ", %" #i ", %9\n"

#define PKMULF32(i) "v_pk_mul_f32 %" #i ", %8, %" #i "\n"

template <int K>
__global__ void __launch_bounds__(256) rate(float *out, int iters) {
  unsigned h[8];
  double d[8];
  unsigned long long q[8];
  const unsigned x = 0x3c003c01u + threadIdx.x, y = 0x3f800000u + threadIdx.x;
  const double dx = 1.0 + threadIdx.x, dy = 2.0;
  for (int i = 0; i < 8; ++i) {
    h[i] = 0x3c003c00u + i;
    d[i] = i * 0.5;
    q[i] = 0x123456789ull * (i + 1);
  }
  for (int it = 0; it < iters; ++it) {
    if (K == 0) R8D(FMA64);
    if (K == 1) R8D(MUL64);
    if (K == 2) R8D(ADD64);
    if (K == 3) R8DX(CVT64I);
    if (K == 4) R8DX(CVT64U);
    if (K == 5) R8DX(CVT64F);
    if (K == 6) R8HD(CVT32F64);
    if (K == 7) R8HD(CVTI32F64);
    if (K == 8) R8(MULLO);
    if (K == 9) R8(MULHI);
    if (K == 10) R8Q(MAD64);
    if (K == 11) R8(MUL24);
    if (K == 12) R8(MULHI24);
    if (K == 13) { asm volatile("s_mov_b64 vcc, -1" ::: "vcc"); R8(CND); }
    if (K == 14) R8(BFE);
    if (K == 15) R8Q(LSHL64);
    if (K == 16) R8(FMAF32);
    if (K == 17) R8D(PKMULF32);
    if (K == 18) R8DT(TRIGPRE);
    if (K == 19) R8D(FRACT64);
    if (K == 20) R8DT(LDEXP64);
  }
  float r = 0;
  for (int i = 0; i < 8; ++i)
    r += __uint_as_float(h[i]) + (float)d[i] + (float)(q[i] & 0xffff);
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
  run<16>("v_fma_f32 (reference point)", out);
  run<0>("v_fma_f64", out);
  run<1>("v_mul_f64", out);
  run<2>("v_add_f64", out);
  run<3>("v_cvt_f64_i32", out);
  run<4>("v_cvt_f64_u32", out);
  run<5>("v_cvt_f64_f32", out);
  run<6>("v_cvt_f32_f64", out);
  run<7>("v_cvt_i32_f64", out);
  run<8>("v_mul_lo_u32", out);
  run<9>("v_mul_hi_u32", out);
  run<10>("v_mad_u64_u32", out);
  run<11>("v_mul_u32_u24", out);
  run<12>("v_mul_hi_u32_u24", out);
  run<13>("v_cndmask_b32", out);
  run<14>("v_bfe_u32", out);
  run<15>("v_lshlrev_b64", out);
  run<17>("v_pk_mul_f32", out);
  run<18>("v_trig_preop_f64", out);
  run<19>("v_fract_f64", out);
  run<20>("v_ldexp_f64", out);
  (void)hipDeviceSynchronize();
  return 0;
}
