// mfma.hpp -- f16 MFMA helpers for the gridder/degridder complex MAC.
//
// The 4-correlation complex multiply-accumulate of IDG is a genuine dense
// GEMM once the phasors are materialised: O[row][col] += sum_k A[row][k] *
// B[k][col] with A = phasors (cos/sin rows) and B = visibilities or pixels
// (8 real components).  v_mfma_f32_16x16x32_f16 does it at 16x the f32 rate;
// fp32 accuracy is kept with a two-term f16 split of both operands:
//   a = a_hi + a_lo   (a_hi = f16(a), a_lo = f16(a - a_hi), |err| ~ 2^-22|a|)
//   A' = [a_hi, a_lo] stacked along K, B' = [b; b] repeated along K,
//   B columns = [b_hi (8) | b_lo (8)], O = O[:, 0:8] + O[:, 8:16].
// (measured: tools/probes/mfma_probe.hip)
#pragma once

#include <hip/hip_runtime.h>

// A scheduling fence after each K-step's MFMAs; the
// IDG_NO_KSTEP_FENCE build is an A/B timing variant only.
#ifdef IDG_NO_KSTEP_FENCE
#define IDG_KSTEP_FENCE() ((void)0)
#else
#define IDG_KSTEP_FENCE() __builtin_amdgcn_sched_barrier(0)
#endif

namespace idg_mi355x {

typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 half2 __attribute__((ext_vector_type(2)));
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx2 __attribute__((ext_vector_type(2)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

// (hi, lo) of one float: hi = f16(x) (RNE), lo = f16(x - hi).
__device__ __forceinline__ half2 split_f16(float x) {
  const _Float16 hi = static_cast<_Float16>(x);
  const _Float16 lo = static_cast<_Float16>(x - static_cast<float>(hi));
  half2 r;
  r.x = hi;
  r.y = lo;
  return r;
}

// Splits the pair (c, s): *hi = (f16(c), f16(s)), *lo = (f16(c - hi.c),
// f16(s - hi.s)): v_cvt_pk_f16_f32, the two f32 residuals (exact) by
// v_fma_mix_f32, one more v_cvt_pk_f16_f32 (the same single rounding as an
// f16-output v_fma_mix, at full issue rate; split_oct below).
__device__ __forceinline__ void split_pair(float c, float s, unsigned *hi,
                                           unsigned *lo) {
  floatx2 v = {c, s};
  const f16x2 h = __builtin_convertvector(v, f16x2);
  const unsigned hu = __builtin_bit_cast(unsigned, h);
  float rc, rs;
  asm volatile("s_nop 0\n\tv_fma_mix_f32 %0, %2, -1.0, %3 op_sel_hi:[1,0,0]\n\t"
               "v_fma_mix_f32 %1, %2, -1.0, %4 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
               : "=&v"(rc), "=&v"(rs)
               : "v"(hu), "v"(c), "v"(s));
  *hi = hu;
  *lo = __builtin_bit_cast(unsigned,
                           __builtin_convertvector(floatx2{rc, rs}, f16x2));
}
// Four packed-f16 dwords as the 8-element MFMA operand.
__device__ __forceinline__ half8 pack4(unsigned a, unsigned b, unsigned c,
                                       unsigned d) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  u32x4 v = {a, b, c, d};
  return __builtin_bit_cast(half8, v);
}

// One f16 part of each of (a, b), packed: the hi part f16(x) where
// m = 0, the lo part f16(x - f16(x)) where m = -1 (m is per lane, so lanes
// holding B's hi columns and lanes holding its lo columns run the same
// instructions): m * f16(x) + x is exact in f32 (v_fma_mix_f32), then one
// v_cvt_pk_f16_f32 rounds both.
__device__ __forceinline__ unsigned split_part(float a, float b, float m) {
  floatx2 v = {a, b};
  const unsigned hu =
      __builtin_bit_cast(unsigned, __builtin_convertvector(v, f16x2));
  float ra, rb;
  asm volatile("v_fma_mix_f32 %0, %2, %3, %4 op_sel_hi:[1,0,0]\n\t"
               "v_fma_mix_f32 %1, %2, %3, %5 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
               : "=&v"(ra), "=&v"(rb)
               : "v"(hu), "v"(m), "v"(a), "v"(b));
  return __builtin_bit_cast(unsigned,
                            __builtin_convertvector(floatx2{ra, rb}, f16x2));
}

// hi parts (f16(a), f16(b)) packed.
__device__ __forceinline__ unsigned split_hi(float a, float b) {
  floatx2 v = {a, b};
  return __builtin_bit_cast(unsigned, __builtin_convertvector(v, f16x2));
}

// lo parts (f16(a - f16(a)), f16(b - f16(b))) packed.
__device__ __forceinline__ unsigned split_lo(float a, float b) {
  unsigned hi, lo;
  split_pair(a, b, &hi, &lo);
  return lo;
}

// Two operands' splits in one asm block (one pair of pads for both):
// *A = (hi(a0, a1), lo(a0, a1), hi(a2, a3), lo(a2, a3)), *B likewise for b.
// The lo parts are formed as f32 residuals r = x - f32(hi) with
// v_fma_mix_f32 (exact: hi is x rounded to 11 bits) and packed to f16 with
// one v_cvt_pk_f16_f32 per pair, i.e. f16(x - hi) with the same single
// rounding as a v_fma_mix{lo,hi}_f16: bit for bit the same operand, but the
// f16-output mix issues at half rate on gfx950 (8.5 vs 4.5 cycles,
// tools/probes/instr_rates_probe.hip), so 8 mix_f32 + 4 cvt_pk cost 13
// cycles less per call than 8 mixlo/hi (split_rates_probe.hip).
// Pads: `s_nop 0` first (the inputs are usually fresh v_sin/v_cos results:
// trans -> VALU forwarding needs 1 state) and `s_nop 1` last (VALU write ->
// MFMA SrcA read needs 2 states; the outputs are the next MFMAs' A operands).
__device__ __forceinline__ void split_oct(float a0, float a1, float a2,
                                          float a3, float b0, float b1,
                                          float b2, float b3, half8 *A,
                                          half8 *B) {
  unsigned h0, l0, h1, l1, h2, l2, h3, l3;
  float r0, r1, r2, r3, r4, r5, r6, r7;
  asm("s_nop 0\n\t"
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
      : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b0), "v"(b1), "v"(b2),
        "v"(b3));
  *A = pack4(h0, l0, h1, l1);
  *B = pack4(h2, l2, h3, l3);
}

__device__ __forceinline__ floatx4 mfma16(const half8 &a, const half8 &b,
                                          const floatx4 &c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// v_mfma_f32_16x16x4_f32: A[row = lane % 16][k = lane / 16] = a,
// B[k = lane / 16][col = lane % 16] = b; C as the f16 form (lane % 16 =
// column, rows 4 (lane / 16) .. +3).  Exact f32 products and sums.
__device__ __forceinline__ floatx4 mfma4(float a, float b, const floatx4 &c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

}  // namespace idg_mi355x
