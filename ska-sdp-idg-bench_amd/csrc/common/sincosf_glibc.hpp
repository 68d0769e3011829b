// sincosf_glibc.hpp -- the reference's phasor function, bit for bit (host +
// device).
//
// The reference's CPU gridder and degridder take the phasor as
// {cosf(phase), sinf(phase)} (app/CPU/kernels/gridder_reference.cpp:72,
// degridder_reference.cpp:106); GCC merges the pair into one call of glibc's
// sincosf (`call sincosf@plt`).  glibc is a third-party
// dependency the reference does not vendor; the build and the GPU box run
// glibc 2.35 (Ubuntu GLIBC 2.35-0ubuntu3), whose x86-64 sincosf dispatches to
// the FMA build of sysdeps/ieee754/flt-32/s_sincosf.c (Szabolcs Nagy's 2018
// algorithm) on any CPU with FMA + AVX2.  This file restates that published
// algorithm -- its three argument classes, its table of 4/pi bits and its
// polynomial coefficients, and the places where the FMA build fuses -- in
// plain double arithmetic with explicit fma(), so the GPU computes the same
// float pair the reference's CPU path does.  It is not correctly rounded
// (1.3% of phases differ from the correctly rounded sin/cos by one ulp);
// matching it is what makes the sequential kernels bit-exact.
//
//   |y| < 2^-12       sin = y, cos = 1
//   |y| < pi/4        poly(y)
//   |y| < 120         n = ((int)(y * 2^24 * 2/pi) + 2^23) >> 24,
//                     r = fma(-n, pi/2, y)                  (one rounding)
//   |y| finite        Payne-Hanek on the 24-bit mantissa with 96 bits of
//                     4/pi (three 32-bit products), r = res0 * pi / 2^62
//   poly(r)           sin: r' + r'^3 (s1 + r^2 (s2 + r^2 s3)), r' = +-r
//                     cos: c0 + r^2 c1 + r^4 c2 + r^6 (c3 + r^2 c4)
//                     with the quadrant's sign / swap; every step rounded in
//                     double, then rounded to float once.
//
// Checked against the host's own glibc sincosf over every float in
// [-2^15, 2^15) (tests/test_host.py, tests/harness/sincosf_check.cpp).
#pragma once

#include <cstdint>
#include <cstring>

#ifndef IDG_HD
#if defined(__HIPCC__)
#define IDG_HD __host__ __device__
#else
#define IDG_HD
#endif
#endif

namespace idg {

// sysdeps/ieee754/flt-32/sincosf.h: __sincosf_table[0] (c0..c4, s1..s3); the
// second table (quadrants 2 and 3) negates c0..c4 and keeps s1..s3.
constexpr double kSincosfHpiInv = 0x1.45f306dc9c883p+23;  // 2/pi * 2^24
constexpr double kSincosfHpi = 0x1.921fb54442d18p+0;      // pi/2
constexpr double kSincosfPi63 = 0x1.921fb54442d18p-62;    // pi/2 * 2^-61
constexpr double kSincosfC0 = 0x1.0p+0;
constexpr double kSincosfC1 = -0x1.ffffffd0c621cp-2;
constexpr double kSincosfC2 = 0x1.55553e1068f19p-5;
constexpr double kSincosfC3 = -0x1.6c087e89a359dp-10;
constexpr double kSincosfC4 = 0x1.99343027bf8c3p-16;
constexpr double kSincosfS1 = -0x1.555545995a603p-3;
constexpr double kSincosfS2 = 0x1.1107605230bc4p-7;
constexpr double kSincosfS3 = -0x1.994eb3774cf24p-13;

// The bits of 4/pi (hex 0.a2f9836e4e44...) as glibc's __inv_pio4 lays them
// out: entry i holds the 32 bits that start i bytes into the expansion.
#define IDG_INV_PIO4_TABLE                                                   \
  {0xa2,       0xa2f9,     0xa2f983,   0xa2f9836e, 0xf9836e4e, 0x836e4e44, \
   0x6e4e4415, 0x4e441529, 0x441529fc, 0x1529fc27, 0x29fc2757, 0xfc2757d1, \
   0x2757d1f5, 0x57d1f534, 0xd1f534dd, 0xf534ddc0, 0x34ddc0db, 0xddc0db62, \
   0xc0db6295, 0xdb629599, 0x6295993c, 0x95993c43, 0x993c4390, 0x3c439041}
#if defined(__HIPCC__)
static __constant__ const uint32_t kInvPio4Dev[24] = IDG_INV_PIO4_TABLE;
#endif

// Entry i of the table.  Every |y| in [120, 2^15) -- all phases the IDG
// kernels form -- reads i in {0, 1} (i = bits 26-29 of the float), so the
// device takes entries i, i + 4, i + 8 for those from immediates (one select
// each, sincosf_large below) and reads the constant table only otherwise.
IDG_HD inline uint32_t inv_pio4(uint32_t i) {
#if defined(__HIP_DEVICE_COMPILE__)
  return kInvPio4Dev[i];
#else
  static constexpr uint32_t t[24] = IDG_INV_PIO4_TABLE;
  return t[i];
#endif
}

IDG_HD inline double sincosf_fma(double a, double b, double c) {
  return __builtin_fma(a, b, c);
}

IDG_HD inline uint32_t sincosf_bits(float y) {
  uint32_t u;
  std::memcpy(&u, &y, sizeof u);
  return u;
}

// The polynomial pair of s_sincosf.c (sincosf_poly) as the FMA build
// evaluates it, on the reduced argument r (x2 = r * r).  glibc multiplies r by
// sign[n & 3] before the sine polynomial and takes the second table (c0..c4
// negated, s1..s3 the same) for quadrants with n & 2; every step of either
// polynomial is sign-symmetric (round to nearest even), so that is exactly
// the negation of the float result: `neg_sin` / `neg_cos` apply it there, and
// `swap` exchanges sin and cos (odd n).
IDG_HD inline void sincosf_poly(double r, double x2, bool neg_sin,
                                bool neg_cos, bool swap, float *sinp,
                                float *cosp) {
  const double x3 = x2 * r, x4 = x2 * x2;
  const double s1p = sincosf_fma(x2, kSincosfS3, kSincosfS2);
  const double c2p = sincosf_fma(x2, kSincosfC4, kSincosfC3);
  const double c1p = sincosf_fma(x2, kSincosfC1, kSincosfC0);
  const double x5 = x2 * x3, x6 = x2 * x4;
  const double s = sincosf_fma(x3, kSincosfS1, r);
  const double c = sincosf_fma(x4, kSincosfC2, c1p);
  float so = static_cast<float>(sincosf_fma(x5, s1p, s));
  float co = static_cast<float>(sincosf_fma(x6, c2p, c));
  so = neg_sin ? -so : so;
  co = neg_cos ? -co : co;
  *sinp = swap ? co : so;
  *cosp = swap ? so : co;
}

// (int64_t) res to double, rounded to nearest as cvtsi2sd does.
IDG_HD inline double sincosf_i64_to_double(int64_t res) {
#if defined(__HIP_DEVICE_COMPILE__)
  const double hi = static_cast<double>(static_cast<int32_t>(res >> 32));
  const double lo = static_cast<double>(static_cast<uint32_t>(res));
  return __builtin_fma(hi, 0x1.0p32, lo);  // exact parts, one rounding
#else
  return static_cast<double>(res);
#endif
}

// The large-argument class (120 <= |y| < inf): glibc's reduce_large, then
// the polynomials.  For |y| < 2^15 (i <= 1) the three table entries are
// selected from immediates.
IDG_HD inline void sincosf_large(uint32_t bits, float *sinp, float *cosp) {
  const uint32_t sign = bits >> 31;
  const uint32_t i = (bits >> 26) & 15;
  const uint32_t xi = ((bits & 0x7fffff) | 0x800000) << ((bits >> 23) & 7);
  uint32_t a0, a4, a8;
#if defined(__HIP_DEVICE_COMPILE__)
  if (i <= 1) {
    a0 = i ? 0xa2f9u : 0xa2u;
    a4 = i ? 0x836e4e44u : 0xf9836e4eu;
    a8 = i ? 0x1529fc27u : 0x441529fcu;
  } else {
    a0 = inv_pio4(i);
    a4 = inv_pio4(i + 4);
    a8 = inv_pio4(i + 8);
  }
#else
  a0 = inv_pio4(i);
  a4 = inv_pio4(i + 4);
  a8 = inv_pio4(i + 8);
#endif
  const uint64_t res0w = static_cast<uint32_t>(xi * a0);
  const uint64_t res1 = static_cast<uint64_t>(xi) * a4;
  const uint64_t res2 = static_cast<uint64_t>(xi) * a8;
  uint64_t res0 = (res2 >> 32) | (res0w << 32);
  res0 += res1;
  const uint64_t n = (res0 + (1ULL << 61)) >> 62;
  res0 -= n << 62;
  const double r =
      sincosf_i64_to_double(static_cast<int64_t>(res0)) * kSincosfPi63;
  const uint32_t q = static_cast<uint32_t>(n) + sign;
  // sign[q & 3] = 1, -1, -1, 1; the second table for q & 2; swap for odd n
  sincosf_poly(r, r * r, ((q + 1) & 2) != 0, (q & 2) != 0, (n & 1) != 0,
               sinp, cosp);
}

#if defined(__HIPCC__)
// ---------------------------------------------------------------------------
// The same function as the kernels evaluate it (round 6).
//
// reduce_large multiplies xi = m << sh (m the 24-bit mantissa, sh = bits
// 23-25 of the float) by A_i = a0:a4:a8, 96 bits of 4/pi picked by i = bits
// 26-29, and keeps floor(xi * A_i / 2^32) mod 2^64.  Since xi * A_i =
// m * (A_i << sh) and the bits of A_i << sh at 2^96 and above only reach
// 2^64 and above after the shift, that is floor(m * W / 2^32) mod 2^64 with
// W = (A_i << sh) mod 2^96 -- a 96-bit window that depends on bits 23-29 of
// the float alone.  For 120 <= |y| < 2^17 (biased exponent 133-143: i = 0
// or 1, every phase the IDG kernels form) that is one of 16 windows indexed
// by bits 23-26, which the kernels keep in LDS (kSincosfWindows, 256 B): one
// ds_read_b128 replaces the shift of m and the three-way table select.
struct SincosfWindow {
  uint32_t w0, w1, w2, pad;  // W = w2:w1:w0
};
constexpr SincosfWindow sincosf_window(int idx) {
  // biased exponent 128 + idx: i = idx >> 3, sh = idx & 7
  const uint32_t a0 = (idx >> 3) ? 0xa2f9u : 0xa2u;
  const uint32_t a4 = (idx >> 3) ? 0x836e4e44u : 0xf9836e4eu;
  const uint32_t a8 = (idx >> 3) ? 0x1529fc27u : 0x441529fcu;
  const int sh = idx & 7;
  return {a8 << sh, (a4 << sh) | (sh ? a8 >> (32 - sh) : 0u),
          (a0 << sh) | (sh ? a4 >> (32 - sh) : 0u), 0u};
}
constexpr int kSincosfWindows = 16;

// Fill the kernel's LDS copy (threads 0..15; the caller's barrier follows).
__device__ __forceinline__ void sincosf_windows_to_lds(SincosfWindow *lds,
                                                       int tid) {
  if (tid < kSincosfWindows) {
    uint32_t w0 = 0, w1 = 0, w2 = 0;
#pragma unroll
    for (int i = 0; i < kSincosfWindows; ++i)
      if (tid == i) {
        w0 = sincosf_window(i).w0;
        w1 = sincosf_window(i).w1;
        w2 = sincosf_window(i).w2;
      }
    lds[tid] = {w0, w1, w2, 0u};
  }
}

// res0 = floor(m * (w2:w1:w0) / 2^32) mod 2^64, reduced to the quadrant
// residue as reduce_large does: n = (res0 + 2^61) >> 62, and res0 - (n <<
// 62), whose high word is the sign-extended low 30 bits of res0's (one
// v_bfe_i32), converted to double exactly once (two exact halves, one fma)
// and scaled by pi/2^62.
__device__ __forceinline__ double sincosf_reduce_words(uint32_t m,
                                                       uint32_t w2,
                                                       uint32_t w1,
                                                       uint32_t w0,
                                                       uint32_t &n) {
  const uint32_t lo2 = m * w2;
  const uint32_t h0 = __umulhi(m, w0);
  const uint64_t res0 = static_cast<uint64_t>(m) * w1 +
                        ((static_cast<uint64_t>(lo2) << 32) | h0);
  const uint32_t hi = static_cast<uint32_t>(res0 >> 32);
  n = (hi + 0x20000000u) >> 30;
  const int32_t hr = __builtin_amdgcn_sbfe(static_cast<int32_t>(hi), 0, 30);
  return __builtin_fma(static_cast<double>(hr), 0x1.0p32,
                       static_cast<double>(static_cast<uint32_t>(res0))) *
         kSincosfPi63;
}

// glibc's sincosf with one polynomial per call: sincosf_glibc below branches
// into three tails that each end in sincosf_poly; here the reductions only
// produce (r, n, q) and the polynomial, signs and swap follow once:
//   120 <= |y| < 2^17  reduce_large through the LDS window (above),
//                      q = n + sign
//   2^17 <= |y| < inf  reduce_large through the 4/pi table (xi, A_i)
//   |y| < 120          reduce_fast: n = ((int)(y * 2^24 * 2/pi) + 2^23) >>
//                      24, r = fma(-n, pi/2, y), q = n -- which for |y| <
//                      0.75 gives n = 0 and r = y exactly, glibc's |y| < pi/4
//                      class, so that class needs no path of its own
//   |y| < 2^-12, inf, nan  the polynomial on r = y already gives glibc's
//                      (y, 1) and nan, except sin(-0) (q = 1 there)
// The two rare classes sit behind branches marked unlikely, which the
// backend then jumps over when none of a wave's lanes needs them (without
// the hint it issued the ~8-instruction |y| < 120 reduction in every wave,
// under an empty mask).
// Every arithmetic step is the one sincosf_glibc takes, so the two agree bit
// for bit (tests/harness/sincosf_gpu_check.hip checks both against the
// host's glibc over every float below 2^15 and a stride beyond).
__device__ __forceinline__ void sincosf_glibc_dev(
    float y, float *sinp, float *cosp, const SincosfWindow *__restrict__ win) {
  const uint32_t bits = __builtin_bit_cast(uint32_t, y);
  const uint32_t abits = bits & 0x7fffffffu;
  double r;
  uint32_t n, q;
  if (__builtin_expect(abits - 0x42f00000u < 0x48000000u - 0x42f00000u, 1)) {
    const SincosfWindow w = win[(bits >> 23) & 15];
    r = sincosf_reduce_words((bits & 0x7fffffu) | 0x800000u, w.w2, w.w1,
                             w.w0, n);
    q = n + (bits >> 31);
  } else if (__builtin_expect(
                 abits - 0x48000000u < 0x7f800000u - 0x48000000u, 0)) {
    const uint32_t i = (bits >> 26) & 15;
    const uint32_t xi = ((bits & 0x7fffffu) | 0x800000u) << ((bits >> 23) & 7);
    r = sincosf_reduce_words(xi, inv_pio4(i), inv_pio4(i + 4),
                             inv_pio4(i + 8), n);
    q = n + (bits >> 31);
  } else {
    const double x = static_cast<double>(y);
    const int nn =
        (static_cast<int32_t>(x * kSincosfHpiInv) + 0x800000) >> 24;
    r = __builtin_fma(-static_cast<double>(nn), kSincosfHpi, x);
    n = static_cast<uint32_t>(nn);
    // glibc returns sin(-0) = -0 (its |y| < 2^-12 class); the polynomial
    // gives +0 there, so q = 1 negates it (and nothing else: n = 0, no swap,
    // cos keeps its sign since q & 2 = 0)
    q = n | (bits == 0x80000000u ? 1u : 0u);
  }
  const double x2 = r * r;
  const double x3 = x2 * r, x4 = x2 * x2;
  const double s1p = __builtin_fma(x2, kSincosfS3, kSincosfS2);
  const double c2p = __builtin_fma(x2, kSincosfC4, kSincosfC3);
  const double c1p = __builtin_fma(x2, kSincosfC1, kSincosfC0);
  const double x5 = x2 * x3, x6 = x2 * x4;
  const double s = __builtin_fma(x3, kSincosfS1, r);
  const double c = __builtin_fma(x4, kSincosfC2, c1p);
  // glibc's sign[q & 3] (sin negated for q & 3 in {1, 2}) and second table
  // (cos negated for q & 2), as the sign bit of the float result
  const uint32_t sb =
      __builtin_bit_cast(uint32_t,
                         static_cast<float>(__builtin_fma(x5, s1p, s))) ^
      (((q + 1) << 30) & 0x80000000u);
  const uint32_t cb =
      __builtin_bit_cast(uint32_t,
                         static_cast<float>(__builtin_fma(x6, c2p, c))) ^
      ((q << 30) & 0x80000000u);
  // glibc's |y| < 2^-12 class returns (y, 1).  The polynomial on r = y
  // gives the same floats there (sin: y (1 - y^2/6), |y^2/6| < 2^-26.5, under
  // the half-ulp 2^-25 below a power of two; cos: 1 - y^2/2 with y^2/2 <
  // 2^-25, the midpoint below 1, which rounds to even 1.0) except for the
  // sign of sin(-0), which q carries (reduce_fast above).  inf / nan come
  // out nan from the polynomial, as glibc's y - y.
  *sinp = __builtin_bit_cast(float, (n & 1) ? cb : sb);
  *cosp = __builtin_bit_cast(float, (n & 1) ? sb : cb);
}
#endif

// glibc 2.35 sincosf(y, sinp, cosp).
IDG_HD inline void sincosf_glibc(float y, float *sinp, float *cosp) {
  const uint32_t bits = sincosf_bits(y);
  const uint32_t top = (bits >> 20) & 0x7ff;
  if (top > 0x42e && top < 0x7f8) {  // 120 <= |y| < inf: the common case
    sincosf_large(bits, sinp, cosp);
    return;
  }
  const double x = static_cast<double>(y);
  if (top <= 0x397) {  // |y| < 2^-12
    *sinp = y;
    *cosp = 1.0f;
  } else if (top <= 0x3f3) {  // |y| < pi/4
    sincosf_poly(x, x * x, false, false, false, sinp, cosp);
  } else if (top <= 0x42e) {  // |y| < 120
    const int n =
        (static_cast<int32_t>(x * kSincosfHpiInv) + 0x800000) >> 24;
    const double r = sincosf_fma(-static_cast<double>(n), kSincosfHpi, x);
    sincosf_poly(r, r * r, ((n + 1) & 2) != 0, (n & 2) != 0, (n & 1) != 0,
                 sinp, cosp);
  } else {  // inf / nan: nan, as glibc's y - y
    *sinp = *cosp = y - y;
  }
}

}  // namespace idg
