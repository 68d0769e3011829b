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
// [-2^13, 2^13) (tests/test_host.py, tests/harness/sincosf_check.cpp).
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
