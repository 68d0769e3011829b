// math.hpp -- image-domain geometry and 2x2 Jones algebra (host + device).
//
// Semantics follow the reference's app/common/math.hpp:9-92:
//   compute_l/m : (i + 0.5 - S/2) * image_size / S, evaluated in double
//   compute_n   : tmp/(1 + sqrt(1 - tmp)), tmp = l*l + m*m, 1 if tmp > 1
//   gridder A-term   : P <- A1^H * P * A2
//   degridder A-term : P <- A1 * P * A2^H
// The multiply-add grouping is spelled with explicit fmaf() so the result
// does not depend on the compiler's contraction mode (see oracle/idg_oracle.c
// for the GCC fusion pattern of the reference build).
#pragma once

#include <cmath>

#ifndef IDG_HD
#if defined(__HIPCC__)
#define IDG_HD __host__ __device__
#else
#define IDG_HD
#endif
#endif

namespace idg {

IDG_HD inline float compute_l(int x, int subgrid_size, float image_size) {
  return static_cast<float>(
      (static_cast<double>(x) + 0.5 - static_cast<double>(subgrid_size / 2)) *
      static_cast<double>(image_size) / static_cast<double>(subgrid_size));
}

IDG_HD inline float compute_m(int y, int subgrid_size, float image_size) {
  return compute_l(y, subgrid_size, image_size);
}

IDG_HD inline float compute_n(float l, float m) {
  const float tmp = fmaf(l, l, m * m);
  return tmp > 1.0f ? 1.0f : tmp / (1.0f + sqrtf(1.0f - tmp));
}

// Complex float as a plain pair so the same code runs on host and device.
struct cfloat {
  float re, im;
};

IDG_HD inline cfloat cmul(cfloat a, cfloat b) {
  return {fmaf(a.re, b.re, -(a.im * b.im)), fmaf(a.re, b.im, a.im * b.re)};
}

IDG_HD inline cfloat cadd(cfloat a, cfloat b) {
  return {a.re + b.re, a.im + b.im};
}

IDG_HD inline cfloat cconj(cfloat a) { return {a.re, -a.im}; }

// c = a * b for 2x2 matrices stored {xx, xy, yx, yy}.
IDG_HD inline void jones_mul(const cfloat *a, const cfloat *b, cfloat *c) {
  c[0] = cadd(cmul(a[0], b[0]), cmul(a[1], b[2]));
  c[1] = cadd(cmul(a[0], b[1]), cmul(a[1], b[3]));
  c[2] = cadd(cmul(a[2], b[0]), cmul(a[3], b[2]));
  c[3] = cadd(cmul(a[2], b[1]), cmul(a[3], b[3]));
}

IDG_HD inline void jones_hermitian(const cfloat *a, cfloat *h) {
  h[0] = cconj(a[0]);
  h[1] = cconj(a[2]);
  h[2] = cconj(a[1]);
  h[3] = cconj(a[3]);
}

// Gridder: pixels <- A1^H * pixels * A2
IDG_HD inline void apply_aterm_gridder(cfloat *pixels, const cfloat *a1,
                                       const cfloat *a2) {
  cfloat a1h[4], tmp[4];
  jones_hermitian(a1, a1h);
  jones_mul(a1h, pixels, tmp);
  jones_mul(tmp, a2, pixels);
}

// Degridder: pixels <- A1 * pixels * A2^H
IDG_HD inline void apply_aterm_degridder(cfloat *pixels, const cfloat *a1,
                                         const cfloat *a2) {
  cfloat a2h[4], tmp[4];
  jones_mul(a1, pixels, tmp);
  jones_hermitian(a2, a2h);
  jones_mul(tmp, a2h, pixels);
}

}  // namespace idg
