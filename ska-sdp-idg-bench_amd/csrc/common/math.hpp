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

// a * b as GCC compiled the reference's std::complex<float> products: the
// real part always fma(ar, br, -(ai*bi)); the imaginary part keeps one of the
// two products in the FMA, chosen per expression (oracle/idg_oracle.c header:
// each site pinned bit for bit against the reference's own outputs).
IDG_HD inline cfloat cmul(cfloat a, cfloat b) {  // form a
  return {fmaf(a.re, b.re, -(a.im * b.im)), fmaf(a.re, b.im, a.im * b.re)};
}

IDG_HD inline cfloat cmul_b(cfloat a, cfloat b) {  // form b
  return {fmaf(a.re, b.re, -(a.im * b.im)), fmaf(a.im, b.re, a.re * b.im)};
}

IDG_HD inline cfloat cadd(cfloat a, cfloat b) {
  return {a.re + b.re, a.im + b.im};
}

IDG_HD inline cfloat cconj(cfloat a) { return {a.re, -a.im}; }

// c = a * b for 2x2 matrices stored {xx, xy, yx, yy}, in the order of
// math.hpp:26-37 (products of c[0..3], then the second term of each added);
// rows 0-1 use the complex-product form B_TOP, rows 2-3 B_BOTTOM.
template <bool B_TOP, bool B_BOTTOM>
IDG_HD inline void jones_mul_f(const cfloat *a, const cfloat *b, cfloat *c) {
  auto mt = [](cfloat x, cfloat y) { return B_TOP ? cmul_b(x, y) : cmul(x, y); };
  auto mb = [](cfloat x, cfloat y) {
    return B_BOTTOM ? cmul_b(x, y) : cmul(x, y);
  };
  c[0] = cadd(mt(a[0], b[0]), mt(a[1], b[2]));
  c[1] = cadd(mt(a[0], b[1]), mt(a[1], b[3]));
  c[2] = cadd(mb(a[2], b[0]), mb(a[3], b[2]));
  c[3] = cadd(mb(a[2], b[1]), mb(a[3], b[3]));
}

IDG_HD inline void jones_mul(const cfloat *a, const cfloat *b, cfloat *c) {
  jones_mul_f<false, false>(a, b, c);
}

IDG_HD inline void jones_hermitian(const cfloat *a, cfloat *h) {
  h[0] = cconj(a[0]);
  h[1] = cconj(a[2]);
  h[2] = cconj(a[1]);
  h[3] = cconj(a[3]);
}

// Gridder: pixels <- A1^H * pixels * A2, with the reference build's product
// forms (A1^H P: rows 0-1 form a, rows 2-3 form b; (A1^H P) A2: form b).
IDG_HD inline void apply_aterm_gridder(cfloat *pixels, const cfloat *a1,
                                       const cfloat *a2) {
  cfloat a1h[4], tmp[4];
  jones_hermitian(a1, a1h);
  jones_mul_f<false, true>(a1h, pixels, tmp);
  jones_mul_f<true, true>(tmp, a2, pixels);
}

// Degridder: pixels <- A1 * pixels * A2^H (A1 P: form a; (A1 P) A2^H: b).
IDG_HD inline void apply_aterm_degridder(cfloat *pixels, const cfloat *a1,
                                         const cfloat *a2) {
  cfloat a2h[4], tmp[4];
  jones_mul_f<false, false>(a1, pixels, tmp);
  jones_hermitian(a2, a2h);
  jones_mul_f<true, true>(tmp, a2h, pixels);
}

}  // namespace idg
