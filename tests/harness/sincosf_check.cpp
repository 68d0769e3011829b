// sincosf_check.cpp -- TEST INFRASTRUCTURE: checks the restated glibc sincosf
// (ska-sdp-idg-bench_amd/csrc/common/sincosf_glibc.hpp, the phasor of the
// sequential kernels) against the host's own glibc sincosf, which is what the
// reference's CPU path calls (app/CPU/kernels/gridder_reference.cpp:72).
//
//   sincosf_check LO HI STRIDE
// walks the float bit patterns LO, LO + STRIDE, ... < HI (non-negative floats)
// and for each y checks
//   * idg::sincosf_glibc(+-y) == glibc sincosf(+-y), bit for bit;
//   * sincosf(-y) == (-sin(y), cos(y)) bit for bit -- the mirror-pixel
//     symmetry the sequential gridder relies on.
// Prints one line "checked N mismatch M asym A" and exits 1 on any failure.
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <cstdint>

#include "common/sincosf_glibc.hpp"

static uint32_t bits_of(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return u;
}

static float float_of(uint32_t u) {
  float f;
  memcpy(&f, &u, 4);
  return f;
}

int main(int argc, char **argv) {
  if (argc != 4) {
    fprintf(stderr, "usage: %s LO HI STRIDE (float bit patterns)\n", argv[0]);
    return 2;
  }
  const uint64_t lo = strtoull(argv[1], nullptr, 0);
  const uint64_t hi = strtoull(argv[2], nullptr, 0);
  const uint64_t stride = strtoull(argv[3], nullptr, 0);
  long long checked = 0, mismatch = 0, asym = 0;
#pragma omp parallel for reduction(+ : checked, mismatch, asym) \
    schedule(static, 65536)
  for (long long k = 0; k < (long long)((hi - lo + stride - 1) / stride); k++) {
    const float y = float_of((uint32_t)(lo + (uint64_t)k * stride));
    for (int sg = 0; sg < 2; sg++) {
      const float x = sg ? -y : y;
      float s0, c0, s1, c1;
      sincosf(x, &s0, &c0);
      idg::sincosf_glibc(x, &s1, &c1);
      checked++;
      if (bits_of(s0) != bits_of(s1) || bits_of(c0) != bits_of(c1)) {
        if (mismatch < 5)
          fprintf(stderr, "mismatch y=%a: glibc (%a, %a) ours (%a, %a)\n", x,
                  s0, c0, s1, c1);
        mismatch++;
      }
    }
    float sp, cp, sn, cn;
    sincosf(y, &sp, &cp);
    sincosf(-y, &sn, &cn);
    if (bits_of(sn) != bits_of(-sp) || bits_of(cn) != bits_of(cp)) asym++;
  }
  printf("checked %lld mismatch %lld asym %lld\n", checked, mismatch, asym);
  return (mismatch || asym) ? 1 : 0;
}
