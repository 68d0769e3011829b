// test_util.hpp -- the harness' parity metric.
//
// TEST INFRASTRUCTURE.  Restates check_error of the reference's
// tests/test_util.hpp:28-92 (A = device result, B = CPU reference):
//   r_max = max(1, max|Re A|), i_max = max(1, max|Im A|)
//   over entries with |B| > 0:  r_err += dRe^2 / r_max,  i_err += dIm^2 / i_max
//   error = sqrt(r_err/nnz + i_err/nnz);  PASS iff error <= 1e-5
// and prints the same ">>> Result PASSED|FAILED" / ">>> Error: x" lines.
// Unlike the reference it also returns the verdict, so the executables can
// exit non-zero on FAILED (the reference always exits 0,
// tests/gridder_common.cpp:133-134).
#pragma once

#include <cmath>
#include <complex>
#include <cstdio>
#include <cstdlib>
#include <iostream>

#include "lib-common.hpp"

constexpr double kParityTolerance = 1e-5;

inline bool check_error(size_t n, const std::complex<float> *A,
                        const std::complex<float> *B) {
  const bool print = std::getenv("IDG_QUIET") == nullptr;
  float r_max = 1.0f, i_max = 1.0f;
  for (size_t i = 0; i < n; ++i) {
    r_max = std::max(r_max, std::fabs(A[i].real()));
    i_max = std::max(i_max, std::fabs(A[i].imag()));
  }
  double r_err = 0.0, i_err = 0.0;
  size_t nnz = 0;
  int shown = 0;
  for (size_t i = 0; i < n; ++i) {
    const double dr = static_cast<double>(B[i].real() - A[i].real());
    const double di = static_cast<double>(B[i].imag() - A[i].imag());
    if (std::abs(B[i]) > 0.0f) {
      if (print && shown < 64 && (std::fabs(dr) > 1e-4 || std::fabs(di) > 1e-4)) {
        std::printf("%zu: (%f, %f) - (%f, %f) = (%f, %f)\n", i, A[i].real(),
                    A[i].imag(), B[i].real(), B[i].imag(), dr, di);
        ++shown;
      }
      ++nnz;
      r_err += dr * dr / r_max;
      i_err += di * di / i_max;
    }
  }
  const double d = static_cast<double>(std::max<size_t>(1, nnz));
  const double error = std::sqrt(r_err / d + i_err / d);
  const bool pass = !(error > kParityTolerance);
  std::cout << (pass ? ">>> Result PASSED" : ">>> Result FAILED") << std::endl;
  std::cout << ">>> Error: " << error << std::endl;
  return pass;
}

inline bool compare_visibilities(
    idg::Array3D<idg::Visibility<std::complex<float>>> &cpu,
    idg::Array3D<idg::Visibility<std::complex<float>>> &gpu) {
  return check_error(cpu.size() * 4,
                     reinterpret_cast<std::complex<float> *>(gpu.data()),
                     reinterpret_cast<std::complex<float> *>(cpu.data()));
}

inline bool compare_subgrids(idg::Array4D<std::complex<float>> &cpu,
                             idg::Array4D<std::complex<float>> &gpu) {
  return check_error(cpu.size(), gpu.data(), cpu.data());
}
