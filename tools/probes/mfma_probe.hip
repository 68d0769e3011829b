// mfma_probe.hip -- verifies the v_mfma_f32_16x16x32_f16 operand / result
// lane maps and the accuracy of the two-term f16 split used by the MFMA
// gridder/degridder (DESIGN EVIDENCE).
//
// (1) integer A (16x32) and asymmetric B (32x16): D must equal A*B exactly
//     with lane l holding A[l&15][8(l>>4)+j], B[8(l>>4)+j][l&15], and
//     D[row=(l>>4)*4+r][col=l&15];
// (2) float A in [-1,1], B ~ N(0,1): A split a = ah + al (f16 pair via
//     v_cvt_pk_f16_f32 + v_fma_mix{lo,hi}_f16), B split into columns
//     [b_hi | b_lo], K stacked as [ah, al] x [B; B]; error vs fp64 GEMM.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#include "hip/kernels/mfma.hpp"

using namespace idg_mi355x;

__global__ void layout(const float *A, const float *B, float *D) {
  const int l = threadIdx.x;
  half8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = (_Float16)A[(l & 15) * 32 + 8 * (l >> 4) + j];
    b[j] = (_Float16)B[(8 * (l >> 4) + j) * 16 + (l & 15)];
  }
  floatx4 d = {0, 0, 0, 0};
  d = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, d, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[((l >> 4) * 4 + r) * 16 + (l & 15)] = d[r];
}

// A: 16 x 16 floats (K = 16 items); B: 16 x 8 floats.  O = A * B (16 x 8).
__global__ void split_gemm(const float *A, const float *B, float *O) {
  const int l = threadIdx.x;
  const int row = l & 15, g = l >> 4, col = l & 15;
  // lane group g covers items 4g .. 4g+3; K slots per item: (hi, lo)
  floatx4 acc = {0, 0, 0, 0};
  // one MFMA: K = 32 = 16 items x {hi, lo}: lane holds items 4g..4g+3
  half8 a, b;
  for (int q = 0; q < 4; ++q) {
    const int item = 4 * g + q;
    const half2 hl = split_f16(A[row * 16 + item]);
    a[2 * q] = hl.x;       // hi
    a[2 * q + 1] = hl.y;   // lo
    const float bv = B[item * 8 + (col & 7)];
    const half2 bs = split_f16(bv);
    const _Float16 part = col < 8 ? bs.x : bs.y;
    b[2 * q] = part;       // multiplies a_hi
    b[2 * q + 1] = part;   // multiplies a_lo
  }
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc, 0, 0, 0);
  for (int r = 0; r < 4; ++r) O[(g * 4 + r) * 16 + col] = acc[r];
}

int main() {
  std::vector<float> A(16 * 32), B(32 * 16), D(256);
  for (int i = 0; i < 16; ++i)
    for (int k = 0; k < 32; ++k) A[i * 32 + k] = float((i + 1) * (k % 7 + 1) % 23 - 11);
  for (int k = 0; k < 32; ++k)
    for (int j = 0; j < 16; ++j) B[k * 16 + j] = float((k + 2 * j + k * j) % 9 - 4);
  float *dA, *dB, *dD;
  (void)hipMalloc(&dA, 4096);
  (void)hipMalloc(&dB, 4096);
  (void)hipMalloc(&dD, 4096);
  (void)hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(layout, dim3(1), dim3(64), 0, 0, dA, dB, dD);
  (void)hipMemcpy(D.data(), dD, 1024, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      double ref = 0;
      for (int k = 0; k < 32; ++k) ref += A[i * 32 + k] * B[k * 16 + j];
      bad += ref != D[i * 16 + j];
    }
  std::printf("layout: %d of 256 mismatches\n", bad);

  std::mt19937 rng(7);
  std::uniform_real_distribution<float> u(-1, 1);
  std::normal_distribution<float> nrm(0, 1);
  std::vector<float> A2(16 * 16), B2(16 * 8), O(256);
  double maxrel = 0;
  for (int trial = 0; trial < 200; ++trial) {
    for (auto &x : A2) x = u(rng);
    for (auto &x : B2) x = nrm(rng);
    (void)hipMemcpy(dA, A2.data(), A2.size() * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(dB, B2.data(), B2.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(split_gemm, dim3(1), dim3(64), 0, 0, dA, dB, dD);
    (void)hipMemcpy(O.data(), dD, 1024, hipMemcpyDeviceToHost);
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 8; ++j) {
        double ref = 0, mag = 0;
        for (int k = 0; k < 16; ++k) {
          ref += double(A2[i * 16 + k]) * B2[k * 8 + j];
          mag += std::fabs(double(A2[i * 16 + k]) * B2[k * 8 + j]);
        }
        const double got = double(O[i * 16 + j]) + O[i * 16 + 8 + j];
        maxrel = std::max(maxrel, std::fabs(got - ref) / mag);
      }
  }
  std::printf("split f16 GEMM: max |err| / sum|a*b| = %.3e (fp32 eps 5.96e-08)\n",
              maxrel);
  return bad != 0;
}
