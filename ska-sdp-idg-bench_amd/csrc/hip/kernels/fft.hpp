// fft.hpp -- the in-register subgrid FFT pieces shared by the pipeline
// kernels (pipeline_mi355x.hip.cpp: batched FFT, fused splitter + FFT) and
// the gridder's FFT epilogue (gridder_mi355x.hip.cpp, idg_gridder_fft_launch).
// One definition, so every path that transforms a plane does the same
// operations in the same order and their outputs agree bit for bit.
#pragma once

#include <hip/hip_runtime.h>

#include "device.hpp"

namespace idg_mi355x {

// exp(sign * 2 pi i * n / d) for integers, argument reduced exactly.
__device__ __forceinline__ float2 unit_phasor(int n, int d, float sign) {
  int r = n % d;
  if (r < 0) r += d;
  const float rev = static_cast<float>(r) / static_cast<float>(d);
  return make_float2(__builtin_amdgcn_cosf(rev),
                     sign * __builtin_amdgcn_sinf(rev));
}

__device__ __forceinline__ float2 cmulf(float2 a, float2 b) {
  return make_float2(fma_(a.x, b.x, -(a.y * b.y)), fma_(a.x, b.y, a.y * b.x));
}

// Radix-2 decimation in frequency over N values in registers, fully
// unrolled: x[bit_reverse(k)] holds output k.  tw[j] = exp(sign 2 pi i j/N).
template <int N>
__device__ __forceinline__ void fft_dif_registers(float2 (&x)[N],
                                                  const float2 (&tw)[N / 2]) {
#pragma unroll
  for (int len = N; len >= 2; len >>= 1) {
    const int half = len >> 1;
    const int step = N / len;  // twiddle stride
#pragma unroll
    for (int start = 0; start < N; start += len) {
#pragma unroll
      for (int j = 0; j < half; ++j) {
        const float2 a = x[start + j], b = x[start + j + half];
        x[start + j] = make_float2(a.x + b.x, a.y + b.y);
        const float2 d = make_float2(a.x - b.x, a.y - b.y);
        x[start + j + half] = j == 0 ? d : cmulf(d, tw[j * step]);
      }
    }
  }
}

template <int N>
__device__ __forceinline__ constexpr int bit_reverse(int i) {
  int r = 0;
  for (int b = 1; b < N; b <<= 1) r = (r << 1) | ((i & b) ? 1 : 0);
  return r;
}

// The 2-D transform of P planes of N x N complex held in LDS at `planes`
// (row stride N + 1 complex, plane stride N (N + 1)), by threads
// tid < P N: thread (p = tid / N, q = tid % N) transforms row q of plane p,
// then (after a barrier every thread of the workgroup reaches) column q;
// returns the column's outputs in f (f[i] = output row bit_reverse(i),
// column q).  Rows then columns, as kernel_subgrid_fft_reg.
template <int N>
__device__ __forceinline__ void fft2_planes_lds(float2 *planes, int tid,
                                                int nthreads_active,
                                                const float2 (&tw)[N / 2],
                                                float2 (&f)[N]) {
  constexpr int RS = N + 1;
  const int p = tid / N, q = tid % N;
  const bool active = tid < nthreads_active;
  if (active) {
#pragma unroll
    for (int i = 0; i < N; ++i) f[i] = planes[p * N * RS + q * RS + i];
    fft_dif_registers<N>(f, tw);
#pragma unroll
    for (int i = 0; i < N; ++i)
      planes[p * N * RS + q * RS + bit_reverse<N>(i)] = f[i];
  }
  __syncthreads();
  if (active) {
#pragma unroll
    for (int i = 0; i < N; ++i) f[i] = planes[p * N * RS + i * RS + q];
    fft_dif_registers<N>(f, tw);
  }
}

}  // namespace idg_mi355x
