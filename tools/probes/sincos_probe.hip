// sincos_probe.hip -- measures the phasor accuracy of the candidate gfx950
// sin/cos paths on IDG-like phases (TEST / DESIGN EVIDENCE, not product).
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I../../ska-sdp-idg-bench_amd/csrc \
//         -o sincos_probe sincos_probe.hip && ./sincos_probe
//
// For N fp32 phases x (|x| up to 3500 rad, the range IDG reaches) it prints
// max / RMS absolute error of sin and cos against double-precision sin/cos of
// the same fp32 value, for:
//   ocml      sincosf (OCML, accurate library path)
//   fast      __sinf/__cosf (v_mul 1/2pi + v_sin/v_cos, no range reduction)
//   rev_hw    revolutions(x) (Dekker-split 1/2pi) + v_sin_f32/v_cos_f32
//   anch_hw   anchored: A within +-2.5 rad, r = fma(x-A, 1/2pi, rev(A))
//   rev_poly  revolutions(x) + quadrant polynomial (IDG_SINCOS_POLY)
//   hw_small  v_sin/v_cos on r uniform in [-0.5, 0.5] (pure unit accuracy)
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#include "hip/kernels/device.hpp"

using namespace idg_mi355x;

namespace poly {
__device__ __forceinline__ void sincos_rev_poly(float r, float *s, float *c) {
  const float q = __builtin_rintf(4.0f * r);
  const float g = fma_(q, -0.25f, r);
  const float x = g * 6.28318530717958647692f;
  const float z = x * x;
  float sp = fma_(fma_(-1.9515295891e-4f, z, 8.3321608736e-3f), z,
                  -1.6666654611e-1f);
  const float sn = fma_(sp * z, x, x);
  float cp = fma_(fma_(2.443315711809948e-5f, z, -1.388731625493765e-3f), z,
                  4.166664568298827e-2f);
  const float cs = fma_(cp * z, z, fma_(-0.5f, z, 1.0f));
  const int qi = static_cast<int>(q) & 3;
  const float s0 = (qi & 1) ? cs : sn;
  const float c0 = (qi & 1) ? sn : cs;
  *s = (qi & 2) ? -s0 : s0;
  *c = ((qi + 1) & 2) ? -c0 : c0;
}
}  // namespace poly

__global__ void probe(const float *x, const float *anchor, const float *small,
                      float *out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float v = x[i];
  float s, c;
  sincosf(v, &s, &c);
  out[12 * i + 0] = s;
  out[12 * i + 1] = c;
  out[12 * i + 2] = __sinf(v);
  out[12 * i + 3] = __cosf(v);
  const float r = revolutions(v);
  out[12 * i + 4] = __builtin_amdgcn_sinf(r);
  out[12 * i + 5] = __builtin_amdgcn_cosf(r);
  const float A = anchor[i];
  const float ra = fma_(v - A, kInv2PiHi, revolutions(A));
  out[12 * i + 6] = __builtin_amdgcn_sinf(ra);
  out[12 * i + 7] = __builtin_amdgcn_cosf(ra);
  poly::sincos_rev_poly(r, &s, &c);
  out[12 * i + 8] = s;
  out[12 * i + 9] = c;
  out[12 * i + 10] = __builtin_amdgcn_sinf(small[i]);
  out[12 * i + 11] = __builtin_amdgcn_cosf(small[i]);
}

int main() {
  const int n = 1 << 22;
  std::mt19937 rng(1234);
  std::uniform_real_distribution<float> ux(-3500.0f, 3500.0f),
      ud(-2.5f, 2.5f), us(-0.5f, 0.5f);
  std::vector<float> x(n), a(n), sm(n), out(12 * static_cast<size_t>(n));
  for (int i = 0; i < n; ++i) {
    x[i] = ux(rng);
    a[i] = x[i] + ud(rng);
    sm[i] = us(rng);
  }
  float *dx, *da, *ds, *dout;
  (void)hipMalloc(&dx, n * 4);
  (void)hipMalloc(&da, n * 4);
  (void)hipMalloc(&ds, n * 4);
  (void)hipMalloc(&dout, out.size() * 4);
  (void)hipMemcpy(dx, x.data(), n * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(da, a.data(), n * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(ds, sm.data(), n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3((n + 255) / 256), dim3(256), 0, 0, dx, da, ds,
                     dout, n);
  if (hipDeviceSynchronize() != hipSuccess) {
    std::printf("kernel failed\n");
    return 1;
  }
  (void)hipMemcpy(out.data(), dout, out.size() * 4, hipMemcpyDeviceToHost);
  const char *names[6] = {"ocml", "fast", "rev_hw", "anch_hw", "rev_poly",
                          "hw_small"};
  std::printf("%-10s %12s %12s %12s %12s\n", "path", "sin_max", "sin_rms",
              "cos_max", "cos_rms");
  for (int k = 0; k < 6; ++k) {
    double smax = 0, srms = 0, cmax = 0, crms = 0;
    for (int i = 0; i < n; ++i) {
      const double v = k == 5 ? 2.0 * M_PI * static_cast<double>(sm[i])
                              : static_cast<double>(x[i]);
      const double es = std::fabs(out[12 * (size_t)i + 2 * k] - std::sin(v));
      const double ec =
          std::fabs(out[12 * (size_t)i + 2 * k + 1] - std::cos(v));
      smax = std::max(smax, es);
      cmax = std::max(cmax, ec);
      srms += es * es;
      crms += ec * ec;
    }
    std::printf("%-10s %12.3e %12.3e %12.3e %12.3e\n", names[k], smax,
                std::sqrt(srms / n), cmax, std::sqrt(crms / n));
  }
  return 0;
}
