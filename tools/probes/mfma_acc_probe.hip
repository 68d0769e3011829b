// mfma_acc_probe.hip -- how v_mfma_f32_16x16x32_f16 rounds its f32
// accumulation (the gridder's error against exact
// accumulation).  The products of two f16 values are exact in f32, so the
// only rounding of one MFMA is in the sum  D = C + sum_k A[i][k] B[k][j].
//
// (1) single-MFMA cases: random C and 32 random exact products per output
//     element; the hardware result is classified against the exact sum
//     rounded to nearest-even (RNE), toward zero (RTZ), down and up, and the
//     signed error is reported in ulps of the exact result (a bias would be
//     coherent in the gridder's sums);
// (2) chains of NK MFMAs accumulating positive-mean products (the coherent
//     growth of a gridded pixel): hardware relative error against the exact
//     sum, beside an emulation that rounds once per MFMA (RNE) and one that
//     adds the 32 products to C one at a time in f32 (RNE).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

__host__ __device__ inline uint32_t mix(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}
// f16-representable value: sign (if signed), mantissa 11 bits, exponent in
// [emin, emin + erange)
__host__ __device__ inline float hval(uint32_t h, int emin, int erange,
                                      bool sgn) {
  const int e = emin + static_cast<int>((h >> 11) % erange);
  const float m = 1.0f + static_cast<float>(h & 1023u) / 1024.0f;
  const float v = ldexpf(m, e);
  return (sgn && (h >> 31)) ? -v : v;
}

// element (i, k) of A and (k, j) of B at step it; A[i][k] for lane l:
// row l & 15, k = 8 (l >> 4) + jj.
struct Gen {
  uint32_t seed;
  int amin, arng, bmin, brng;
  bool sgn;
  __host__ __device__ float a(int it, int i, int k) const {
    return hval(mix(seed ^ mix(it * 7919u + i * 131u + k)), amin, arng, sgn);
  }
  __host__ __device__ float b(int it, int k, int j) const {
    return hval(mix(~seed ^ mix(it * 104729u + k * 61u + j)), bmin, brng,
                sgn);
  }
};

__global__ void chain(Gen g, const float *c0, int nk, float *D) {
  const int l = threadIdx.x;
  floatx4 acc;
  for (int r = 0; r < 4; ++r) acc[r] = c0[(4 * (l >> 4) + r) * 16 + (l & 15)];
  for (int it = 0; it < nk; ++it) {
    half8 a, b;
    for (int jj = 0; jj < 8; ++jj) {
      a[jj] = static_cast<_Float16>(g.a(it, l & 15, 8 * (l >> 4) + jj));
      b[jj] = static_cast<_Float16>(g.b(it, 8 * (l >> 4) + jj, l & 15));
    }
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc, 0, 0, 0);
  }
  for (int r = 0; r < 4; ++r) D[(4 * (l >> 4) + r) * 16 + (l & 15)] = acc[r];
}

static float ulp_of(long double x) {
  const float f = static_cast<float>(fabsl(x));
  return nextafterf(f, INFINITY) - f;
}

int main() {
  float *dC, *dD;
  (void)hipMalloc(&dC, 1024);
  (void)hipMalloc(&dD, 1024);
  std::vector<float> C(256), D(256);

  // (1) single MFMAs: C of magnitude ~2^6 .. 2^7, products ~2^-4 .. 2^0
  long cnt = 0, n_rne = 0, n_rtz = 0, n_dn = 0, n_up = 0, n_inexact = 0;
  double bias = 0.0, rms = 0.0;
  for (int trial = 0; trial < 4000; ++trial) {
    Gen g{static_cast<uint32_t>(trial * 2654435761u), -3, 2, -2, 2, true};
    for (int i = 0; i < 256; ++i)
      C[i] = hval(mix(trial * 977u + i), 6, 2, true);
    (void)hipMemcpy(dC, C.data(), 1024, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(chain, dim3(1), dim3(64), 0, 0, g, dC, 1, dD);
    (void)hipMemcpy(D.data(), dD, 1024, hipMemcpyDeviceToHost);
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j) {
        long double e = C[i * 16 + j];
        for (int k = 0; k < 32; ++k)
          e += static_cast<long double>(g.a(0, i, k)) * g.b(0, k, j);
        const float rne = static_cast<float>(e);
        const float d = D[i * 16 + j];
        ++cnt;
        if (static_cast<long double>(rne) == e) {
          n_rne += d == rne;
          continue;
        }
        ++n_inexact;
        const float lo = static_cast<long double>(rne) < e
                             ? rne : nextafterf(rne, -INFINITY);
        const float hi = nextafterf(lo, INFINITY);
        const float rtz = e > 0 ? lo : hi;
        n_rne += d == rne;
        n_rtz += d == rtz;
        n_dn += d == lo;
        n_up += d == hi;
        const double err = static_cast<double>((d - e) / ulp_of(e));
        bias += err;
        rms += err * err;
      }
  }
  std::printf("single MFMA (C ~ 2^6, 32 products ~ 2^-4): %ld elements, %ld "
              "inexact\n  hw == RNE %ld, == RTZ %ld, == down %ld, == up %ld\n"
              "  signed error: mean %+.4f ulp, rms %.4f ulp (RNE: 0, 0.29)\n",
              cnt, n_inexact, n_rne, n_rtz, n_dn, n_up,
              bias / std::max(1L, n_inexact),
              std::sqrt(rms / std::max(1L, n_inexact)));

  // (2) chains: positive products (coherent growth), C = 0
  for (int nk : {128, 2048}) {
    double e_hw = 0, e_mf = 0, e_seq = 0, b_hw = 0;
    int n = 0;
    for (int trial = 0; trial < 8; ++trial) {
      Gen g{static_cast<uint32_t>(0x51ed27u + trial * 97u), -2, 2, -2, 2,
            false};
      for (auto &x : C) x = 0.0f;
      (void)hipMemcpy(dC, C.data(), 1024, hipMemcpyHostToDevice);
      hipLaunchKernelGGL(chain, dim3(1), dim3(64), 0, 0, g, dC, nk, dD);
      (void)hipMemcpy(D.data(), dD, 1024, hipMemcpyDeviceToHost);
      for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j) {
          long double ex = 0;
          float mf = 0.0f, seq = 0.0f;
          for (int it = 0; it < nk; ++it) {
            long double s = 0;
            for (int k = 0; k < 32; ++k) {
              const float p = g.a(it, i, k) * g.b(it, k, j);  // exact
              s += p;
              seq = seq + p;
            }
            ex += s;
            mf = static_cast<float>(static_cast<long double>(mf) + s);
          }
          const double d = D[i * 16 + j];
          e_hw += std::pow(static_cast<double>((d - ex) / ex), 2);
          b_hw += static_cast<double>((d - ex) / ex);
          e_mf += std::pow(static_cast<double>((mf - ex) / ex), 2);
          e_seq += std::pow(static_cast<double>((seq - ex) / ex), 2);
          ++n;
        }
    }
    std::printf("chain of %d MFMAs (K = %d products): relative rms error hw "
                "%.3e (mean %+.3e), one RNE per MFMA %.3e, sequential f32 "
                "%.3e\n",
                nk, 32 * nk, std::sqrt(e_hw / n), b_hw / n,
                std::sqrt(e_mf / n), std::sqrt(e_seq / n));
  }
  return 0;
}
