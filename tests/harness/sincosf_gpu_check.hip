// sincosf_gpu_check.hip -- TEST INFRASTRUCTURE: the restated glibc sincosf
// (csrc/common/sincosf_glibc.hpp) evaluated ON THE GPU against the host's own
// glibc sincosf, bit for bit (tests/test_gpu_sequential.py).  The device
// build differs from the host one in its 4/pi table lookup (immediates for
// |y| < 2^15, a __constant__ table beyond) and its int64 -> double
// conversion (two exact halves and one FMA), so it is checked separately.
//
//   sincosf_gpu_check LO HI STRIDE
// walks the float bit patterns LO, LO + STRIDE, ... < HI, both signs.
// Prints "checked N mismatch M mismatch_dev D" (the restatement and the
// kernels' form, sincosf_glibc_dev) and exits 1 on any mismatch.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <cstdint>
#include <vector>

#include "common/sincosf_glibc.hpp"

__global__ void eval(uint64_t lo, uint64_t stride, long long n, float *s,
                     float *c, float *s2, float *c2) {
  __shared__ idg::SincosfWindow win[idg::kSincosfWindows];
  idg::sincosf_windows_to_lds(win, threadIdx.x);
  __syncthreads();
  const long long k = blockIdx.x * static_cast<long long>(blockDim.x) +
                      threadIdx.x;
  if (k >= n) return;
  uint32_t b = static_cast<uint32_t>(lo + static_cast<uint64_t>(k >> 1) *
                                              stride);
  if (k & 1) b |= 0x80000000u;
  float y;
  memcpy(&y, &b, 4);
  idg::sincosf_glibc(y, &s[k], &c[k]);
  idg::sincosf_glibc_dev(y, &s2[k], &c2[k], win);
}

#define CHECK(x)                                                        \
  do {                                                                  \
    hipError_t e_ = (x);                                                \
    if (e_ != hipSuccess) {                                             \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
      return 2;                                                         \
    }                                                                   \
  } while (0)

int main(int argc, char **argv) {
  if (argc != 4) {
    fprintf(stderr, "usage: %s LO HI STRIDE\n", argv[0]);
    return 2;
  }
  const uint64_t lo = strtoull(argv[1], nullptr, 0);
  const uint64_t hi = strtoull(argv[2], nullptr, 0);
  const uint64_t stride = strtoull(argv[3], nullptr, 0);
  const long long total = 2 * (long long)((hi - lo + stride - 1) / stride);
  const long long chunk = 1LL << 26;
  float *ds = nullptr, *dc = nullptr, *ds2 = nullptr, *dc2 = nullptr;
  CHECK(hipMalloc(&ds, chunk * sizeof(float)));
  CHECK(hipMalloc(&dc, chunk * sizeof(float)));
  CHECK(hipMalloc(&ds2, chunk * sizeof(float)));
  CHECK(hipMalloc(&dc2, chunk * sizeof(float)));
  std::vector<float> hs(chunk), hc(chunk), hs2(chunk), hc2(chunk);
  long long mismatch = 0, mismatch_dev = 0;
  for (long long k0 = 0; k0 < total; k0 += chunk) {
    const long long n = total - k0 < chunk ? total - k0 : chunk;
    const uint64_t lo_k = lo + static_cast<uint64_t>(k0 >> 1) * stride;
    hipLaunchKernelGGL(eval, dim3((n + 255) / 256), dim3(256), 0, 0, lo_k,
                       stride, n, ds, dc, ds2, dc2);
    CHECK(hipGetLastError());
    CHECK(hipMemcpy(hs.data(), ds, n * sizeof(float), hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(hc.data(), dc, n * sizeof(float), hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(hs2.data(), ds2, n * sizeof(float), hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(hc2.data(), dc2, n * sizeof(float), hipMemcpyDeviceToHost));
    long long bad = 0, bad_dev = 0;
#pragma omp parallel for reduction(+ : bad, bad_dev) schedule(static, 65536)
    for (long long k = 0; k < n; k++) {
      uint32_t b = static_cast<uint32_t>(lo_k + static_cast<uint64_t>(k >> 1) *
                                                    stride);
      if (k & 1) b |= 0x80000000u;
      float y, s, c;
      memcpy(&y, &b, 4);
      sincosf(y, &s, &c);
      if (memcmp(&s, &hs[k], 4) || memcmp(&c, &hc[k], 4)) bad++;
      // the kernels' form (sincosf_glibc_dev); NaN results compared as NaN
      // (the device's default NaN is not x86's)
      const bool nan = s != s && hs2[k] != hs2[k] && c != c && hc2[k] != hc2[k];
      if (!nan && (memcmp(&s, &hs2[k], 4) || memcmp(&c, &hc2[k], 4)))
        bad_dev++;
    }
    mismatch += bad;
    mismatch_dev += bad_dev;
  }
  // "mismatch": the restatement (sincosf_glibc); "mismatch_dev": the kernels'
  // form (sincosf_glibc_dev)
  printf("checked %lld mismatch %lld mismatch_dev %lld\n", total,
         mismatch, mismatch_dev);
  (void)hipFree(ds);
  (void)hipFree(dc);
  (void)hipFree(ds2);
  (void)hipFree(dc2);
  return (mismatch || mismatch_dev) ? 1 : 0;
}
