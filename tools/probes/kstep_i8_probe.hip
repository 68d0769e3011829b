// kstep_i8_probe.hip -- DESIGN EVIDENCE for a fixed-point phasor operand:
// the gridder's mirror-path K-step with the phasor fed to the i8 matrix core
// as a 24-bit fixed-point number instead of an f16 hi + lo split.
//
// Phasor component c in [-1, 1]:  t = fma(c, 63/64, K), K = 3 + 0x8080 2^-22,
// lies in [2, 4) (ulp 2^-22), and the bytes of bits(t) ^ 0x00808080 read as
// signed int8 (a0, a1, a2, a3 = 64) give exactly
//   X = round(c 63/64 2^22) = a0 + 256 a1 + 65536 (a2 + a3),
// so the four bytes of one VGPR are four K-slots of v_mfma_i32_16x16x64_i8
// (slots 2 and 3 share a significance): one v_pk_fma_f32 per (cos, sin) pair
// and one v_xor_b32 per value replace the f16 split's four VOP3 conversions
// per pair.  B (the visibilities) carries balanced base-256 digits; the
// column sets s = 1..4 (significance 256^s) of two MFMAs per GEMM collect
// the digit products.
//
// Part 1 checks the lane map of v_mfma_i32_16x16x64_i8 with exact integers
// (A lane l byte j and B lane l byte j meet in the same k).  Part 2 times the
// f16 K-step (as kstep_probe "B from LDS") against the i8 K-step.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off \
//     -I../../ska-sdp-idg-bench_amd/csrc -mllvm -amdgpu-sched-strategy=max-ilp \
//     kstep_i8_probe.hip -o kstep_i8_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "hip/kernels/device.hpp"
#include "hip/kernels/mfma.hpp"

using namespace idg_mi355x;

typedef int intx4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ intx4 mfma_i8(const intx4 &a, const intx4 &b,
                                         const intx4 &c) {
  return __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
}

// ---- part 1: lane map -------------------------------------------------
// A[16][64], B[64][16] int8 in global memory (row-major), C[16][16] int32.
// Assumed map: lane l holds A[l & 15][16 (l >> 4) + j] and
// B[16 (l >> 4) + j][l & 15] in byte j = 0..15; C row (l >> 4) * 4 + r,
// column l & 15 in register r.
__global__ void map_test(const signed char *A, const signed char *B, int *C) {
  const int l = threadIdx.x;
  intx4 a, b;
  signed char *pa = reinterpret_cast<signed char *>(&a);
  signed char *pb = reinterpret_cast<signed char *>(&b);
  for (int j = 0; j < 16; ++j) {
    pa[j] = A[(l & 15) * 64 + 16 * (l >> 4) + j];
    pb[j] = B[(16 * (l >> 4) + j) * 16 + (l & 15)];
  }
  intx4 c = {0, 0, 0, 0};
  c = mfma_i8(a, b, c);
  for (int r = 0; r < 4; ++r) C[((l >> 4) * 4 + r) * 16 + (l & 15)] = c[r];
}

// ---- part 3: MFMA throughput alone (4 independent accumulators) -------
template <int I8, int NV>
__global__ void __launch_bounds__(256) mfma_rate(float *out, int iters) {
  float va[8];
  for (int i = 0; i < 8; ++i) va[i] = threadIdx.x * 1e-3f + i;
  const int lane = threadIdx.x & 63;
  intx4 ia = {lane, 3 * lane, 5, 7}, ib = {lane ^ 9, 11, lane, 13};
  half8 ha, hb;
  for (int i = 0; i < 8; ++i) {
    ha[i] = (_Float16)(lane * 1e-3f + i);
    hb[i] = (_Float16)(i * 0.5f);
  }
  intx4 ic[4];
  floatx4 fc[4];
  for (int i = 0; i < 4; ++i) {
    ic[i] = intx4{0, 0, 0, 0};
    fc[i] = floatx4{0, 0, 0, 0};
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (I8 == 1) ic[i] = mfma_i8(ia, ib, ic[i]);
      if (I8 == 0) fc[i] = mfma16(ha, hb, fc[i]);
#pragma unroll
      for (int v = 0; v < NV; ++v)
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(va[v & 7]) : "v"(va[(v + 1) & 7]), "v"(va[(v + 3) & 7]));
    }
  }
  float r = 0;
  for (int i = 0; i < 4; ++i) r += (float)ic[i][0] + fc[i][1];
  for (int i = 0; i < 8; ++i) r += va[i];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

template <int I8, int NV>
void run_rate(const char *name, float *out) {
  const int grid = 256 * 8, iters = 20000;  // 8 waves per SIMD
  hipLaunchKernelGGL((mfma_rate<I8, NV>), dim3(grid), dim3(256), 0, 0, out, 100);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, 0);
  hipLaunchKernelGGL((mfma_rate<I8, NV>), dim3(grid), dim3(256), 0, 0, out, iters);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double mfma_per_simd = grid * 4.0 / 1024.0 * iters * 4;
  std::printf("%-30s +%d v_fma each: %8.3f ms  %6.2f cycles per (MFMA + VALU) per SIMD\n",
              name, NV, ms, ms * 1e-3 * 2.4e9 / mfma_per_simd);
}

// ---- part 2: K-step timing ---------------------------------------------
constexpr float kFixS = 63.0f / 64.0f;
constexpr float kFixK = 3.0f + 0x8080 * 0x1p-22f;

template <int I8, int NH>
__global__ void __launch_bounds__(512, 2)
    kstep(float *out, const float *kin, int iters) {
  __shared__ uint4 bbuf[4 * 64 * 4];
  const int lane = threadIdx.x & 63;
  floatx2 L2[2], M2[2], PG2[2], NP[2], NM[2];
  for (int h = 0; h < 2; ++h) {
    L2[h] = floatx2{(lane - 32) * 1.5e-3f, (h - 0.5f) * 2e-2f};
    M2[h] = floatx2{(h + 1) * 1e-2f, (lane - 20) * 1.1e-3f};
    PG2[h] = floatx2{lane * 0.013f, h * 0.7f};
    NP[h] = floatx2{-(lane * 0.37f + h), -(lane * 0.11f + 2 * h)};
    NM[h] = floatx2{-3.0f, -5.0f};
  }
  float kb[4];
  for (int j = 0; j < 4; ++j) kb[j] = kin[j];
  const floatx2 ih = {kInv2PiHi, kInv2PiHi};
  floatx4 accx[4], accy[4];
  intx4 iax[4][2], iay[4][2];
  for (int i = 0; i < 4; ++i) {
    accx[i] = accy[i] = floatx4{0, 0, 0, 0};
    iax[i][0] = iax[i][1] = iay[i][0] = iay[i][1] = intx4{0, 0, 0, 0};
  }
  for (int i = threadIdx.x; i < 4 * 64 * 4; i += 512)
    bbuf[i] = make_uint4(0x3c003c00u + i, 0x3c003c00u, 0x38003800u, 0x3400u);
  __syncthreads();
  const floatx2 fs = {kFixS, kFixS}, fk = {kFixK, kFixK};
  intx4 pcx = {0, 0, 0, 0}, psx = pcx, pcy = pcx, psy = pcx;
  for (int it = 0; it < iters; ++it) {
    const int ks = it & 3;
    const uint4 b0 = bbuf[(ks * 64 + lane) * 4];
    const uint4 b1 = bbuf[(ks * 64 + lane) * 4 + 1];
    uint4 b2, b3;
    if (I8) {
      b2 = bbuf[(ks * 64 + lane) * 4 + 2];
      b3 = bbuf[(ks * 64 + lane) * 4 + 3];
    }
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      float snx[4], csx[4], sny[4], csy[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float kj = kb[j];
        const floatx2 ph =
            __builtin_elementwise_fma(NP[h], floatx2{kj, kj}, PG2[h]);
        const floatx2 r = __builtin_elementwise_fma(ph, ih, NM[h]);
        sincos_rev(r.x, &snx[j], &csx[j]);
        sincos_rev(r.y, &sny[j], &csy[j]);
      }
      if (I8 == 4 || I8 == 5) {
        // VALU only: the operands are folded into the accumulators by one
        // v_xor per 4 VGPRs instead of MFMAs
        intx4 cx, sx, cy, sy;
        if (I8 == 4) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const floatx2 tc = __builtin_elementwise_fma(floatx2{csx[j], csy[j]}, fs, fk);
            const floatx2 ts = __builtin_elementwise_fma(floatx2{snx[j], sny[j]}, fs, fk);
            cx[j] = __float_as_int(tc.x) ^ 0x00808080;
            cy[j] = __float_as_int(tc.y) ^ 0x00808080;
            sx[j] = __float_as_int(ts.x) ^ 0x00808080;
            sy[j] = __float_as_int(ts.y) ^ 0x00808080;
          }
        } else {
          half8 ac, as, ac2, as2;
          split_oct(csx[0], csx[1], csx[2], csx[3], snx[0], snx[1], snx[2],
                    snx[3], &ac, &as);
          split_oct(csy[0], csy[1], csy[2], csy[3], sny[0], sny[1], sny[2],
                    sny[3], &ac2, &as2);
          cx = __builtin_bit_cast(intx4, ac);
          sx = __builtin_bit_cast(intx4, as);
          cy = __builtin_bit_cast(intx4, ac2);
          sy = __builtin_bit_cast(intx4, as2);
        }
        iax[2 * h][0][0] ^= cx[0] ^ cx[1] ^ cx[2] ^ cx[3] ^ (int)b0.x;
        iay[2 * h][0][0] ^= sx[0] ^ sx[1] ^ sx[2] ^ sx[3];
        iax[2 * h + 1][0][0] ^= cy[0] ^ cy[1] ^ cy[2] ^ cy[3];
        iay[2 * h + 1][0][0] ^= sy[0] ^ sy[1] ^ sy[2] ^ sy[3];
      } else if (I8 >= 2) {
        // software pipelined: this tile pair's conversion, then the MFMAs
        // of the previous tile pair (held in pa*) interleaved with it
        intx4 cx, sx, cy, sy;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const floatx2 tc = __builtin_elementwise_fma(floatx2{csx[j], csy[j]}, fs, fk);
          const floatx2 ts = __builtin_elementwise_fma(floatx2{snx[j], sny[j]}, fs, fk);
          cx[j] = __float_as_int(tc.x) ^ 0x00808080;
          cy[j] = __float_as_int(tc.y) ^ 0x00808080;
          sx[j] = __float_as_int(ts.x) ^ 0x00808080;
          sy[j] = __float_as_int(ts.y) ^ 0x00808080;
        }
        const intx4 B0 = {(int)b0.x, (int)b0.y, (int)b0.z, (int)b0.w};
        const intx4 B1 = {(int)b1.x, (int)b1.y, (int)b1.z, (int)b1.w};
        const intx4 B2 = {(int)b2.x, (int)b2.y, (int)b2.z, (int)b2.w};
        const intx4 B3 = {(int)b3.x, (int)b3.y, (int)b3.z, (int)b3.w};
        const int hp = h ^ 1;  // previous tile pair (the other slot)
        iax[2 * hp][0] = mfma_i8(pcx, B0, iax[2 * hp][0]);
        iax[2 * hp][1] = mfma_i8(pcx, B1, iax[2 * hp][1]);
        iay[2 * hp][0] = mfma_i8(psx, B2, iay[2 * hp][0]);
        iay[2 * hp][1] = mfma_i8(psx, B3, iay[2 * hp][1]);
        iax[2 * hp + 1][0] = mfma_i8(pcy, B0, iax[2 * hp + 1][0]);
        iax[2 * hp + 1][1] = mfma_i8(pcy, B1, iax[2 * hp + 1][1]);
        iay[2 * hp + 1][0] = mfma_i8(psy, B2, iay[2 * hp + 1][0]);
        iay[2 * hp + 1][1] = mfma_i8(psy, B3, iay[2 * hp + 1][1]);
        pcx = cx; psx = sx; pcy = cy; psy = sy;
        if (I8 == 3) {
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x400, 2, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
          }
        }
      } else if (I8 == 1 || I8 == 6) {
        intx4 cx, sx, cy, sy;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const floatx2 tc = __builtin_elementwise_fma(floatx2{csx[j], csy[j]}, fs, fk);
          const floatx2 ts = __builtin_elementwise_fma(floatx2{snx[j], sny[j]}, fs, fk);
          cx[j] = __float_as_int(tc.x) ^ 0x00808080;
          cy[j] = __float_as_int(tc.y) ^ 0x00808080;
          sx[j] = __float_as_int(ts.x) ^ 0x00808080;
          sy[j] = __float_as_int(ts.y) ^ 0x00808080;
        }
        const intx4 B0 = {(int)b0.x, (int)b0.y, (int)b0.z, (int)b0.w};
        const intx4 B1 = {(int)b1.x, (int)b1.y, (int)b1.z, (int)b1.w};
        const intx4 B2 = {(int)b2.x, (int)b2.y, (int)b2.z, (int)b2.w};
        const intx4 B3 = {(int)b3.x, (int)b3.y, (int)b3.z, (int)b3.w};
        iax[2 * h][0] = mfma_i8(cx, B0, iax[2 * h][0]);
        iax[2 * h][1] = mfma_i8(cx, B1, iax[2 * h][1]);
        iay[2 * h][0] = mfma_i8(sx, B2, iay[2 * h][0]);
        iay[2 * h][1] = mfma_i8(sx, B3, iay[2 * h][1]);
        iax[2 * h + 1][0] = mfma_i8(cy, B0, iax[2 * h + 1][0]);
        iax[2 * h + 1][1] = mfma_i8(cy, B1, iax[2 * h + 1][1]);
        iay[2 * h + 1][0] = mfma_i8(sy, B2, iay[2 * h + 1][0]);
        iay[2 * h + 1][1] = mfma_i8(sy, B3, iay[2 * h + 1][1]);
        if (I8 == 6) {
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
          }
        }
      } else {
        const half8 bfx = pack4(b0.x, b0.y, b0.z, b0.w);
        const half8 bfy = pack4(b1.x, b1.y, b1.z, b1.w);
        half8 ac, as;
        split_oct(csx[0], csx[1], csx[2], csx[3], snx[0], snx[1], snx[2],
                  snx[3], &ac, &as);
        accx[2 * h] = mfma16(ac, bfx, accx[2 * h]);
        accy[2 * h] = mfma16(as, bfy, accy[2 * h]);
        split_oct(csy[0], csy[1], csy[2], csy[3], sny[0], sny[1], sny[2],
                  sny[3], &ac, &as);
        accx[2 * h + 1] = mfma16(ac, bfx, accx[2 * h + 1]);
        accy[2 * h + 1] = mfma16(as, bfy, accy[2 * h + 1]);
      }
    }
    IDG_KSTEP_FENCE();
    NM[0] = NM[0] + floatx2{1.0f, 1.0f};
    NM[1] = NM[1] - floatx2{1.0f, 1.0f};
  }
  float r = 0;
  for (int i = 0; i < 4; ++i) {
    r += accx[i][0] + accx[i][3] + accy[i][1] + accy[i][2];
    r += (float)(iax[i][0][0] + iax[i][1][3] + iay[i][0][1] + iay[i][1][2]);
  }
  out[blockIdx.x * 512 + threadIdx.x] = r;
}

template <int I8, int NH>
void run(const char *name, float *out, const float *k, int wg_per_cu) {
  const int grid = 256 * wg_per_cu, iters = 4000;
  hipLaunchKernelGGL((kstep<I8, NH>), dim3(grid), dim3(512), 0, 0, out, k, 50);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, 0);
  hipLaunchKernelGGL((kstep<I8, NH>), dim3(grid), dim3(512), 0, 0, out, k, iters);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double waves_per_simd = grid * 8.0 / 1024.0;
  const double cyc = ms * 1e-3 * 2.4e9 / (iters * waves_per_simd);
  std::printf("%-30s tile pairs %d  waves/SIMD %.0f  %8.3f ms  %7.1f cyc per "
              "K-step and wave  (%.2f per phasor)\n", name, NH, waves_per_simd,
              ms, cyc, cyc / (8.0 * NH));
}

int main() {
  // part 1
  signed char hA[16 * 64], hB[64 * 16];
  srand(7);
  for (int i = 0; i < 16 * 64; ++i) hA[i] = (signed char)(rand() % 256 - 128);
  for (int i = 0; i < 64 * 16; ++i) hB[i] = (signed char)(rand() % 256 - 128);
  signed char *dA, *dB;
  int *dC, hC[256];
  (void)hipMalloc(&dA, sizeof(hA));
  (void)hipMalloc(&dB, sizeof(hB));
  (void)hipMalloc(&dC, sizeof(hC));
  (void)hipMemcpy(dA, hA, sizeof(hA), hipMemcpyHostToDevice);
  (void)hipMemcpy(dB, hB, sizeof(hB), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(map_test, dim3(1), dim3(64), 0, 0, dA, dB, dC);
  (void)hipMemcpy(hC, dC, sizeof(hC), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int m = 0; m < 16; ++m)
    for (int n = 0; n < 16; ++n) {
      long s = 0;
      for (int k = 0; k < 64; ++k) s += (long)hA[m * 64 + k] * hB[k * 16 + n];
      bad += s != hC[m * 16 + n];
    }
  std::printf("i8 16x16x64 lane map: %d of 256 outputs differ\n", bad);
  // part 2
  float *out, *k;
  (void)hipMalloc(&out, 256 * 8 * 512 * sizeof(float));
  (void)hipMalloc(&k, 4 * sizeof(float));
  const float kh[4] = {31.4f, 31.6f, 31.8f, 32.0f};
  (void)hipMemcpy(k, kh, sizeof(kh), hipMemcpyHostToDevice);
  run_rate<0, 0>("mfma_f32_16x16x32_f16", out);
  run_rate<1, 0>("mfma_i32_16x16x64_i8", out);
  run_rate<2, 4>("no MFMA", out);
  run_rate<0, 4>("mfma_f32_16x16x32_f16", out);
  run_rate<1, 4>("mfma_i32_16x16x64_i8", out);
  run_rate<2, 8>("no MFMA", out);
  run_rate<0, 8>("mfma_f32_16x16x32_f16", out);
  run_rate<1, 8>("mfma_i32_16x16x64_i8", out);
  for (int w = 1; w <= 2; ++w) {
    run<0, 2>("f16 split (B from LDS)", out, k, w);
    run<1, 2>("i8 fixed point (B from LDS)", out, k, w);
    run<0, 1>("f16 split (B from LDS)", out, k, w);
    run<1, 1>("i8 fixed point (B from LDS)", out, k, w);
    run<4, 1>("i8 conversion, no MFMA", out, k, w);
    run<5, 1>("f16 split, no MFMA", out, k, w);
    run<4, 2>("i8 conversion, no MFMA", out, k, w);
    run<5, 2>("f16 split, no MFMA", out, k, w);
    run<6, 1>("i8 + group barriers", out, k, w);
    run<2, 1>("i8 pipelined", out, k, w);
    run<3, 1>("i8 pipelined + group barriers", out, k, w);
    run<2, 2>("i8 pipelined", out, k, w);
    run<3, 2>("i8 pipelined + group barriers", out, k, w);
  }
  (void)hipDeviceSynchronize();
  return bad != 0;
}
