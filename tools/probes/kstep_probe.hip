// kstep_probe.hip -- the gridder's mirror-path K-step in isolation (DESIGN
// EVIDENCE, §5.1): per lane two tile pairs x four channels of the exact
// phase chain (two v_pk_fma), v_sin/v_cos, the f16 split (split_oct) and
// four f16 MFMAs per tile pair, looped over K-steps on registers, at the
// kernel's occupancy (8-wave workgroups, WG_PER_CU per CU).  Flags add the
// kernel's context one piece at a time:
//   LDSB  B fragments read from LDS per K-step (2 ds_read_b128), as the kernel
//   SMALL revolutions in [-0.7, 0.7] (the kernel's range) instead of ~100
//   ANCH  the per-timestep-quad anchor (phase_index, -m) every 4 K-steps
// Prints cycles per K-step and wave, to compare with the kernel's own loop
// (7.75 ms at configs[1] = ~760 cycles per K-step and wave).
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off \
//     -I../../ska-sdp-idg-bench_amd/csrc -mllvm -amdgpu-sched-strategy=max-ilp \
//     kstep_probe.hip -o kstep_probe
#include <hip/hip_runtime.h>

#include <cstdio>

#include "hip/kernels/device.hpp"
#include "hip/kernels/mfma.hpp"

using namespace idg_mi355x;

#ifndef WG_PER_CU
#define WG_PER_CU 2
#endif
enum { LDSB = 1, SMALL = 2, ANCH = 4 };

// FR of every 4 K-steps run on v_mfma_f32_16x16x4_f32 with the unsplit f32
// cos/sin (one MFMA per tile, channel and X/Y: 32 per K-step and wave against
// 8 f16 MFMAs; the B columns 8..15 of the f32 form are unused), the rest on
// the f16 split (the matrix pipe is ~84% idle while the
// split is ~40% of the VALU issue).
// (mfma4: mfma.hpp)

template <int F, int FR = 0>
__global__ void __launch_bounds__(512, 4)
    kstep(float *out, const float *kin, const float4 *uvwin, int iters) {
  __shared__ uint4 bbuf[4 * 64 * 2];
  const int lane = threadIdx.x & 63, grp = lane >> 4;
  floatx2 L2[2], M2[2], PG2[2], NP[2], NM[2];
  for (int h = 0; h < 2; ++h) {
    L2[h] = floatx2{(lane - 32) * 1.5e-3f, (h - 0.5f) * 2e-2f};
    M2[h] = floatx2{(h + 1) * 1e-2f, (lane - 20) * 1.1e-3f};
    PG2[h] = floatx2{lane * 0.013f, h * 0.7f};
    NP[h] = floatx2{-(lane * 0.37f + h), -(lane * 0.11f + 2 * h)};
    NM[h] = floatx2{-3.0f, -5.0f};
  }
  float kb[4];
  for (int j = 0; j < 4; ++j) kb[j] = kin[j];  // wave-uniform (SGPRs)
  const floatx2 ih = {kInv2PiHi, kInv2PiHi};
  floatx4 accx[4], accy[4];
  for (int i = 0; i < 4; ++i) accx[i] = accy[i] = floatx4{0, 0, 0, 0};
  half8 bfx, bfy;
  float b32x = lane * 1e-3f, b32y = lane * 2e-3f;
  for (int i = 0; i < 8; ++i) {
    bfx[i] = (_Float16)(lane * 1e-3f + i);
    bfy[i] = (_Float16)(i * 0.25f);
  }
  for (int i = threadIdx.x; i < 4 * 64 * 2; i += 512)
    bbuf[i] = make_uint4(0x3c003c00u + i, 0x3c003c00u, 0x38003800u, 0x3400u);
  __syncthreads();
  for (int it = 0; it < iters; ++it) {
    if ((F & ANCH) && (it & 3) == 0) {
      const float4 c4 = uvwin[(it >> 2) & 63 | grp];
      const floatx2 cu = {c4.x, c4.x}, cv = {c4.y, c4.y};
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const floatx2 pidx = __builtin_elementwise_fma(cu, L2[h], cv * M2[h]);
        NP[h] = -pidx;
        const floatx2 a =
            __builtin_elementwise_fma(NP[h], floatx2{kb[0], kb[0]}, PG2[h]);
        const floatx2 t = a * ih;
        NM[h] = floatx2{-__builtin_rintf(t.x), -__builtin_rintf(t.y)};
      }
    }
    if (F & LDSB) {
      const int ks = it & 3;
      const uint4 bx = bbuf[(ks * 64 + lane) * 2];
      const uint4 by = bbuf[(ks * 64 + lane) * 2 + 1];
      bfx = pack4(bx.x, bx.y, bx.z, bx.w);
      bfy = pack4(by.x, by.y, by.z, by.w);
      b32x = __builtin_bit_cast(float, bx.x);
      b32y = __builtin_bit_cast(float, by.y);
    }
    if (FR > 0 && (it & 3) < FR) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        float snx[4], csx[4], sny[4], csy[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float kj = kb[j];
          const floatx2 ph =
              __builtin_elementwise_fma(NP[h], floatx2{kj, kj}, PG2[h]);
          floatx2 r = __builtin_elementwise_fma(ph, ih, NM[h]);
          sincos_rev(r.x, &snx[j], &csx[j]);
          sincos_rev(r.y, &sny[j], &csy[j]);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          accx[2 * h] = mfma4(csx[j], b32x, accx[2 * h]);
          accy[2 * h] = mfma4(snx[j], b32y, accy[2 * h]);
          accx[2 * h + 1] = mfma4(csy[j], b32x, accx[2 * h + 1]);
          accy[2 * h + 1] = mfma4(sny[j], b32y, accy[2 * h + 1]);
        }
      }
      IDG_KSTEP_FENCE();
      NM[0] = NM[0] + floatx2{1.0f, 1.0f};
      NM[1] = NM[1] - floatx2{1.0f, 1.0f};
      continue;
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      float snx[4], csx[4], sny[4], csy[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float kj = kb[j];
        const floatx2 ph =
            __builtin_elementwise_fma(NP[h], floatx2{kj, kj}, PG2[h]);
        floatx2 r = __builtin_elementwise_fma(ph, ih, NM[h]);
        if ((F & SMALL) && !(F & ANCH)) r = r * floatx2{1e-3f, 1e-3f};
        sincos_rev(r.x, &snx[j], &csx[j]);
        sincos_rev(r.y, &sny[j], &csy[j]);
      }
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
    IDG_KSTEP_FENCE();
    // the anchors change per timestep quad in the kernel: keep the phases
    // loop-variant here too (one v_pk_add per K-step), or the compiler
    // hoists v_sin/v_cos out of the loop
    NM[0] = NM[0] + floatx2{1.0f, 1.0f};
    NM[1] = NM[1] - floatx2{1.0f, 1.0f};
  }
  float r = 0;
  for (int i = 0; i < 4; ++i)
    r += accx[i][0] + accx[i][3] + accy[i][1] + accy[i][2];
  out[blockIdx.x * 512 + threadIdx.x] = r;
}

template <int F, int FR = 0>
void run(const char *name, float *out, const float *k, const float4 *uvw) {
  const int grid = 256 * WG_PER_CU, iters = 4000;
  hipLaunchKernelGGL((kstep<F, FR>), dim3(grid), dim3(512), 0, 0, out, k, uvw, 50);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, 0);
  hipLaunchKernelGGL((kstep<F, FR>), dim3(grid), dim3(512), 0, 0, out, k, uvw,
                     iters);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double waves_per_simd = grid * 8.0 / 1024.0;
  const double cyc = ms * 1e-3 * 2.4e9 / (iters * waves_per_simd);
  std::printf("%-34s waves/SIMD %.0f  %8.3f ms  %7.1f cyc per K-step and wave"
              "  (%.2f per phasor)\n", name, waves_per_simd, ms, cyc,
              cyc / 16.0);
}

int main() {
  float *out, *k;
  float4 *uvw;
  (void)hipMalloc(&out, 256 * 8 * 512 * sizeof(float));
  (void)hipMalloc(&k, 4 * sizeof(float));
  (void)hipMalloc(&uvw, 64 * sizeof(float4));
  const float kh[4] = {31.4f, 31.6f, 31.8f, 32.0f};
  (void)hipMemcpy(k, kh, sizeof(kh), hipMemcpyHostToDevice);
  float4 uh[64];
  for (int i = 0; i < 64; ++i)
    uh[i] = make_float4(300.0f + 37.0f * i, -200.0f + 11.0f * i, 0.0f, 0.0f);
  (void)hipMemcpy(uvw, uh, sizeof(uh), hipMemcpyHostToDevice);
  run<0>("registers only", out, k, uvw);
  run<SMALL>("small revolutions", out, k, uvw);
  run<LDSB>("B from LDS", out, k, uvw);
  run<LDSB | SMALL>("B from LDS, small rev", out, k, uvw);
  run<LDSB | ANCH>("B from LDS + anchors", out, k, uvw);
  run<LDSB | ANCH, 1>("+ f32 MFMA on 1/4 of K-steps", out, k, uvw);
  run<LDSB | ANCH, 2>("+ f32 MFMA on 2/4 of K-steps", out, k, uvw);
  run<LDSB | ANCH, 3>("+ f32 MFMA on 3/4 of K-steps", out, k, uvw);
  run<LDSB | ANCH, 4>("+ f32 MFMA on 4/4 of K-steps", out, k, uvw);
  (void)hipDeviceSynchronize();
  return 0;
}
