// degridder_mi355x.hip.cpp -- IDG degridder for MI355X (gfx950).
//
// Replaces the reference's app/HIP/kernels/degridder_*.hip.cpp behind the same
// kernel-TU contract (hip::p_run_degridder, hip::c_run_degridder; harness
// declarations tests/degridder_common.cpp:13-31) and 13-argument kernel ABI
// (grid = nr_subgrids, block = 256).  It computes
// cpu::kernel_degridder_reference
// (app/CPU/kernels/degridder_reference.cpp:6-129):
//
//   P'(y,x) = A1 * (sph * P(y,x)) * A2^H
//   V_p(t,c) = sum_{y,x} P'_p(y,x) * exp(i*phase),
//   phase    = fl(phase_index(t,y,x) * k_c - phase_offset(y,x))   [one FMA]
//
// Design:
//  * one workgroup per subgrid; a lane owns one (timestep, group of CG
//    channels) output unit and keeps CG x 4 complex accumulators in VGPRs;
//  * the workgroup first writes a pixel table into LDS -- P' (8 floats) and
//    (l, m, n, phase_offset) per pixel, 48 B, 1024-pixel chunks (48 KiB) --
//    and every lane then walks the pixels in reference order reading the
//    table with wave-uniform (broadcast) ds_read_b128;
//  * phase reduction as in the gridder: per (lane, pixel) the first channel's
//    phase is converted to revolutions with a Dekker-split 1/(2*pi), the
//    other channels of the group are exact offsets from it;
//  * mirror pixels (even S, w = 0, w_offset = 0): phase(S-1-y, S-1-x) =
//    -phase(y, x) exactly, so each sin/cos pair serves a pixel pair; the
//    table then holds pairs (P'(base), P'(mirror), geometry(base));
//  * 16 v_fma_f32 per (pixel, t, c) complex 4-correlation MAC.
#include <hip/hip_runtime.h>

#include "../util.hpp"
#include "device.hpp"
#include "lib-hip.hpp"

namespace idg_mi355x {

constexpr int kChunk = 1024;  // general path: pixels per LDS table chunk
constexpr int kPairChunk = 512;  // mirror path: pixel pairs per chunk

namespace {

// sum += pixel * phasor for 4 correlations (pa = xx|xy, pb = yx|yy).
__device__ __forceinline__ void cmac4(float *a, const float4 &pa,
                                      const float4 &pb, float cs, float sn) {
  a[0] = fma_(pa.x, cs, a[0]); a[0] = fma_(-pa.y, sn, a[0]);
  a[1] = fma_(pa.x, sn, a[1]); a[1] = fma_(pa.y, cs, a[1]);
  a[2] = fma_(pa.z, cs, a[2]); a[2] = fma_(-pa.w, sn, a[2]);
  a[3] = fma_(pa.z, sn, a[3]); a[3] = fma_(pa.w, cs, a[3]);
  a[4] = fma_(pb.x, cs, a[4]); a[4] = fma_(-pb.y, sn, a[4]);
  a[5] = fma_(pb.x, sn, a[5]); a[5] = fma_(pb.y, cs, a[5]);
  a[6] = fma_(pb.z, cs, a[6]); a[6] = fma_(-pb.w, sn, a[6]);
  a[7] = fma_(pb.z, sn, a[7]); a[7] = fma_(pb.w, cs, a[7]);
}

// P' = A1 * (sph * P) * A2^H of pixel p, and its geometry.
__device__ __forceinline__ void pixel_entry(
    int p, int S, int npix, float image_size, const SubgridSetup &g,
    int nr_stations, const float *__restrict__ spheroidal,
    const float2 *__restrict__ aterms, const float2 *__restrict__ sg,
    float4 &pa, float4 &pb, float4 &geo) {
  const int y = p / S, x = p - (p / S) * S;
  const float sph = spheroidal[p];
  idg::cfloat pix[4], a1[4], a2[4];
#pragma unroll
  for (int cr = 0; cr < 4; ++cr) {
    const float2 v = sg[static_cast<size_t>(cr) * npix + p];
    pix[cr] = {sph * v.x, sph * v.y};
  }
  load_jones(aterm_ptr(aterms, nr_stations, S, g.aterm_index, g.station1, y,
                       x), a1);
  load_jones(aterm_ptr(aterms, nr_stations, S, g.aterm_index, g.station2, y,
                       x), a2);
  idg::apply_aterm_degridder(pix, a1, a2);
  const float l = idg::compute_l(x, S, image_size);
  const float m = idg::compute_m(y, S, image_size);
  const float n = idg::compute_n(l, m);
  // phase_offset = fma(u_o, l, v_o*m) + w_o*n (degridder fusion)
  const float poff = fma_(g.u_offset, l, g.v_offset * m) + g.w_offset * n;
  pa = make_float4(pix[0].re, pix[0].im, pix[1].re, pix[1].im);
  pb = make_float4(pix[2].re, pix[2].im, pix[3].re, pix[3].im);
  geo = make_float4(l, m, n, poff);
}

}  // namespace

template <int S_CT, int CG>
__global__ void __launch_bounds__(kBlock)
    kernel_degridder_mi355x(const int grid_size, int subgrid_size,
                            float image_size, float w_step_in_lambda,
                            int nr_channels, int nr_stations,
                            const idg::UVWCoordinate<float> *__restrict__ uvw,
                            const float *__restrict__ wavenumbers,
                            float2 *__restrict__ visibilities,
                            const float *__restrict__ spheroidal,
                            const float2 *__restrict__ aterms,
                            const idg::Metadata *__restrict__ metadata,
                            const float2 *__restrict__ subgrids) {
  // general: [pixel][0..1] = P' (xx, xy | yx, yy), [pixel][2] = (l,m,n,poff)
  // mirror : [pair][0..1] = P'(base), [pair][2..3] = P'(mirror),
  //          [pair][4] = geometry of the base pixel
  __shared__ float4 table[kChunk * 3];
  static_assert(kPairChunk * 5 <= kChunk * 3, "table size");

  const int S = S_CT > 0 ? S_CT : subgrid_size;
  const int npix = S * S;
  const int s = blockIdx.x;
  const int tid = threadIdx.x;
  const SubgridSetup g = setup_subgrid(metadata, s, grid_size, S, image_size,
                                       w_step_in_lambda);
  const float2 *sg = subgrids + static_cast<size_t>(s) * 4 * npix;
  const int C = nr_channels;
  const int ncg = (C + CG - 1) / CG;
  const int nunits = g.nr_timesteps * ncg;
  const bool mirror_ok = (S % 2 == 0) && g.w_offset == 0.0f;

  for (int ubase = 0; ubase < nunits; ubase += kBlock) {
    const int unit = min(ubase + tid, nunits - 1);
    const bool active = ubase + tid < nunits;
    const int t = unit / ncg;
    const int c0 = (unit - t * ncg) * CG;
    const long long row = g.time_offset + t;
    const idg::UVWCoordinate<float> c = uvw[row];
    float k[CG];
#pragma unroll
    for (int j = 0; j < CG; ++j) k[j] = wavenumbers[min(c0 + j, C - 1)];
    float acc[CG][8];
#pragma unroll
    for (int j = 0; j < CG; ++j)
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[j][q] = 0.0f;

    // Workgroup-uniform: every unit of this pass has w = 0.
    const bool mirror = __syncthreads_and(mirror_ok && c.w == 0.0f);

    if (mirror) {
      // phase(mirror pixel) = -phase(base pixel) exactly.
      const int half = npix / 2;
      for (int pbase = 0; pbase < half; pbase += kPairChunk) {
        const int cnt = min(kPairChunk, half - pbase);
        __syncthreads();
        for (int q = tid; q < cnt; q += kBlock) {
          const int b = pbase + q;
          float4 pa, pb, geo, ma, mb, mgeo;
          pixel_entry(b, S, npix, image_size, g, nr_stations, spheroidal,
                      aterms, sg, pa, pb, geo);
          pixel_entry(npix - 1 - b, S, npix, image_size, g, nr_stations,
                      spheroidal, aterms, sg, ma, mb, mgeo);
          table[5 * q + 0] = pa;
          table[5 * q + 1] = pb;
          table[5 * q + 2] = ma;
          table[5 * q + 3] = mb;
          table[5 * q + 4] = geo;
        }
        __syncthreads();
        for (int q = 0; q < cnt; ++q) {
          const float4 pa = table[5 * q + 0], pb = table[5 * q + 1];
          const float4 ma = table[5 * q + 2], mb = table[5 * q + 3];
          const float4 geo = table[5 * q + 4];
          // phase_index = fma(u, l, v*m) + w*n with w = 0
          const float pidx = fma_(c.u, geo.x, c.v * geo.y);
          const float A = fma_(pidx, k[0], -geo.w);
          const float R = revolutions(A);
#pragma unroll
          for (int j = 0; j < CG; ++j) {
            const float ph = fma_(pidx, k[j], -geo.w);
            const float r = fma_(ph - A, kInv2PiHi, R);
            float sn, cs;
            sincos_rev(r, &sn, &cs);
            cmac4(acc[j], pa, pb, cs, sn);
            cmac4(acc[j], ma, mb, cs, -sn);
          }
        }
      }
    } else {
      for (int pbase = 0; pbase < npix; pbase += kChunk) {
        const int cnt = min(kChunk, npix - pbase);
        __syncthreads();  // previous chunk fully consumed
        for (int q = tid; q < cnt; q += kBlock)
          pixel_entry(pbase + q, S, npix, image_size, g, nr_stations,
                      spheroidal, aterms, sg, table[3 * q + 0],
                      table[3 * q + 1], table[3 * q + 2]);
        __syncthreads();
        for (int q = 0; q < cnt; ++q) {
          const float4 pa = table[3 * q + 0];
          const float4 pb = table[3 * q + 1];
          const float4 geo = table[3 * q + 2];
          // phase_index = fma(u, l, v*m) + w*n (degridder fusion)
          const float pidx = fma_(c.u, geo.x, c.v * geo.y) + c.w * geo.z;
          const float A = fma_(pidx, k[0], -geo.w);
          const float R = revolutions(A);
#pragma unroll
          for (int j = 0; j < CG; ++j) {
            const float ph = fma_(pidx, k[j], -geo.w);
            const float r = fma_(ph - A, kInv2PiHi, R);
            float sn, cs;
            sincos_rev(r, &sn, &cs);
            cmac4(acc[j], pa, pb, cs, sn);
          }
        }
      }
    }

    if (active) {
      float4 *dst = reinterpret_cast<float4 *>(
          visibilities + (row * C + c0) * 4);
#pragma unroll
      for (int j = 0; j < CG; ++j) {
        if (c0 + j < C) {
          dst[2 * j] = make_float4(acc[j][0], acc[j][1], acc[j][2], acc[j][3]);
          dst[2 * j + 1] =
              make_float4(acc[j][4], acc[j][5], acc[j][6], acc[j][7]);
        }
      }
    }
  }
}

#define IDG_DEGRIDDER(S_, CG_) \
  reinterpret_cast<const void *>(&kernel_degridder_mi355x<S_, CG_>)

KernelChoice select_degridder(const Problem &p) {
  KernelChoice k;
  k.grid = p.nr_subgrids;
  k.block = kBlock;
  const int C = p.nr_channels;
  const int cg = C % 8 == 0 ? 8 : (C % 4 == 0 ? 4 : (C >= 8 ? 8 : 4));
  const bool s32 = p.subgrid_size == 32, s64 = p.subgrid_size == 64;
  if (cg == 8) {
    k.func = s32 ? IDG_DEGRIDDER(32, 8)
                 : (s64 ? IDG_DEGRIDDER(64, 8) : IDG_DEGRIDDER(0, 8));
  } else {
    k.func = s32 ? IDG_DEGRIDDER(32, 4)
                 : (s64 ? IDG_DEGRIDDER(64, 4) : IDG_DEGRIDDER(0, 4));
  }
  k.name = s32 ? "degridder_mi355x_s32"
               : (s64 ? "degridder_mi355x_s64" : "degridder_mi355x_generic");
  return k;
}

}  // namespace idg_mi355x

namespace hip {

void p_run_degridder() {
  idg_mi355x::Problem p;
  p.subgrid_size = static_cast<int>(get_env_var("SUBGRID_SIZE", 32));
  p.nr_channels = static_cast<int>(get_env_var("NR_CHANNELS", 16));
  const idg_mi355x::KernelChoice k = idg_mi355x::select_degridder(p);
  p_run_degridder_(k.func, "degridder_mi355x", k.block);
}

void c_run_degridder(
    int nr_subgrids, int grid_size, int subgrid_size, float image_size,
    float w_step_in_lambda, int nr_channels, int nr_stations,
    idg::Array2D<idg::UVWCoordinate<float>> &uvw,
    idg::Array1D<float> &wavenumbers,
    idg::Array3D<idg::Visibility<std::complex<float>>> &visibilities,
    idg::Array2D<float> &spheroidal,
    idg::Array4D<idg::Matrix2x2<std::complex<float>>> &aterms,
    idg::Array1D<idg::Metadata> &metadata,
    idg::Array4D<std::complex<float>> &subgrids) {
  c_run_degridder_(nr_subgrids, grid_size, subgrid_size, image_size,
                   w_step_in_lambda, nr_channels, nr_stations, uvw,
                   wavenumbers, visibilities, spheroidal, aterms, metadata,
                   subgrids, nullptr, idg_mi355x::kBlock);
}

}  // namespace hip
