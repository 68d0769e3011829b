// gridder_mi355x.hip.cpp -- IDG gridder for MI355X (gfx950).
//
// Replaces the reference's app/HIP/kernels/gridder_*.hip.cpp behind the same
// kernel-TU contract (hip::p_run_gridder, hip::c_run_gridder; the harness
// forward-declares them at tests/gridder_common.cpp:13-31) and the same
// 13-argument kernel ABI / launch shape (grid = nr_subgrids, block = 256,
// reference app/HIP/util.cpp:237-244), so it also runs under the reference's
// own util.cpp.  It computes cpu::kernel_gridder_reference
// (app/CPU/kernels/gridder_reference.cpp:6-114):
//
//   P_p(y,x) = sum_t sum_c V_p(t,c) * exp(i*phase),
//   phase    = fl(phase_offset(y,x) - phase_index(t,y,x) * k_c)   [one FMA]
//   subgrid  = sph(y,x) * A1^H P A2
//
// Design:
//  * one workgroup (4 wave64) per subgrid; each lane owns PPT pixels spread
//    256 apart, so every visibility is a wave-uniform operand: uvw, k_c and
//    the 8 floats of V(t,c) are scalar loads (s_load) feeding v_fma directly,
//    with no LDS traffic at all;
//  * the fp32 phase is formed exactly as the reference rounds it, then
//    reduced without losing its low bits: once per (pixel, timestep, channel
//    block) the block's first phase A is converted to revolutions R with a
//    Dekker-split 1/(2*pi) (device.hpp:revolutions); every other channel's
//    phase is fl(phase) = A + d with d computed exactly, and its revolutions
//    are R + d/(2*pi), small enough for v_sin_f32/v_cos_f32 (which take
//    revolutions);
//  * 4 correlations x complex MAC = 16 v_fma_f32 per (pixel, t, c) with the
//    visibility operands in SGPRs;
//  * the A-term sandwich, taper and store happen once per pixel at the end.
#include <hip/hip_runtime.h>

#include "../util.hpp"
#include "device.hpp"
#include "lib-hip.hpp"

namespace idg_mi355x {

// S_CT: subgrid size known at compile time (0 = runtime).
// PPT : pixels per lane.   CB: channels per phase anchor.
template <int S_CT, int PPT, int CB>
__global__ void __launch_bounds__(kBlock)
    kernel_gridder_mi355x(const int grid_size, int subgrid_size,
                          float image_size, float w_step_in_lambda,
                          int nr_channels, int nr_stations,
                          const idg::UVWCoordinate<float> *__restrict__ uvw,
                          const float *__restrict__ wavenumbers,
                          const float2 *__restrict__ visibilities,
                          const float *__restrict__ spheroidal,
                          const float2 *__restrict__ aterms,
                          const idg::Metadata *__restrict__ metadata,
                          float2 *__restrict__ subgrids) {
  const int S = S_CT > 0 ? S_CT : subgrid_size;
  const int npix = S * S;
  const int s = blockIdx.x;
  const SubgridSetup g = setup_subgrid(metadata, s, grid_size, S, image_size,
                                       w_step_in_lambda);
  const int C = nr_channels;

  for (int tile = 0; tile < npix; tile += kBlock * PPT) {
    float l[PPT], m[PPT], n[PPT], poff[PPT];
    float acc[PPT][8];
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const int p = min(tile + i * kBlock + static_cast<int>(threadIdx.x),
                        npix - 1);
      const int y = p / S, x = p - (p / S) * S;
      l[i] = idg::compute_l(x, S, image_size);
      m[i] = idg::compute_m(y, S, image_size);
      n[i] = idg::compute_n(l[i], m[i]);
      // phase_offset = u_o*l + v_o*m + w_o*n, fused as fma(w_o,n,fma(u_o,l,v_o*m))
      poff[i] = fma_(g.w_offset, n[i], fma_(g.u_offset, l[i], g.v_offset * m[i]));
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = 0.0f;
    }

    for (int t = 0; t < g.nr_timesteps; ++t) {
      const long long row = g.time_offset + t;
      const idg::UVWCoordinate<float> c = uvw[row];
      float pidx[PPT];
#pragma unroll
      for (int i = 0; i < PPT; ++i)
        pidx[i] = fma_(c.w, n[i], fma_(c.u, l[i], c.v * m[i]));
      const float4 *vrow =
          reinterpret_cast<const float4 *>(visibilities + row * C * 4);

      for (int cb = 0; cb < C; cb += CB) {
        const int ce = min(cb + CB, C);
        // Phase anchor for this channel block: A = the block's first phase,
        // R = its revolutions (accurate to ~3e-8).
        const float k0 = wavenumbers[cb];
        float A[PPT], R[PPT];
#pragma unroll
        for (int i = 0; i < PPT; ++i) {
          A[i] = fma_(-pidx[i], k0, poff[i]);
          R[i] = revolutions(A[i]);
        }
        for (int ch = cb; ch < ce; ++ch) {
          const float k = wavenumbers[ch];
          const float4 va = vrow[2 * ch];      // xx, xy
          const float4 vb = vrow[2 * ch + 1];  // yx, yy
#pragma unroll
          for (int i = 0; i < PPT; ++i) {
            // The reference's rounded phase, then its revolutions.
            const float ph = fma_(-pidx[i], k, poff[i]);
            const float r = fma_(ph - A[i], kInv2PiHi, R[i]);
            float sn, cs;
            sincos_rev(r, &sn, &cs);
            float *a = acc[i];
            a[0] = fma_(va.x, cs, a[0]); a[0] = fma_(-va.y, sn, a[0]);
            a[1] = fma_(va.x, sn, a[1]); a[1] = fma_(va.y, cs, a[1]);
            a[2] = fma_(va.z, cs, a[2]); a[2] = fma_(-va.w, sn, a[2]);
            a[3] = fma_(va.z, sn, a[3]); a[3] = fma_(va.w, cs, a[3]);
            a[4] = fma_(vb.x, cs, a[4]); a[4] = fma_(-vb.y, sn, a[4]);
            a[5] = fma_(vb.x, sn, a[5]); a[5] = fma_(vb.y, cs, a[5]);
            a[6] = fma_(vb.z, cs, a[6]); a[6] = fma_(-vb.w, sn, a[6]);
            a[7] = fma_(vb.z, sn, a[7]); a[7] = fma_(vb.w, cs, a[7]);
          }
        }
      }
    }

    // Epilogue: P <- sph * A1^H P A2, correlation-planar store.
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const int p = tile + i * kBlock + static_cast<int>(threadIdx.x);
      if (p >= npix) continue;
      const int y = p / S, x = p - (p / S) * S;
      idg::cfloat pix[4], a1[4], a2[4];
      for (int q = 0; q < 4; ++q) pix[q] = {acc[i][2 * q], acc[i][2 * q + 1]};
      load_jones(aterm_ptr(aterms, nr_stations, S, g.aterm_index, g.station1,
                           y, x), a1);
      load_jones(aterm_ptr(aterms, nr_stations, S, g.aterm_index, g.station2,
                           y, x), a2);
      idg::apply_aterm_gridder(pix, a1, a2);
      const float sph = spheroidal[p];
      float2 *dst = subgrids + static_cast<size_t>(s) * 4 * npix + p;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        dst[static_cast<size_t>(q) * npix] =
            make_float2(pix[q].re * sph, pix[q].im * sph);
    }
  }
}

#define IDG_GRIDDER(S_, PPT_, CB_) \
  reinterpret_cast<const void *>(&kernel_gridder_mi355x<S_, PPT_, CB_>)

KernelChoice select_gridder(const Problem &p) {
  KernelChoice k;
  k.grid = p.nr_subgrids;
  k.block = kBlock;
  switch (p.subgrid_size) {
    case 32:
      k.func = IDG_GRIDDER(32, 4, 16);
      k.name = "gridder_mi355x_s32";
      break;
    case 64:
      k.func = IDG_GRIDDER(64, 4, 16);
      k.name = "gridder_mi355x_s64";
      break;
    default:
      k.func = IDG_GRIDDER(0, 2, 16);
      k.name = "gridder_mi355x_generic";
      break;
  }
  return k;
}

}  // namespace idg_mi355x

namespace hip {

void p_run_gridder() {
  idg_mi355x::Problem p;
  p.subgrid_size = static_cast<int>(get_env_var("SUBGRID_SIZE", 32));
  p.nr_channels = static_cast<int>(get_env_var("NR_CHANNELS", 16));
  const idg_mi355x::KernelChoice k = idg_mi355x::select_gridder(p);
  p_run_gridder_(k.func, "gridder_mi355x", k.block);
}

void c_run_gridder(
    int nr_subgrids, int grid_size, int subgrid_size, float image_size,
    float w_step_in_lambda, int nr_channels, int nr_stations,
    idg::Array2D<idg::UVWCoordinate<float>> &uvw,
    idg::Array1D<float> &wavenumbers,
    idg::Array3D<idg::Visibility<std::complex<float>>> &visibilities,
    idg::Array2D<float> &spheroidal,
    idg::Array4D<idg::Matrix2x2<std::complex<float>>> &aterms,
    idg::Array1D<idg::Metadata> &metadata,
    idg::Array4D<std::complex<float>> &subgrids) {
  c_run_gridder_(nr_subgrids, grid_size, subgrid_size, image_size,
                 w_step_in_lambda, nr_channels, nr_stations, uvw, wavenumbers,
                 visibilities, spheroidal, aterms, metadata, subgrids, nullptr,
                 idg_mi355x::kBlock);
}

}  // namespace hip
