// sequential_mi355x.hip.cpp -- the order-preserving ("sequential") gridder
// and degridder for MI355X (gfx950): the reference's CPU arithmetic, bit for
// bit, on the GPU.
//
// The default kernels (gridder_mi355x.hip.cpp, degridder_mi355x.hip.cpp) run
// the complex MAC on the matrix cores in K-blocked f16x2-split GEMMs: closer
// to the exact sum of the reference's phases than the reference itself, but
// in a different rounding sequence.  At T x C = 32,768 (BASELINE configs[2])
// the reference metric puts that 1.30e-5 from the reference's own output
// (DESIGN.md §3.1), because the reference's output is itself 1.27e-5 from
// exact.  These kernels instead repeat the reference's rounding sequence:
//
//   gridder   (app/CPU/kernels/gridder_reference.cpp:42-110)
//     per pixel, per correlation: for t, for c (in that order)
//       phase   = fma(-phase_index, k_c, phase_offset)          (f32, a3)
//       (s, c)  = glibc sincosf(phase)      (common/sincosf_glibc.hpp)
//       prod    = (fma(vr, c, -(vi*s)), fma(vi, c, vr*s))        (cmul_b)
//       pixel  += prod                               (two f32 adds)
//     then A1^H P A2 with the reference's product forms, then * taper;
//   degridder (app/CPU/kernels/degridder_reference.cpp:35-125)
//     P' = A1 (sph P) A2^H per pixel, then per (t, c): for y, for x (in that
//     order) sum += P'(y, x) * (s, c) (cmul_b), phase = fma(phase_index, k,
//     -phase_offset) with phase_index = fma(u, l, v*m) + w*n.
//
// Every operation is the one GCC emitted for the reference (oracle/
// idg_oracle.c is the same arithmetic restated in C and is bit-exact to the
// reference build on every golden case), so the outputs are the reference's
// bits.  Selected by IDG_GRIDDER_IMPL=sequential / IDG_DEGRIDDER_IMPL=
// sequential (read per call, util.hpp select_*); same 13-argument kernel ABI
// and launch shape (grid = nr_subgrids, block = 256) as every other kernel.
//
// Layout of the work:
//  * gridder: one workgroup of 256 lanes per subgrid; a lane owns pixels
//    whole (all four correlations, 8 f32 accumulators each), loops t then c
//    with the timestep's uvw and the visibility (wave-uniform: scalar loads)
//    and sums in the reference order.  Mirror pairs (even S, w = 0 and
//    w_offset = 0 on the subgrid, as the MFMA kernels): pixel npix-1-p has
//    the exact negated phase, and glibc's sincosf is exactly odd / even
//    (tests/test_host.py: every finite float), so one sincosf serves both;
//    the lane checks the negation bit for bit per phasor and evaluates the
//    mirror's own sincosf where it does not hold.
//  * degridder: one workgroup per subgrid; the A-termed, tapered pixels and
//    their (l, m, n, phase_offset) go to LDS in chunks of 1,024 pixels; a
//    lane owns (t, c) visibilities and sums over the pixels in y, x order,
//    its partial sums carried from one chunk to the next.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <string>

#include "../util.hpp"
#include "common/sincosf_glibc.hpp"
#include "device.hpp"

namespace idg_mi355x {

namespace {

constexpr int kSeqBlock = 256;
constexpr int kSeqStage = 512;  // gridder: (t, c) items per LDS block

__device__ __forceinline__ unsigned fbits(float x) {
  return __builtin_bit_cast(unsigned, x);
}

// Packed f32 pairs (re, im): v_pk_mul_f32 / v_pk_fma_f32 / v_pk_add_f32
// round each half exactly as the scalar instruction does, so the packed MACs
// below are the reference's scalar arithmetic two lanes at a time (round 6:
// one packed instruction issues in 4.7-4.8 cycles against 2.5-2.7 for each
// of the two scalar ones, profiles/r02/rates/).
typedef float f2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f2v pk_fma(f2v a, f2v b, f2v c) {
  return __builtin_elementwise_fma(a, b, c);
}

// pixel += V_p * (c, s) for the 4 correlations, the reference's product form
// (gridder_reference.cpp:79; oracle cmul_b) then the two f32 adds:
//   re = fma(vr, c, -(vi * s)),  im = fma(vi, c, vr * s),
// with t = (vi, vr) * (-s, s) = (-(vi * s), vr * s) exactly (negation is
// exact), so re, im = fma((vr, vi), (c, c), t) in one packed FMA.
__device__ __forceinline__ void mac_ref(f2v (&a)[4], const float4 &va,
                                        const float4 &vb, float cs, float sn) {
  const f2v v[4] = {{va.x, va.y}, {va.z, va.w}, {vb.x, vb.y}, {vb.z, vb.w}};
  const f2v ns = {-sn, sn}, cc = {cs, cs};
#pragma unroll
  for (int q = 0; q < 4; ++q)
    a[q] = a[q] + pk_fma(v[q], cc, v[q].yx * ns);
}

// The same for a base pixel (phasor (c, s)) and its mirror (phasor (c, -s),
// exactly: the mirror phase is the negated base phase and sincosf is odd /
// even), sharing the products: the mirror's t is (vi * s, -(vr * s)) = -t
// exactly, so its re, im = fma((vr, vi), (c, c), -t) (the packed FMA's
// negate modifiers).
__device__ __forceinline__ void mac_ref_pair(f2v (&a)[4], f2v (&b)[4],
                                             const float4 &va,
                                             const float4 &vb, float cs,
                                             float sn) {
  const f2v v[4] = {{va.x, va.y}, {va.z, va.w}, {vb.x, vb.y}, {vb.z, vb.w}};
  const f2v ns = {-sn, sn}, cc = {cs, cs};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const f2v t = v[q].yx * ns;
    a[q] = a[q] + pk_fma(v[q], cc, t);
    b[q] = b[q] + pk_fma(v[q], cc, -t);
  }
}

// Output pixel p: sph * (A1^H P A2) with the reference's forms (common/
// math.hpp apply_aterm_gridder), correlation-planar store.
__device__ __forceinline__ void seq_store_pixel(
    const f2v (&a)[4], int p, int S, int npix, const SubgridSetup &g,
    int nr_stations, const float *__restrict__ spheroidal,
    const float2 *__restrict__ aterms, float2 *__restrict__ out) {
  const int y = p / S, x = p - y * S;
  idg::cfloat pix[4], a1[4], a2[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) pix[q] = {a[q].x, a[q].y};
  load_jones(aterm_ptr(aterms, nr_stations, S, g.aterm_index, g.station1, y,
                       x), a1);
  load_jones(aterm_ptr(aterms, nr_stations, S, g.aterm_index, g.station2, y,
                       x), a2);
  idg::apply_aterm_gridder(pix, a1, a2);
  const float sph = spheroidal[p];
#pragma unroll
  for (int q = 0; q < 4; ++q)
    out[static_cast<size_t>(q) * npix + p] =
        make_float2(pix[q].re * sph, pix[q].im * sph);
}

// Pixel geometry as the reference gridder forms it (gridder_reference.cpp:
// 49-64): l, m via double, n = compute_n, phase_offset = fma(w_o, n,
// fma(u_o, l, v_o*m)) -- with n on mirror subgrids too (w_offset = 0 there,
// but fma(0, n, x) is formed exactly as the reference forms it).
__device__ __forceinline__ void seq_geometry(int p, int S, float image_size,
                                             const SubgridSetup &g, float &l,
                                             float &m, float &n, float &poff) {
  const int y = p / S, x = p - y * S;
  l = idg::compute_l(x, S, image_size);
  m = idg::compute_m(y, S, image_size);
  n = idg::compute_n(l, m);
  poff = fma_(g.w_offset, n, fma_(g.u_offset, l, g.v_offset * m));
}

// NP base pixels of this lane (base[i] < nbase; clamped duplicates are
// computed and not stored) and, with MIRROR, their mirrors npix-1-base[i].
template <int NP, bool MIRROR>
__device__ __forceinline__ void seq_grid_pixels(
    const int (&base)[NP], int nbase, int S, int npix, float image_size,
    const SubgridSetup &g, int C, int nr_stations,
    const idg::UVWCoordinate<float> *__restrict__ uvw,
    const float *__restrict__ wavenumbers,
    const float2 *__restrict__ visibilities,
    const float *__restrict__ spheroidal, const float2 *__restrict__ aterms,
    float2 *__restrict__ out, const idg::SincosfWindow *__restrict__ win,
    float4 *__restrict__ st_vis, float4 *__restrict__ st_uvwk) {
  constexpr int NQ = MIRROR ? 2 * NP : NP;
  float l[NQ], m[NQ], n[NQ], po[NQ];
  f2v acc[NQ][4];
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    const int b = min(base[i % NP], nbase - 1);
    const int p = i < NP ? b : npix - 1 - b;
    seq_geometry(p, S, image_size, g, l[i], m[i], n[i], po[i]);
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f2v{0.0f, 0.0f};
  }
  // The visibilities come through LDS, kSeqStage (t, c) items at a time,
  // in the reference's t-then-c order: the workgroup stages a block (both
  // correlation quads of each item and its (u, v, w, k)) between two
  // barriers, and every wave walks it.  Loaded per wave from global memory
  // instead (wave-uniform scalar loads), each channel waited on its loads
  // at the top of the loop -- the lgkm counter they share with the LDS
  // reads of the sincosf windows makes every window wait a wait for them
  // too (the gridder issued at 0.90 of its instruction stream, round 6).
  const long long items = static_cast<long long>(g.nr_timesteps) * C;
  const float4 *vis4 = reinterpret_cast<const float4 *>(visibilities) +
                       g.time_offset * C * 2;
  float pidx[NQ];
  for (long long i0 = 0; i0 < items; i0 += kSeqStage) {
    const int ne = static_cast<int>(items - i0 < kSeqStage ? items - i0 : kSeqStage);
    __syncthreads();  // the previous block's readers are done
    for (int e = threadIdx.x; e < ne; e += kSeqBlock) {
      const long long it = i0 + e;
      const int t = static_cast<int>(it / C), c = static_cast<int>(it % C);
      st_vis[2 * e] = vis4[it * 2];
      st_vis[2 * e + 1] = vis4[it * 2 + 1];
      const idg::UVWCoordinate<float> c3 = uvw[g.time_offset + t];
      st_uvwk[e] = make_float4(c3.u, c3.v, c3.w, wavenumbers[c]);
    }
    __syncthreads();
    int ch = static_cast<int>(i0 % C);
    for (int e = 0; e < ne; ++e) {
      const float4 uvwk = st_uvwk[e];
      const float4 va = st_vis[2 * e], vb = st_vis[2 * e + 1];
      if (ch == 0 || e == 0) {  // a new timestep (or block): phase_index
#pragma unroll
        for (int i = 0; i < NQ; ++i)
          pidx[i] = fma_(uvwk.z, n[i], fma_(uvwk.x, l[i], uvwk.y * m[i]));
      }
      ch = ch + 1 == C ? 0 : ch + 1;
      const float k = uvwk.w;
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        const float ph = fma_(-pidx[i], k, po[i]);
        float sn, cs;
        idg::sincosf_glibc_dev(ph, &sn, &cs, win);
        if constexpr (MIRROR) {
          // the mirror's own phase, formed as the reference forms it; where
          // it is the exact negation (every lane of every wave on the
          // benchmark data) one sincosf and one set of products serve both
          const float phm = fma_(-pidx[NP + i], k, po[NP + i]);
          const bool neg = fbits(phm) == (fbits(ph) ^ 0x80000000u);
          if (__all(neg)) {
            mac_ref_pair(acc[i], acc[NP + i], va, vb, cs, sn);
          } else {
            float snm = -sn, csm = cs;
            if (!neg) idg::sincosf_glibc_dev(phm, &snm, &csm, win);
            mac_ref(acc[i], va, vb, cs, sn);
            mac_ref(acc[NP + i], va, vb, csm, snm);
          }
        } else {
          mac_ref(acc[i], va, vb, cs, sn);
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    if (base[i % NP] >= nbase) continue;
    const int p = i < NP ? base[i] : npix - 1 - base[i - NP];
    seq_store_pixel(acc[i], p, S, npix, g, nr_stations, spheroidal, aterms,
                    out);
  }
}

}  // namespace

// grid = nr_subgrids, block = kSeqBlock; the 13-argument kernel ABI.
template <int S_CT>
__global__ void __launch_bounds__(kSeqBlock)
    kernel_gridder_sequential_mi355x(
        const int grid_size, int subgrid_size, float image_size,
        float w_step_in_lambda, int nr_channels, int nr_stations,
        const idg::UVWCoordinate<float> *__restrict__ uvw,
        const float *__restrict__ wavenumbers,
        const float2 *__restrict__ visibilities,
        const float *__restrict__ spheroidal,
        const float2 *__restrict__ aterms,
        const idg::Metadata *__restrict__ metadata,
        float2 *__restrict__ subgrids) {
  __shared__ idg::SincosfWindow win[idg::kSincosfWindows];
  __shared__ float4 st_vis[kSeqStage * 2];  // staged visibilities (24 KB
  __shared__ float4 st_uvwk[kSeqStage];     // with their (u, v, w, k))
  const int S = S_CT > 0 ? S_CT : subgrid_size;
  const int npix = S * S;
  const int s = xcd_subgrid(blockIdx.x, gridDim.x);
  const int tid = threadIdx.x;
  idg::sincosf_windows_to_lds(win, tid);  // the barrier below publishes it
  const SubgridSetup g = setup_subgrid(metadata, s, grid_size, S, image_size,
                                       w_step_in_lambda);
  float2 *out = subgrids + static_cast<size_t>(s) * 4 * npix;
  bool w_nonzero = false;
  for (int t = tid; t < g.nr_timesteps; t += kSeqBlock)
    w_nonzero |= uvw[g.time_offset + t].w != 0.0f;
  const bool mirror = __syncthreads_or(w_nonzero) == 0 && S % 2 == 0 &&
                      g.w_offset == 0.0f;
  if (mirror) {
    constexpr int NP = 2;
    const int half = npix / 2;
    for (int tile = 0; tile < half; tile += kSeqBlock * NP) {
      int base[NP];
#pragma unroll
      for (int i = 0; i < NP; ++i) base[i] = tile + i * kSeqBlock + tid;
      seq_grid_pixels<NP, true>(base, half, S, npix, image_size, g,
                                nr_channels, nr_stations, uvw, wavenumbers,
                                visibilities, spheroidal, aterms, out, win,
                                st_vis, st_uvwk);
    }
    return;
  }
  constexpr int NP = 4;
  for (int tile = 0; tile < npix; tile += kSeqBlock * NP) {
    int base[NP];
#pragma unroll
    for (int i = 0; i < NP; ++i) base[i] = tile + i * kSeqBlock + tid;
    seq_grid_pixels<NP, false>(base, npix, S, npix, image_size, g,
                               nr_channels, nr_stations, uvw, wavenumbers,
                               visibilities, spheroidal, aterms, out, win,
                               st_vis, st_uvwk);
  }
}

// ---------------------------------------------------------------------------
// Degridder.
// ---------------------------------------------------------------------------
constexpr int kSeqChunk = 1024;  // pixels per LDS chunk
constexpr int kSeqItems = 4;     // (t, c) visibilities per lane per pass

// One LDS chunk of np pixels, in y, x order, into the lane's kSeqItems
// partial sums.
//  WZ      every item's w is +0.0 (the wave's choice), so w * n is +0 (n =
//          compute_n is finite and >= +0) and phase_index = fma(u, l, v*m) +
//          w*n is fma(u, l, v*m) + 0.0f bit for bit, one multiply fewer;
//  SAME_T  the lane's items are consecutive channels of one timestep (C a
//          multiple of kSeqItems), so they share phase_index: formed once
//          per pixel instead of once per item.
template <bool WZ, bool SAME_T>
__device__ __forceinline__ void seq_degrid_chunk(
    int np, const float4 *__restrict__ lds_geo,
    const float4 *__restrict__ lds_pix, const float (&u)[kSeqItems],
    const float (&v)[kSeqItems], const float (&w)[kSeqItems],
    const float (&k)[kSeqItems], f2v (&sum)[kSeqItems][4],
    const idg::SincosfWindow *__restrict__ win) {
  for (int e = 0; e < np; ++e) {
    const float4 geo = lds_geo[e];
    const float4 pa = lds_pix[2 * e], pb = lds_pix[2 * e + 1];
    float pidx[kSeqItems];
#pragma unroll
    for (int j = 0; j < kSeqItems; ++j) {
      // phase_index = fma(u, l, v*m) + w*n
      if (SAME_T && j > 0) {
        pidx[j] = pidx[0];
      } else {
        pidx[j] = fma_(u[j], geo.x, v[j] * geo.y) +
                  (WZ ? 0.0f : w[j] * geo.z);
      }
    }
#pragma unroll
    for (int j = 0; j < kSeqItems; ++j) {
      const float ph = fma_(pidx[j], k[j], -geo.w);  // fma(pidx, k, -poff)
      float sn, cs;
      idg::sincosf_glibc_dev(ph, &sn, &cs, win);
      mac_ref(sum[j], pa, pb, cs, sn);
    }
  }
}

template <int S_CT>
__global__ void __launch_bounds__(kSeqBlock)
    kernel_degridder_sequential_mi355x(
        const int grid_size, int subgrid_size, float image_size,
        float w_step_in_lambda, int nr_channels, int nr_stations,
        const idg::UVWCoordinate<float> *__restrict__ uvw,
        const float *__restrict__ wavenumbers,
        float2 *__restrict__ visibilities,
        const float *__restrict__ spheroidal,
        const float2 *__restrict__ aterms,
        const idg::Metadata *__restrict__ metadata,
        const float2 *__restrict__ subgrids) {
  __shared__ float4 lds_pix[kSeqChunk * 2];  // P' of the chunk: xx|xy, yx|yy
  __shared__ float4 lds_geo[kSeqChunk];      // (l, m, n, phase_offset)
  __shared__ idg::SincosfWindow win[idg::kSincosfWindows];
  const int S = S_CT > 0 ? S_CT : subgrid_size;
  const int npix = S * S;
  const int s = xcd_subgrid(blockIdx.x, gridDim.x);
  const int tid = threadIdx.x;
  // published by the chunk loop's first barrier, before any phasor
  idg::sincosf_windows_to_lds(win, tid);
  const SubgridSetup g = setup_subgrid(metadata, s, grid_size, S, image_size,
                                       w_step_in_lambda);
  const int C = nr_channels;
  const float2 *sg = subgrids + static_cast<size_t>(s) * 4 * npix;
  const long long items = static_cast<long long>(g.nr_timesteps) * C;
  // C a multiple of kSeqItems: a lane's items are kSeqItems consecutive
  // channels of one timestep (all valid or all past the end together, since
  // items and every i0 are multiples of kSeqItems); otherwise kSeqBlock
  // apart
  const bool same_t = C % kSeqItems == 0;
  for (long long i0 = 0; i0 < items; i0 += kSeqBlock * kSeqItems) {
    f2v sum[kSeqItems][4];
    float u[kSeqItems], v[kSeqItems], w[kSeqItems], k[kSeqItems];
#pragma unroll
    for (int j = 0; j < kSeqItems; ++j) {
      const long long it =
          min(i0 + (same_t ? kSeqItems * tid + j : j * kSeqBlock + tid),
              items - 1);
      const int t = static_cast<int>(it / C), c = static_cast<int>(it % C);
      const idg::UVWCoordinate<float> c3 = uvw[g.time_offset + t];
      u[j] = c3.u;
      v[j] = c3.v;
      w[j] = c3.w;
      k[j] = wavenumbers[c];
#pragma unroll
      for (int q = 0; q < 4; ++q) sum[j][q] = f2v{0.0f, 0.0f};
    }
    bool wz = true;
#pragma unroll
    for (int j = 0; j < kSeqItems; ++j)
      wz = wz && __builtin_bit_cast(unsigned, w[j]) == 0u;
    for (int p0 = 0; p0 < npix; p0 += kSeqChunk) {
      const int np = min(kSeqChunk, npix - p0);
      __syncthreads();  // the previous chunk's readers are done
      for (int e = tid; e < np; e += kSeqBlock) {
        const int p = p0 + e, y = p / S, x = p - y * S;
        const float sph = spheroidal[p];
        idg::cfloat pix[4], a1[4], a2[4];
#pragma unroll
        for (int cr = 0; cr < 4; ++cr) {
          const float2 q = sg[static_cast<size_t>(cr) * npix + p];
          pix[cr] = {sph * q.x, sph * q.y};
        }
        load_jones(aterm_ptr(aterms, nr_stations, S, g.aterm_index,
                             g.station1, y, x), a1);
        load_jones(aterm_ptr(aterms, nr_stations, S, g.aterm_index,
                             g.station2, y, x), a2);
        idg::apply_aterm_degridder(pix, a1, a2);
        const float l = idg::compute_l(x, S, image_size);
        const float m = idg::compute_m(y, S, image_size);
        const float n = idg::compute_n(l, m);
        // phase_offset = fma(u_o, l, v_o*m) + w_o*n (degridder fusion)
        const float poff = fma_(g.u_offset, l, g.v_offset * m) + g.w_offset * n;
        lds_pix[2 * e] = make_float4(pix[0].re, pix[0].im, pix[1].re, pix[1].im);
        lds_pix[2 * e + 1] =
            make_float4(pix[2].re, pix[2].im, pix[3].re, pix[3].im);
        lds_geo[e] = make_float4(l, m, n, poff);
      }
      __syncthreads();
      if (same_t) {
        if (__all(wz))
          seq_degrid_chunk<true, true>(np, lds_geo, lds_pix, u, v, w, k, sum,
                                       win);
        else
          seq_degrid_chunk<false, true>(np, lds_geo, lds_pix, u, v, w, k, sum,
                                        win);
      } else {
        if (__all(wz))
          seq_degrid_chunk<true, false>(np, lds_geo, lds_pix, u, v, w, k, sum,
                                        win);
        else
          seq_degrid_chunk<false, false>(np, lds_geo, lds_pix, u, v, w, k,
                                         sum, win);
      }
    }
#pragma unroll
    for (int j = 0; j < kSeqItems; ++j) {
      const long long it =
          i0 + (same_t ? kSeqItems * tid + j : j * kSeqBlock + tid);
      if (it >= items) continue;
      const int t = static_cast<int>(it / C), c = static_cast<int>(it % C);
      float4 *dst = reinterpret_cast<float4 *>(
          visibilities + ((g.time_offset + t) * C + c) * 4);
      dst[0] = make_float4(sum[j][0].x, sum[j][0].y, sum[j][1].x, sum[j][1].y);
      dst[1] = make_float4(sum[j][2].x, sum[j][2].y, sum[j][3].x, sum[j][3].y);
    }
  }
}

// The sequential kernels of subgrid size S (32, 64, or 0 = runtime S).
const void *sequential_gridder(int S) {
  switch (S) {
    case 32: return reinterpret_cast<const void *>(
        &kernel_gridder_sequential_mi355x<32>);
    case 64: return reinterpret_cast<const void *>(
        &kernel_gridder_sequential_mi355x<64>);
    default: return reinterpret_cast<const void *>(
        &kernel_gridder_sequential_mi355x<0>);
  }
}

const void *sequential_degridder(int S) {
  switch (S) {
    case 32: return reinterpret_cast<const void *>(
        &kernel_degridder_sequential_mi355x<32>);
    case 64: return reinterpret_cast<const void *>(
        &kernel_degridder_sequential_mi355x<64>);
    default: return reinterpret_cast<const void *>(
        &kernel_degridder_sequential_mi355x<0>);
  }
}

int sequential_block() { return kSeqBlock; }

}  // namespace idg_mi355x
