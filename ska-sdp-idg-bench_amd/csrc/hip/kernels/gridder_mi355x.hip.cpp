// gridder_mi355x.hip.cpp -- IDG gridder for MI355X (gfx950).
//
// Replaces the reference's app/HIP/kernels/gridder_*.hip.cpp behind the same
// kernel-TU contract (hip::p_run_gridder, hip::c_run_gridder; the harness
// forward-declares them at tests/gridder_common.cpp:13-31) and the same
// 13-argument kernel ABI / launch shape (grid = nr_subgrids, block = the
// kernel's own: 512 lanes for the MFMA kernel, 256 for the VALU kernel;
// reference app/HIP/util.cpp:237-244), so it also runs under the reference's
// own util.cpp.  It computes cpu::kernel_gridder_reference
// (app/CPU/kernels/gridder_reference.cpp:6-114):
//
//   P_p(y,x) = sum_t sum_c V_p(t,c) * exp(i*phase),
//   phase    = fl(phase_offset(y,x) - phase_index(t,y,x) * k_c)   [one FMA]
//   subgrid  = sph(y,x) * A1^H P A2
//
// Design:
//  * one workgroup per subgrid: 8 wave64 (MFMA kernel), 4 (VALU kernel);
//  * the fp32 phase is formed exactly as the reference rounds it and reduced
//    to revolutions without losing its low bits: r = fma(phase, 1/2pi_hi,
//    -m) + c with an integer m per (pixel, timestep, channel block) and c
//    the tail -k * phase_index * (1/2pi - 1/2pi_hi) at the block's first
//    channel; the tail's phase_offset part is applied to each pixel as one
//    phasor exp(i * phase_offset * kPhaseTail) in the epilogue (device.hpp);
//  * default (MODE 1): the complex MAC runs on the matrix cores as f16
//    two-term-split GEMMs (v_mfma_f32_16x16x32_f16, grid_mfma below), pixels
//    x (timestep, channel) x correlation components;
//  * mirror pixels: for even S, pixel (y,x) and (S-1-y, S-1-x) have exactly
//    negated l, m; when w = 0 and the subgrid's w_offset = 0 (every benchmark
//    configuration) their reference phases are exact negatives (fma rounding
//    is sign-symmetric), so one range reduction and one v_sin/v_cos pair
//    serve both pixels.  Subgrids with any w != 0 (or odd S) run the same
//    GEMMs over every pixel with the w-term in the phase;
//  * IDG_GRIDDER_IMPL=valu (MODE 0) selects the all-VALU kernel: 16 FMAs per
//    (pixel, t, c) with wave-uniform visibilities in SGPRs (A/B reference).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <string>

#include "../util.hpp"
#include "device.hpp"
#include "fft.hpp"
#include "lib-hip.hpp"
#include "mfma.hpp"

// MFMA tiles per wave and the waves-per-SIMD launch bound (tuning knobs).
#ifndef IDG_GRID_PT
#define IDG_GRID_PT 4
#endif
#ifndef IDG_GRID_WAVES
#define IDG_GRID_WAVES 4
#endif
// the same bound for the general-only kernel of the two-launch form
#ifndef IDG_GRID_WAVES_GENERAL
#define IDG_GRID_WAVES_GENERAL 4
#endif
// general path (w != 0): X + Y in one accumulator tile, 2 PT tiles per wave
#ifndef IDG_GRID_FUSED_GENERAL
#define IDG_GRID_FUSED_GENERAL 1
#endif
// the B operand's (visibilities') power-of-two scale targets a first-fill
// maximum in [2^(kBS-1), 2^kBS)
#ifndef IDG_GRID_BSCALE
#define IDG_GRID_BSCALE 12
#endif
// non-temporal B-fill loads (A/B; see the fill loop)
#ifndef IDG_GRID_NT_FILL
#define IDG_GRID_NT_FILL 0
#endif
// waves per workgroup of the MFMA kernel (the VALU kernel uses kBlock)
#ifndef IDG_GRID_NW
#define IDG_GRID_NW 8
#endif

namespace idg_mi355x {

namespace {

// acc += V * (c, s) for the 4 correlations.
__device__ __forceinline__ void mac4(float *a, const float4 &va,
                                     const float4 &vb, float cs, float sn) {
  a[0] = fma_(va.x, cs, a[0]); a[0] = fma_(-va.y, sn, a[0]);
  a[1] = fma_(va.x, sn, a[1]); a[1] = fma_(va.y, cs, a[1]);
  a[2] = fma_(va.z, cs, a[2]); a[2] = fma_(-va.w, sn, a[2]);
  a[3] = fma_(va.z, sn, a[3]); a[3] = fma_(va.w, cs, a[3]);
  a[4] = fma_(vb.x, cs, a[4]); a[4] = fma_(-vb.y, sn, a[4]);
  a[5] = fma_(vb.x, sn, a[5]); a[5] = fma_(vb.y, cs, a[5]);
  a[6] = fma_(vb.z, cs, a[6]); a[6] = fma_(-vb.w, sn, a[6]);
  a[7] = fma_(vb.z, sn, a[7]); a[7] = fma_(vb.w, cs, a[7]);
}

// One timestep for NP pixels, each with its own phase (general path).
template <int NP, int CB>
__device__ __forceinline__ void timestep_general(
    const float (&l)[NP], const float (&m)[NP], const float (&n)[NP],
    const float (&poff)[NP], float (&acc)[NP][8],
    const idg::UVWCoordinate<float> c, const float4 *__restrict__ vrow,
    const float *__restrict__ wavenumbers, int C) {
  float pidx[NP];
#pragma unroll
  for (int i = 0; i < NP; ++i)
    pidx[i] = fma_(c.w, n[i], fma_(c.u, l[i], c.v * m[i]));
  for (int cb = 0; cb < C; cb += CB) {
    const int ce = min(cb + CB, C);
    const float k0 = wavenumbers[cb];
    float A[NP], R[NP];
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      A[i] = fma_(-pidx[i], k0, poff[i]);
      R[i] = revolutions(A[i]);
    }
    // Scalar operands of the next channel are requested one iteration
    // ahead so the s_load latency hides under this channel's VALU work.
    float k = k0;
    float4 va = vrow[2 * cb], vb = vrow[2 * cb + 1];
    for (int ch = cb; ch < ce; ++ch) {
      const int nx = min(ch + 1, C - 1);
      const float kn = wavenumbers[nx];
      const float4 van = vrow[2 * nx], vbn = vrow[2 * nx + 1];
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        const float ph = fma_(-pidx[i], k, poff[i]);
        const float r = fma_(ph - A[i], kInv2PiHi, R[i]);
        float sn, cs;
        sincos_rev(r, &sn, &cs);
        mac4(acc[i], va, vb, cs, sn);
      }
      k = kn;
      va = van;
      vb = vbn;
    }
  }
}

// One timestep with w = 0 for NB base pixels and their mirrors (acc[NB+i]):
// phase(mirror) = -phase(base) exactly.
template <int NB, int CB>
__device__ __forceinline__ void timestep_mirror(
    const float (&l)[2 * NB], const float (&m)[2 * NB],
    const float (&poff)[2 * NB], float (&acc)[2 * NB][8],
    const idg::UVWCoordinate<float> c, const float4 *__restrict__ vrow,
    const float *__restrict__ wavenumbers, int C) {
  float pidx[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) pidx[i] = fma_(c.u, l[i], c.v * m[i]);
  for (int cb = 0; cb < C; cb += CB) {
    const int ce = min(cb + CB, C);
    const float k0 = wavenumbers[cb];
    float A[NB], R[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      A[i] = fma_(-pidx[i], k0, poff[i]);
      R[i] = revolutions(A[i]);
    }
    float k = k0;
    float4 va = vrow[2 * cb], vb = vrow[2 * cb + 1];
    for (int ch = cb; ch < ce; ++ch) {
      const int nx = min(ch + 1, C - 1);
      const float kn = wavenumbers[nx];
      const float4 van = vrow[2 * nx], vbn = vrow[2 * nx + 1];
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const float ph = fma_(-pidx[i], k, poff[i]);
        const float r = fma_(ph - A[i], kInv2PiHi, R[i]);
        float sn, cs;
        sincos_rev(r, &sn, &cs);
        mac4(acc[i], va, vb, cs, sn);
        mac4(acc[NB + i], va, vb, cs, -sn);
      }
      k = kn;
      va = van;
      vb = vbn;
    }
  }
}

// Epilogue for one pixel: o = sph * A1^H P A2 (4 correlations) ...
__device__ __forceinline__ void pixel_out(const float (&a)[8], int p, int S,
                                          const SubgridSetup &g,
                                          int nr_stations,
                                          const float *__restrict__ spheroidal,
                                          const float2 *__restrict__ aterms,
                                          float2 (&o)[4]) {
  const int y = p / S, x = p - (p / S) * S;
  idg::cfloat pix[4], a1[4], a2[4];
  for (int q = 0; q < 4; ++q) pix[q] = {a[2 * q], a[2 * q + 1]};
  load_jones(aterm_ptr(aterms, nr_stations, S, g.aterm_index, g.station1, y,
                       x), a1);
  load_jones(aterm_ptr(aterms, nr_stations, S, g.aterm_index, g.station2, y,
                       x), a2);
  idg::apply_aterm_gridder(pix, a1, a2);
  const float sph = spheroidal[p];
#pragma unroll
  for (int q = 0; q < 4; ++q) o[q] = make_float2(pix[q].re * sph, pix[q].im * sph);
}

// ... and its correlation-planar store.
__device__ __forceinline__ void store_pixel(
    const float (&a)[8], int p, int S, int npix, const SubgridSetup &g,
    int nr_stations, const float *__restrict__ spheroidal,
    const float2 *__restrict__ aterms, float2 *__restrict__ out) {
  float2 o[4];
  pixel_out(a, p, S, g, nr_stations, spheroidal, aterms, o);
#pragma unroll
  for (int q = 0; q < 4; ++q) out[static_cast<size_t>(q) * npix + p] = o[q];
}

// W_TERMS = false: the caller guarantees w_offset = 0 (mirror subgrids), so
// phase_offset = fma(0, n, x) = x and n (a divide and a square root) is not
// formed; n is returned as 0.
template <bool W_TERMS = true>
__device__ __forceinline__ void pixel_geometry(int p, int S, float image_size,
                                               const SubgridSetup &g,
                                               float &l, float &m, float &n,
                                               float &poff) {
  const int y = p / S, x = p - (p / S) * S;
  l = idg::compute_l(x, S, image_size);
  m = idg::compute_m(y, S, image_size);
  // phase_offset = fma(w_o, n, fma(u_o, l, v_o*m))
  if constexpr (W_TERMS) {
    n = idg::compute_n(l, m);
    poff = fma_(g.w_offset, n, fma_(g.u_offset, l, g.v_offset * m));
  } else {
    n = 0.0f;
    poff = fma_(g.u_offset, l, g.v_offset * m);
  }
}


// ---------------------------------------------------------------------------
// MFMA mirror path (even S, w = 0 on every timestep, w_offset = 0).
//
// For a base pixel with phasor (c, s) = exp(i*phase) and its mirror (phase
// exactly negated), the contribution of a visibility V is
//   base   += X + Y,   mirror += X - Y,   X = c * Bc,  Y = s * Bs,
// with Bc = (V.re | V.im) and Bs = (-V.im | V.re) per correlation.  X and Y
// are two dense GEMMs per 16-pixel tile (v_mfma_f32_16x16x32_f16):
//   X[pixel][col] += sum_k Ac[pixel][k] * Bc[k][col]      (Y likewise)
// K = 16 items (4 timesteps x 4 channels) x {hi, lo} of the f16-split phasor
// component; B columns = 8 components [hi | lo] of the f16-split visibility.
// Lane l = (group g = l/16, pixel/column l%16): group g takes timestep 4q+g of
// timestep quad q and 4 consecutive channels, so the lane's K-block is
//   [cA_h, cB_h, cA_l, cB_l, cC_h, cD_h, cC_l, cD_l]
// (split_pair on channel pairs: one v_cvt_pk + two v_fma_mix per pair) and
// B's rows for it are (bcA, bcB, bcA, bcB, bcC, bcD, bcC, bcD): 4 dwords
// (x, x, y, y) per lane, stored pre-expanded in LDS.  Per phasor: 1 packed
// phase instruction, v_sin + v_cos, 3 split instructions, half an MFMA.
// ---------------------------------------------------------------------------
#ifndef IDG_GRID_KSBUF
#define IDG_GRID_KSBUF 32
#endif
constexpr int kKsBuf = IDG_GRID_KSBUF;  // K-steps (16 items each) of B fragments per fill

// NW waves per workgroup, AT 16 x 16 accumulator tiles per wave (mirror
// path: X and Y of PT pixel tiles, AT = 2 PT; general path: one fused X + Y
// tile per pixel tile, AT = PT).
template <int AT, int NW>
struct MfmaLds {
  static constexpr int kObufFloats = NW * 16 * AT * 16;  // accumulator tiles
  static constexpr int kBbufWords = kKsBuf * 64 * 8;  // uint4 X + uint4 Y
  // uvw of the fill's timesteps (at most 4 * kKsBuf), float4 each
  static constexpr int kUvwOff =
      kObufFloats > kBbufWords ? kObufFloats : kBbufWords;
  static constexpr int kRedOff = kUvwOff + 4 * 4 * kKsBuf;  // 8 floats
  static constexpr int kSlotOff = kRedOff + 8;   // 2 fill maxima (bits)
  static constexpr int kSinkOff = kSlotOff + 2;  // 64 words: prefetch sink
  static constexpr int kWords = kSinkOff + 64;
  // general path at S = 32 (kGeoLds): the subgrid's pixel geometry, l by
  // column and m by row (32 each), then n and phase_offset per pixel
  static constexpr int kGeoOff = kWords;
  static constexpr int kWordsGeo = kGeoOff + 64 + 2 * 1024;
};
// LDS words of a kernel that runs grid_mfma's general path at S_CT
template <int S_CT, int NW, int AT>
constexpr int general_lds_words() {
  return S_CT == 32 ? MfmaLds<AT, NW>::kWordsGeo : MfmaLds<AT, NW>::kWords;
}

// LDS-DMA of 4 bytes per lane from the lane's global address into
// lds_dst + 4 * lane (lds_dst wave-uniform), as inline asm: the gridder uses
// it only to pull the next fill's rows into L2 (the LDS words are a sink
// nobody reads), and hipcc, which cannot see the asm, inserts no wait for
// it; every __syncthreads() drains it (s_waitcnt vmcnt(0)).  M0 is a
// reserved register the compiler manages itself (a clobber of it is
// ignored), so the asm saves and restores it around its own use; and the
// SALU write of M0 is followed by one wait state before the LDS-DMA reads
// it (the gfx9 "M0 write -> LDS DMA" hazard, which the compiler cannot pad
// inside an asm string; tools/probes/dma_drain_check.py checks the listing).
__device__ __forceinline__ void l2_prefetch_dma(const void *src,
                                                const void *lds_dst) {
  const unsigned m0 = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(
      reinterpret_cast<size_t>((const __attribute__((address_space(3))) void *)
                                   lds_dst)));
  unsigned saved;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(saved)
      : "v"(src), "s"(m0)
      : "memory");
}

// FFT: the subgrid leaves as its 2-D FFT (sign +1, scale 1; S = 32 only),
// what launch_subgrid_fft(+1, 1) would make of the plain output, bit for
// bit: the pixels go to LDS planes instead of HBM and fft.hpp's transform
// (kernel_subgrid_fft_reg's) runs on them (idg_gridder_fft_launch).
// PREC: kPrecTail adds the k * phase_index part of the reduction's tail to
// every phasor's revolutions (device.hpp tail_k_rev: one v_pk_add_f32 per
// two phasors, ~5 % of the MFMA loop); kPrecTailAlt adds 4x that to the
// first channel of every quad only (the default: the same sum over each
// quad for a quarter of the adds); kPrecFlush (S = 32) adds the
// accumulator tiles to an f32 master every kFlushFills fills and restarts
// them from zero (blocked summation, DESIGN.md §3.1: the MFMA rounds its
// f32 sum several times per instruction, so 2,048 K-steps into one tile put
// the C = 256 gridder 8.4e-6 from exact accumulation).  The master lives in
// the subgrid's own output slot (32 KB at S = 32, one pass), which only the
// epilogue writes, after the master is read back.
template <int S_CT, int PT, int CB, int NW, bool MIRROR, bool FFT = false,
          int PREC = kPrecTail, bool PRESCAN = false, bool OPAQUE_TID = !MIRROR>
__device__ __forceinline__ void grid_mfma(
    const SubgridSetup &g, int S, int npix, float image_size, int C,
    int nr_stations, const idg::UVWCoordinate<float> *__restrict__ uvw,
    const float *__restrict__ wavenumbers,
    const float2 *__restrict__ visibilities,
    const float *__restrict__ spheroidal, const float2 *__restrict__ aterms,
    float2 *__restrict__ out, unsigned *lds, float vmax_pre = 0.0f,
    int pass_lo = 0, int pass_hi = 1 << 30) {
  static_assert(CB % 4 == 0, "anchor blocks hold whole channel quads");
  // General path (and the persistent mirror kernel): an opaque copy of the
  // thread index, so values derived from it are formed per call, not hoisted
  // out of the kernel's loop over subgrids and kept live (spilled) across it
  // (scratch 408 -> 160 B/lane gridder, 168 -> 68 degridder at S = 32; the
  // mirror path, one subgrid per workgroup, is better without it).
  int tid = threadIdx.x;
  if constexpr (OPAQUE_TID) asm volatile("" : "+v"(tid));
  const int lane = tid & 63, wave = tid >> 6;
  const int grp = lane >> 4, col = lane & 15;
  // MIRROR: base pixels b < npix/2 (mirror npix-1-b shares the phasor);
  // general: every pixel is a base pixel and Y is added, not mirrored.
  const int half = MIRROR ? npix / 2 : npix;
  // General path: X + Y accumulate into one tile (nothing to mirror), so a
  // wave holds twice the pixel tiles in the same accumulator registers and
  // the S = 32 subgrid is one pass (B built once per subgrid, not twice).
  constexpr bool kFused = !MIRROR && IDG_GRID_FUSED_GENERAL;
  // the reduction tail on every phasor, or 4x on one channel per quad
  constexpr bool kTailAlt = (PREC & kPrecTailAlt) != 0;
  constexpr bool kTailAll = (PREC & kPrecTail) != 0 && !kTailAlt;
  constexpr int AT = kFused ? PT : 2 * PT;  // accumulator tiles per wave
  using Lds = MfmaLds<AT, NW>;
  // General path at S = 32: the pixel geometry lives in LDS, not in 32
  // VGPRs across the whole subgrid (the general path's spills).  A lane's
  // tile pair h covers pixels b0 = (wave PT + 2h) 16 + col and b0 + 16: l
  // by column col and col + 16 for every pair, m wave-uniform per pair
  // (row wave PT / 2 + h), n and phase_offset read per pair and timestep
  // quad.
  constexpr bool kGeoLds = kFused && S_CT == 32;
  float *geo = reinterpret_cast<float *>(lds + Lds::kGeoOff);
  const int nt = g.nr_timesteps;
  const int nchq = (C + 3) / 4;  // channel quads
  const int nquads = (nt + 3) / 4;
  const int quads_per_fill = nchq <= kKsBuf ? kKsBuf / nchq : 1;
  const int cq_per_fill = nchq <= kKsBuf ? nchq : kKsBuf;
  unsigned *slots = lds + Lds::kSlotOff;

  // A power-of-two scale 2^-e keeps the visibilities inside f16 range.  It
  // is set by the maximum over the first fill's timesteps (all channels),
  // and every fill reports its own maximum (an integer LDS max of the
  // non-negative float bits): a fill whose values would leave the range
  // (|V| 2^-e >= 2^15), or the first non-zero fill when the scale is not
  // yet set, is split again with the new scale after the f32 sums so far
  // are rescaled by the exact power of two.  Each input byte is thus read
  // once per fill (the first fill's rows twice, back to back, from L2).
  // PRESCAN: the caller scanned them already (prologue_scan: vmax_pre).
  float vmax = vmax_pre;
  if (tid < 2) slots[tid] = 0u;
  if constexpr (!PRESCAN) {
    vmax = 0.0f;
    const float4 *v4 = reinterpret_cast<const float4 *>(
        visibilities + g.time_offset * C * 4);
    const int n4 = min(4 * quads_per_fill, nt) * C * 2;
    for (int i = tid; i < n4; i += NW * 64) {
      const float4 q = v4[i];
      vmax = fmaxf(vmax, fmaxf(fmaxf(fabsf(q.x), fabsf(q.y)),
                               fmaxf(fabsf(q.z), fabsf(q.w))));
    }
    for (int off = 32; off > 0; off >>= 1)
      vmax = fmaxf(vmax, __shfl_xor(vmax, off));
    float *red = reinterpret_cast<float *>(lds + Lds::kRedOff);
    if (lane == 0) red[wave] = vmax;
    __syncthreads();
#pragma unroll
    for (int w = 0; w < NW; ++w) vmax = fmaxf(vmax, red[w]);
  }
  // the scaled values sit below 2^kBS (IDG_GRID_BSCALE): high in f16 range,
  // so the lo part of the split stays a normal f16 down to 2^(kBS-17) of
  // the maximum instead of 2^-3 (f16 subnormals hold only 2^-24 absolute)
  constexpr int kBS = IDG_GRID_BSCALE;
  static_assert(kBS >= 0 && kBS <= 14, "a fill may reach 2^15 before it re-splits");
  int e = 0;
  bool have_scale = vmax > 0.0f && vmax <= 3.0e38f;
  if (have_scale) frexpf(vmax, &e);
  float scale = ldexpf(1.0f, kBS - e);
  int fidx = 0;  // fills so far (parity selects the fill's max slot)

  const float2 *__restrict__ vsub = visibilities + g.time_offset * C * 4;

  uint4 *bbuf = reinterpret_cast<uint4 *>(lds);  // [ks][64][X, Y]
  float *obuf = reinterpret_cast<float *>(lds);
  float4 *tuvw = reinterpret_cast<float4 *>(lds + Lds::kUvwOff);

  constexpr int kPass = NW * 16 * PT;  // base pixels per pass
  // [pass_lo, pass_hi): the base pixels this workgroup takes (a multiple of
  // kPass; all of them unless the subgrid's passes are split over
  // workgroups, kernel_gridder_mirror_mi355x SPLIT)
  for (int gbase = pass_lo; gbase < min(half, pass_hi); gbase += kPass) {
    // Pixel terms of tile pairs (2h, 2h+1), packed: every phase operation
    // below is one v_pk_* over the pair with the channel's wavenumber
    // broadcast from an SGPR, so no operand has to be duplicated.
    static_assert(PT % 2 == 0, "phases are packed over tile pairs");
    constexpr int PH = PT / 2;
    floatx2 L2[PH], M2[PH], N2[PH], PG2[PH];
    if constexpr (kGeoLds) {
      static_assert(PT == 8 && NW == 8, "one S = 32 pass: 1,024 pixels");
      // (read after the first fill's barrier)
      for (int p = tid; p < 1024; p += NW * 64) {
        float l, m, n, pg;
        pixel_geometry<true>(p, 32, image_size, g, l, m, n, pg);
        geo[64 + p] = n;
        geo[64 + 1024 + p] = pg;
        if (p < 32) geo[p] = l;
        if (p % 32 == 0) geo[32 + p / 32] = m;
      }
    } else {
#pragma unroll
      for (int i = 0; i < PT; ++i) {
        const int b = min(gbase + (wave * PT + i) * 16 + col, half - 1);
        float l, m, n, pg;
        pixel_geometry<!MIRROR>(b, S, image_size, g, l, m, n, pg);
        L2[i / 2][i % 2] = l;
        M2[i / 2][i % 2] = m;
        N2[i / 2][i % 2] = n;
        PG2[i / 2][i % 2] = pg;
      }
    }
    constexpr int PY = kFused ? 1 : PT;  // separate Y tiles (mirror path)
    floatx4 accx[PT], accy[PY];
#pragma unroll
    for (int i = 0; i < PT; ++i) accx[i] = floatx4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int i = 0; i < PY; ++i) accy[i] = floatx4{0.0f, 0.0f, 0.0f, 0.0f};

    // Blocked summation (PREC & kPrecFlush): lane (grp, col < 8) of tile t
    // owns master word block ((wave * AT + t) * 32 + grp * 8 + col) of the
    // subgrid's output slot, 4 floats (its 4 rows); the hi and lo columns
    // of a component (lanes col and col + 8) are summed into it by one DPP
    // row_ror:8 add.  The master is kept unscaled (x 2^e, exact).
    constexpr bool kFlush = (PREC & kPrecFlush) != 0;
    static_assert(!kFlush || S_CT == 32,
                  "the master fills the S = 32 output slot in one pass");
    bool flushed = false;
    auto master = [&](int t) {
      return reinterpret_cast<float4 *>(out) +
             ((wave * AT + t) * 32 + grp * 8 + (col & 7));
    };
    // (the four elements are taken into named scalars before their DPP
    // moves: written as a loop over a[r], this hipcc moved a[0] four times;
    // tools/probes/dpp_vector_probe.hip)
    auto flush_tile = [&](floatx4 &a, int t, float unsc) {
      const float a0 = a[0], a1 = a[1], a2 = a[2], a3 = a[3];
      const float v0 = (a0 + row_ror8(a0)) * unsc;
      const float v1 = (a1 + row_ror8(a1)) * unsc;
      const float v2 = (a2 + row_ror8(a2)) * unsc;
      const float v3 = (a3 + row_ror8(a3)) * unsc;
      if (col < 8) {
        float4 m = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (flushed) m = *master(t);
        *master(t) = make_float4(m.x + v0, m.y + v1, m.z + v2, m.w + v3);
      }
      a = floatx4{0.0f, 0.0f, 0.0f, 0.0f};
    };

    for (int q0 = 0; q0 < nquads; q0 += quads_per_fill) {
      const int nq = min(quads_per_fill, nquads - q0);
      for (int j0 = 0; j0 < nchq; j0 += cq_per_fill, ++fidx) {
        const int nj = min(cq_per_fill, nchq - j0);
        // ---- B fragments for nq timestep quads x nj channel quads -> LDS.
        // One wave fills one K-step (lane = group g, column col): items
        // (t = 4q+g, c0..c0+3), two word loads each, scaled, then split to
        // the column's f16 part.  Redone (rarely) when the fill's maximum
        // leaves the scale's range.
        for (;;) {
        __syncthreads();
        // the other slot was read before this barrier; it is next written
        // by the following fill, after the barrier that ends this one
        if (tid == 0) slots[(fidx + 1) & 1] = 0u;
        {
          // this lane's B column: correlation bpol, re (even col) or im
          // (odd col) part, and which f16 part (hi: 0, lo: -1) it holds.
          // Column re: bc = re, bs = -im;  column im: bc = im, bs = re --
          // so the lane loads exactly the two words it needs and only
          // scales them (the sign of bs folded into its scale).
          const int bpol = (col & 7) >> 1;
          const int w_c = 2 * bpol + (col & 1);        // word of bc
          const int w_s = 2 * bpol + 1 - (col & 1);    // word of bs
          const float sc_s = (col & 1) ? scale : -scale;
          const float bpart = (col & 8) ? -1.0f : 0.0f;
          const float *vsubf = reinterpret_cast<const float *>(vsub);
          const int nks = nq * nj;
          const bool full = (q0 + nq) * 4 <= nt && 4 * (j0 + nj) <= C;
          // K-steps are wave-uniform (scalar loop, qq/jj on the SALU), the
          // block base pointer too; the lane adds a 32-bit byte offset that
          // is fixed for the kernel (timestep group grp, column words), so
          // the loads take the SGPR-base + VGPR-offset form with no 64-bit
          // address arithmetic per K-step.
          const int wv = __builtin_amdgcn_readfirstlane(wave);
          const unsigned off_c = (grp * C * 8 + w_c) * 4u;
          const unsigned off_s = (grp * C * 8 + w_s) * 4u;
          int qq = wv / nj, jj = wv - (wv / nj) * nj;
          float lmax = 0.0f;  // max |raw value| this lane loads
#ifdef IDG_DEBUG_SKIPFILL
          // timing experiment only (wrong output): every fill after the
          // first reuses its B fragments
          for (int ks = fidx > 0 ? nks : wv; ks < nks; ks += NW) {
#else
          for (int ks = wv; ks < nks; ks += NW) {
#endif
            const int t = (q0 + qq) * 4 + grp;
            const int c0 = 4 * (j0 + jj);
            float bc[4], bs[4];
            if (full) {
              const char *blk = reinterpret_cast<const char *>(
                  vsubf + ((q0 + qq) * 4 * C + c0) * 8);
#pragma unroll
              for (int u = 0; u < 4; ++u) {
#if IDG_GRID_NT_FILL
                // the fill is the rows' last use: non-temporal (a raw buffer
                // load keeps the SGPR-base + VGPR-offset form), so L2 keeps
                // the blocked-summation masters rather than spent rows
                const __amdgpu_buffer_rsrc_t rsrc =
                    __builtin_amdgcn_make_buffer_rsrc(
                        const_cast<char *>(blk), static_cast<short>(0),
                        0x7ffffff0, 0x00020000);
                const float rc = __builtin_bit_cast(
                    float, __builtin_amdgcn_raw_buffer_load_b32(
                               rsrc, static_cast<int>(off_c), 32 * u, 2));
                const float rs = __builtin_bit_cast(
                    float, __builtin_amdgcn_raw_buffer_load_b32(
                               rsrc, static_cast<int>(off_s), 32 * u, 2));
#else
                const float rc =
                    *reinterpret_cast<const float *>(blk + off_c + 32 * u);
                const float rs =
                    *reinterpret_cast<const float *>(blk + off_s + 32 * u);
#endif
                lmax = fmaxf(lmax, fmaxf(fabsf(rc), fabsf(rs)));
                bc[u] = rc * scale;
                bs[u] = rs * sc_s;
              }
            } else {
#pragma unroll
              for (int u = 0; u < 4; ++u) {
                const bool ok = t < nt && c0 + u < C;
                const int it = ok ? t * C + c0 + u : 0;
                const float rc = ok ? vsubf[it * 8 + w_c] : 0.0f;
                const float rs = ok ? vsubf[it * 8 + w_s] : 0.0f;
                lmax = fmaxf(lmax, fmaxf(fabsf(rc), fabsf(rs)));
                bc[u] = rc * scale;
                bs[u] = rs * sc_s;
              }
            }
            jj += NW;
            while (jj >= nj) {
              jj -= nj;
              ++qq;
            }
            const unsigned xc = split_part(bc[0], bc[1], bpart);
            const unsigned yc = split_part(bc[2], bc[3], bpart);
            const unsigned xs = split_part(bs[0], bs[1], bpart);
            const unsigned ys = split_part(bs[2], bs[3], bpart);
            bbuf[(ks * 64 + lane) * 2] = make_uint4(xc, xc, yc, yc);
            bbuf[(ks * 64 + lane) * 2 + 1] = make_uint4(xs, xs, ys, ys);
          }
          // wave max (rows of 16 by DPP, then the four row maxima), one LDS
          // atomic per wave (an atomicMax from every lane would be expanded
          // into a 64-step scalar loop by the atomic optimizer)
          {
            unsigned v = __float_as_uint(lmax);
            v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false));
            v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false));
            v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xF, 0xF, false));
            v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xF, 0xF, false));
            const unsigned wmax =
                max(max(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16)),
                    max(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48)));
            if (lane == 0) atomicMax(&slots[fidx & 1], wmax);
          }
          // the fill's timesteps' uvw, so the MFMA loop reads LDS, not HBM
          for (int i = tid; i < nq * 4; i += NW * 64) {
            const idg::UVWCoordinate<float> c =
                uvw[g.time_offset + min(q0 * 4 + i, nt - 1)];
            tuvw[i] = make_float4(c.u, c.v, c.w, 0.0f);
          }
        }
        __syncthreads();
        // The fill's maximum against the scale (wave-uniform branch).
        const float fm = __uint_as_float(
            __builtin_amdgcn_readfirstlane(slots[fidx & 1]));
        if (!(fm > 0.0f && fm <= 3.0e38f)) break;  // all zero (or non-finite)
        int em;
        frexpf(fm, &em);
        if (have_scale ? em <= e + 15 - kBS : em == e) {
          have_scale = true;
          break;
        }
        // Out of range: rescale the sums so far (zero while the scale was
        // unset) and split this fill again; the slot keeps the fill's max.
        if (have_scale) {
          const float r = ldexpf(1.0f, e - em);
#pragma unroll
          for (int i = 0; i < PT; ++i) accx[i] *= r;
#pragma unroll
          for (int i = 0; i < PY; ++i) accy[i] *= r;
        }
        e = em;
        scale = ldexpf(1.0f, kBS - e);
        have_scale = true;
        }
        // Pull the next fill's rows into L2 while this fill's MFMA loop
        // runs (one 4-byte LDS-DMA per 128-byte line, into a sink).
        {
          int q0n = q0, j0n = j0 + cq_per_fill;
          if (j0n >= nchq) {
            j0n = 0;
            q0n = q0 + quads_per_fill;
          }
          if (q0n < nquads) {
            const int rows = min(4 * (q0n + quads_per_fill), nt) - 4 * q0n;
            const int lpr = (min(cq_per_fill, nchq - j0n) * 128 + 127) / 128;
            const char *vb = reinterpret_cast<const char *>(vsub);
            for (int ln = tid; ln < rows * lpr; ln += NW * 64) {
              const int row = ln / lpr, cl = ln - (ln / lpr) * lpr;
              l2_prefetch_dma(
                  vb + (static_cast<size_t>(4 * q0n + row) * C + 4 * j0n) * 32 +
                      cl * 128,
                  lds + Lds::kSinkOff);
            }
          }
        }
        // ---- MFMA over the buffered K-steps ----
        // Channel blocks outermost: the block's CB wavenumbers are loaded
        // into SGPRs once per fill, not once per timestep quad.
        for (int jb = 0; jb < nj; jb += CB / 4) {
          const int je = min(jb + CB / 4, nj);
          const float ka = wavenumbers[4 * (j0 + jb)];
          float kb[CB];
#pragma unroll
          for (int v = 0; v < CB; ++v)
            kb[v] = wavenumbers[min(4 * (j0 + jb) + v, C - 1)];
          for (int qq = 0; qq < nq; ++qq) {
            const float4 c4 = tuvw[qq * 4 + grp];
            const idg::UVWCoordinate<float> c = {c4.x, c4.y, c4.z};
            const floatx2 cu = {c.u, c.u}, cv = {c.v, c.v};
            const floatx2 ih = {kInv2PiHi, kInv2PiHi};
            if constexpr (kFused) {
              // Tile pairs outermost: only one pair's phase terms are live,
              // and each K-step's B fragments are re-read from LDS per pair.
#pragma unroll
              for (int h = 0; h < PH; ++h) {
                if constexpr (kGeoLds) {
                  const int b0 = (wave * PT + 2 * h) * 16 + col;
                  L2[h] = floatx2{geo[col], geo[col + 16]};
                  const float mh = geo[32 + wave * (PT / 2) + h];
                  M2[h] = floatx2{mh, mh};
                  N2[h] = floatx2{geo[64 + b0], geo[64 + b0 + 16]};
                  PG2[h] = floatx2{geo[64 + 1024 + b0], geo[64 + 1024 + b0 + 16]};
                }
                floatx2 pidx = __builtin_elementwise_fma(cu, L2[h], cv * M2[h]);
                pidx = __builtin_elementwise_fma(floatx2{c.w, c.w}, N2[h], pidx);
                const floatx2 np = -pidx;
                const floatx2 a =
                    __builtin_elementwise_fma(np, floatx2{ka, ka}, PG2[h]);
                const floatx2 t = a * ih;
                const floatx2 nm = {-__builtin_rintf(t.x), -__builtin_rintf(t.y)};
                // the k * phase_index part of the reduction's tail, at the
                // block's first channel (device.hpp: kPhaseTail)
                floatx2 cr = {0.0f, 0.0f};
                if constexpr (kTailAll) cr = tail_k_rev(np, ka);
                if constexpr (kTailAlt)
                  cr = tail_k_rev(np, 4.0f * ka);
#pragma unroll
                for (int u = 0; u < CB / 4; ++u) {
                  const int jj = jb + u;
                  if (jj >= je) break;
                  const int ks = qq * nj + jj;
                  const uint4 bx = bbuf[(ks * 64 + lane) * 2];
                  const uint4 by = bbuf[(ks * 64 + lane) * 2 + 1];
                  const half8 bfx = pack4(bx.x, bx.y, bx.z, bx.w);
                  const half8 bfy = pack4(by.x, by.y, by.z, by.w);
                  float snx[4], csx[4], sny[4], csy[4];
#pragma unroll
                  for (int j = 0; j < 4; ++j) {
                    const float kj = kb[4 * u + j];
                    const floatx2 ph =
                        __builtin_elementwise_fma(np, floatx2{kj, kj}, PG2[h]);
                    floatx2 r = __builtin_elementwise_fma(ph, ih, nm);
                    if constexpr (kTailAll) r = r + cr;
                    if constexpr (kTailAlt)
                      if (j == 0) r = r + cr;
                    sincos_rev(r.x, &snx[j], &csx[j]);
                    sincos_rev(r.y, &sny[j], &csy[j]);
                  }
                  half8 ac, as, ac1, as1;
                  split_oct(csx[0], csx[1], csx[2], csx[3], snx[0], snx[1],
                            snx[2], snx[3], &ac, &as);
                  split_oct(csy[0], csy[1], csy[2], csy[3], sny[0], sny[1],
                            sny[2], sny[3], &ac1, &as1);
                  accx[2 * h] = mfma16(ac, bfx, accx[2 * h]);
                  accx[2 * h + 1] = mfma16(ac1, bfx, accx[2 * h + 1]);
                  accx[2 * h] = mfma16(as, bfy, accx[2 * h]);
                  accx[2 * h + 1] = mfma16(as1, bfy, accx[2 * h + 1]);
                  IDG_KSTEP_FENCE();
                }
              }
              continue;
            }
            floatx2 NP[PH], NM[PH], CR[PH];
#pragma unroll
            for (int h = 0; h < PH; ++h) {
              // phase_index = fma(w, n, fma(u, l, v*m)); w = 0 on mirror
              // subgrids, where fma(0, n, x) == x
              floatx2 pidx = __builtin_elementwise_fma(cu, L2[h], cv * M2[h]);
              if constexpr (!MIRROR)
                pidx = __builtin_elementwise_fma(floatx2{c.w, c.w}, N2[h],
                                                 pidx);
              NP[h] = -pidx;
              // -m: the whole revolutions of the block's first-channel
              // phase, so every r below stays within ~0.7 revolutions
              const floatx2 a =
                  __builtin_elementwise_fma(NP[h], floatx2{ka, ka}, PG2[h]);
              const floatx2 t = a * ih;
              NM[h] = floatx2{-__builtin_rintf(t.x), -__builtin_rintf(t.y)};
              // the k * phase_index part of the reduction's tail at the
              // block's first channel (device.hpp: kPhaseTail)
              if constexpr (kTailAll)
                CR[h] = tail_k_rev(NP[h], ka);
              if constexpr (kTailAlt)
                CR[h] = tail_k_rev(NP[h], 4.0f * ka);
            }
#pragma unroll
            for (int u = 0; u < CB / 4; ++u) {
              const int jj = jb + u;
              if (jj >= je) break;
              const int ks = qq * nj + jj;
              const uint4 bx = bbuf[(ks * 64 + lane) * 2];
              const uint4 by = bbuf[(ks * 64 + lane) * 2 + 1];
              const half8 bfx = pack4(bx.x, bx.y, bx.z, bx.w);
              const half8 bfy = pack4(by.x, by.y, by.z, by.w);
#pragma unroll
              for (int h = 0; h < PH; ++h) {
                // r[j] = (revolutions of channel 4u+j) for tiles (2h, 2h+1):
                // the reference's phase, then phase * 1/2pi_hi - m exactly
                // rounded once (the product is exact inside the FMA)
                float snx[4], csx[4], sny[4], csy[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                  const float kj = kb[4 * u + j];
                  const floatx2 ph =
                      __builtin_elementwise_fma(NP[h], floatx2{kj, kj}, PG2[h]);
                  floatx2 r = __builtin_elementwise_fma(ph, ih, NM[h]);
                  if constexpr (kTailAll) r = r + CR[h];
                  if constexpr (kTailAlt)
                    if (j == 0) r = r + CR[h];
                  sincos_rev(r.x, &snx[j], &csx[j]);
                  sincos_rev(r.y, &sny[j], &csy[j]);
                }
                // one asm block splits a tile's cos and sin quads (one pair of
                // wait-state pads for both MFMA operands)
                half8 ac, as;
                split_oct(csx[0], csx[1], csx[2], csx[3], snx[0], snx[1],
                          snx[2], snx[3], &ac, &as);
                accx[2 * h] = mfma16(ac, bfx, accx[2 * h]);
                accy[2 * h] = mfma16(as, bfy, accy[2 * h]);
                split_oct(csy[0], csy[1], csy[2], csy[3], sny[0], sny[1],
                          sny[2], sny[3], &ac, &as);
                accx[2 * h + 1] = mfma16(ac, bfx, accx[2 * h + 1]);
                accy[2 * h + 1] = mfma16(as, bfy, accy[2 * h + 1]);
              }
              // Keep each K-step's MFMAs inside its own iteration.  When the
              // scheduler sank all of an iteration's MFMAs to the end of the
              // loop body, the last tile's accumulators came out corrupted
              // (a few % of subgrids, run-to-run different, only with >1
              // wave per SIMD; DESIGN.md §4.4, tools/debug/diff_detail.py).
              IDG_KSTEP_FENCE();
            }
          }
        }
        if constexpr (kFlush) {
          // every kFlushFills fills except the last (wave-uniform)
          const bool last =
              j0 + cq_per_fill >= nchq && q0 + quads_per_fill >= nquads;
          if (!last && (fidx + 1) % kFlushFills == 0) {
            const float unsc = ldexpf(1.0f, e - kBS);
#pragma unroll
            for (int i = 0; i < PT; ++i) flush_tile(accx[i], i, unsc);
            if constexpr (!kFused) {
#pragma unroll
              for (int i = 0; i < PY; ++i) flush_tile(accy[i], PT + i, unsc);
            }
            flushed = true;
          }
        }
      }
    }
    if constexpr (kFlush) {
      // the master back into the hi columns (lanes col < 8), rescaled to
      // the current 2^-e (exact); the epilogue sums hi + lo as before
      if (flushed && col < 8) {
        const float sc = ldexpf(1.0f, kBS - e);
#pragma unroll
        for (int i = 0; i < PT; ++i) {
          const float4 m = *master(i);
          accx[i] += floatx4{m.x, m.y, m.z, m.w} * sc;
        }
        if constexpr (!kFused) {
#pragma unroll
          for (int i = 0; i < PY; ++i) {
            const float4 m = *master(PT + i);
            accy[i] += floatx4{m.x, m.y, m.z, m.w} * sc;
          }
        }
      }
    }

    const float unscale = ldexpf(1.0f, e - kBS);
    // ---- epilogue: X, Y tiles -> LDS [pixel][16]; base = X + Y, mirror =
    // X - Y; hi + lo; A-term; store ----
    __syncthreads();
#pragma unroll
    for (int i = 0; i < PT; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int lp = (wave * PT + i) * 16 + grp * 4 + r;
        obuf[lp * 16 + col] = accx[i][r];
        if constexpr (!kFused) obuf[(kPass + lp) * 16 + col] = accy[i][r];
      }
    __syncthreads();
    // FFT: each thread's pixels stay in registers until every obuf row is
    // read (the planes reuse that LDS)
    static_assert(!FFT || (S_CT == 32 && kPass >= (MIRROR ? 512 : 1024)),
                  "the FFT epilogue takes a whole S = 32 subgrid in one pass");
    constexpr int kIt = FFT ? kPass / (NW * 64) : 1;
    float2 keep[kIt][MIRROR ? 2 : 1][4];
    auto emit = [&](const float (&a)[8], int p, int it, int slot) {
      if constexpr (FFT)
        pixel_out(a, p, S, g, nr_stations, spheroidal, aterms, keep[it][slot]);
      else
        store_pixel(a, p, S, npix, g, nr_stations, spheroidal, aterms, out);
    };
    auto body = [&](int q, int it) {
      const int b = gbase + q;
      if (b >= half) return;
      const float4 *xr = reinterpret_cast<const float4 *>(obuf + q * 16);
      const float4 xh0 = xr[0], xh1 = xr[1], xl0 = xr[2], xl1 = xr[3];
      const float x[8] = {xh0.x + xl0.x, xh0.y + xl0.y, xh0.z + xl0.z,
                          xh0.w + xl0.w, xh1.x + xl1.x, xh1.y + xl1.y,
                          xh1.z + xl1.z, xh1.w + xl1.w};
      float y[8] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
      if constexpr (!kFused) {  // the Y tiles (fused: already in x)
        const float4 *yr =
            reinterpret_cast<const float4 *>(obuf + (kPass + q) * 16);
        const float4 yh0 = yr[0], yh1 = yr[1], yl0 = yr[2], yl1 = yr[3];
        const float yv[8] = {yh0.x + yl0.x, yh0.y + yl0.y, yh0.z + yl0.z,
                             yh0.w + yl0.w, yh1.x + yl1.x, yh1.y + yl1.y,
                             yh1.z + yl1.z, yh1.w + yl1.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) y[j] = yv[j];
      }
      // the phase tail of the reduction: base pixel * exp(i poff eps),
      // mirror pixel (phase_offset -poff) * exp(-i poff eps)
      float l, m, n, poff;
      pixel_geometry<!MIRROR>(b, S, image_size, g, l, m, n, poff);
      float tc, ts;
      phase_tail(poff, &tc, &ts);
      float ab[8];
#pragma unroll
      for (int j = 0; j < 8; ++j)
        ab[j] = (kFused ? x[j] : x[j] + y[j]) * unscale;
      rotate4(ab, tc, ts);
      emit(ab, b, it, 0);
      if constexpr (MIRROR) {
        float am[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) am[j] = (x[j] - y[j]) * unscale;
        rotate4(am, tc, -ts);
        emit(am, npix - 1 - b, it, 1);
      }
    };
    if constexpr (FFT) {
#pragma unroll
      for (int it = 0; it < kIt; ++it) body(tid + it * NW * 64, it);
      constexpr int N = 32, RS = N + 1;
      float2 *planes = reinterpret_cast<float2 *>(lds);  // [4][N][N + 1]
      __syncthreads();  // every obuf row is read
#pragma unroll
      for (int it = 0; it < kIt; ++it) {
        const int b = tid + it * NW * 64;
        if (b >= half) continue;
#pragma unroll
        for (int slot = 0; slot < (MIRROR ? 2 : 1); ++slot) {
          const int p = slot ? npix - 1 - b : b;
          const int row = p / N, col = p % N;
#pragma unroll
          for (int pol = 0; pol < 4; ++pol)
            planes[pol * N * RS + row * RS + col] = keep[it][slot][pol];
        }
      }
      __syncthreads();
      float2 tw[N / 2];
#pragma unroll
      for (int k = 0; k < N / 2; ++k) tw[k] = unit_phasor(k, N, 1.0f);
      float2 f[N];
      fft2_planes_lds<N>(planes, tid, 4 * N, tw, f);
      if (tid < 4 * N) {
        const int pp = tid / N, qq = tid % N;
#pragma unroll
        for (int i = 0; i < N; ++i)
          out[static_cast<size_t>(pp) * npix + bit_reverse<N>(i) * N + qq] =
              f[i];
      }
    } else {
      for (int q = tid; q < kPass; q += NW * 64) body(q, 0);
    }
    __syncthreads();
  }
}

// The mirror check's uvw loads and grid_mfma's max-|V| scan of the first
// fill's rows in one pass: both depend only on the subgrid's metadata, so
// the prologue waits for one memory round trip and one barrier instead of
// two of each (the first round of workgroups, all in their prologue at
// once, has no other workgroup computing beside it).  Returns this thread's
// w != 0 flag and leaves each wave's maximum in red[wave]; the caller's
// __syncthreads_or is the barrier before prologue_max reads them.
template <int NW>
__device__ __forceinline__ bool prologue_scan(
    const SubgridSetup &g, int C,
    const idg::UVWCoordinate<float> *__restrict__ uvw,
    const float2 *__restrict__ visibilities, float *red) {
  const int tid = threadIdx.x;
  bool w_nonzero = false;
  for (int t = tid; t < g.nr_timesteps; t += NW * 64)
    w_nonzero |= uvw[g.time_offset + t].w != 0.0f;
  // grid_mfma's first fill: quads_per_fill timestep quads, all channels
  const int nchq = (C + 3) / 4;
  const int quads_per_fill = nchq <= kKsBuf ? kKsBuf / nchq : 1;
  const float4 *v4 = reinterpret_cast<const float4 *>(
      visibilities + g.time_offset * C * 4);
  const int n4 = min(4 * quads_per_fill, g.nr_timesteps) * C * 2;
  float vmax = 0.0f;
  for (int i = tid; i < n4; i += NW * 64) {
    const float4 q = v4[i];
    vmax = fmaxf(vmax, fmaxf(fmaxf(fabsf(q.x), fabsf(q.y)),
                             fmaxf(fabsf(q.z), fabsf(q.w))));
  }
  for (int off = 32; off > 0; off >>= 1)
    vmax = fmaxf(vmax, __shfl_xor(vmax, off));
  if ((tid & 63) == 0) red[tid >> 6] = vmax;
  return w_nonzero;
}

template <int NW>
__device__ __forceinline__ float prologue_max(const float *red) {
  float vmax = red[0];
#pragma unroll
  for (int w = 1; w < NW; ++w) vmax = fmaxf(vmax, red[w]);
  return vmax;
}

}  // namespace

#if defined(IDG_WG_TIMELINE) && IDG_WG_TIMELINE
__device__ WgStamp idg_debug_timeline_gridder[kTimelineMax];
#endif

// S_CT: subgrid size known at compile time (0 = runtime).
// PPT : pixels per lane (VALU paths).   CB: channels per phase anchor.
// MODE: 0 = VALU kernel (VALU mirror path + general path, every subgrid),
//       1 = MFMA kernel (mirror path on eligible subgrids, the same GEMMs
//           over every pixel with the w-term on the others).
// PT  : 16-pixel base tiles per wave in the MFMA path.
// (One launch over every subgrid, each on its path: the reference's launch
// shape.  The device entries launch the two-kernel form instead:
// kernel_gridder_mirror_mi355x + kernel_gridder_general_mi355x.)
template <int S_CT, int PPT, int CB, int MODE, int PT, bool FFT = false,
          int PREC = kPrecTail>
__global__ void __launch_bounds__(MODE == 1 ? 64 * IDG_GRID_NW : kBlock,
                                  IDG_GRID_WAVES)
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
  static_assert(PPT % 2 == 0, "PPT must be even (pixel pairs)");
  constexpr int NB = PPT / 2;
  const int S = S_CT > 0 ? S_CT : subgrid_size;
  const int npix = S * S;
  const int s = xcd_subgrid(blockIdx.x, gridDim.x);
  const int tid = threadIdx.x;
  const SubgridSetup g = setup_subgrid(metadata, s, grid_size, S, image_size,
                                       w_step_in_lambda);
  const int C = nr_channels;
  float2 *out = subgrids + static_cast<size_t>(s) * 4 * npix;

  // Mirror pairs need w = 0 on every timestep of the subgrid (checked once,
  // so the two paths below stay separate loops with separate registers).
  if constexpr (MODE == 1) {
    constexpr int NW = IDG_GRID_NW;
    // both paths hold 2 PT accumulator tiles per wave
    __shared__ unsigned lds[general_lds_words<S_CT, NW, 2 * PT>()];
#if defined(IDG_WG_TIMELINE) && IDG_WG_TIMELINE
    timeline_start(idg_debug_timeline_gridder);
#endif
    float *red = reinterpret_cast<float *>(lds + MfmaLds<2 * PT, NW>::kRedOff);
    const bool mirror =
        __syncthreads_or(prologue_scan<NW>(g, C, uvw, visibilities, red)) ==
            0 &&
        S % 2 == 0 && g.w_offset == 0.0f;
    const float vmax = prologue_max<NW>(red);
    if (mirror)
      grid_mfma<S_CT, PT, CB, NW, true, FFT, PREC, true>(
          g, S, npix, image_size, C, nr_stations, uvw, wavenumbers,
          visibilities, spheroidal, aterms, out, lds, vmax);
    else
      grid_mfma<S_CT, IDG_GRID_FUSED_GENERAL ? 2 * PT : PT, CB, NW, false,
                FFT, PREC, true>(g, S, npix, image_size, C, nr_stations, uvw,
                                 wavenumbers, visibilities, spheroidal, aterms,
                                 out, lds, vmax);
#if defined(IDG_WG_TIMELINE) && IDG_WG_TIMELINE
    timeline_end(idg_debug_timeline_gridder);
#endif
    return;
  }

  bool w_nonzero = false;
  for (int t = tid; t < g.nr_timesteps; t += blockDim.x)
    w_nonzero |= uvw[g.time_offset + t].w != 0.0f;
  const bool mirror = __syncthreads_or(w_nonzero) == 0 && S % 2 == 0 &&
                      g.w_offset == 0.0f;

  if (mirror) {
    // Mirror-pair path: lane owns base pixels b (< npix/2) and npix-1-b.
    const int half = npix / 2;
    for (int tile = 0; tile < half; tile += kBlock * NB) {
      float l[PPT], m[PPT], n[PPT], poff[PPT], acc[PPT][8];
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int b = min(tile + i * kBlock + tid, half - 1);
        pixel_geometry(b, S, image_size, g, l[i], m[i], n[i], poff[i]);
        pixel_geometry(npix - 1 - b, S, image_size, g, l[NB + i], m[NB + i],
                       n[NB + i], poff[NB + i]);
      }
#pragma unroll
      for (int i = 0; i < PPT; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = 0.0f;

      for (int t = 0; t < g.nr_timesteps; ++t) {
        const long long row = g.time_offset + t;
        const idg::UVWCoordinate<float> c = uvw[row];
        const float4 *vrow =
            reinterpret_cast<const float4 *>(visibilities + row * C * 4);
        timestep_mirror<NB, CB>(l, m, poff, acc, c, vrow, wavenumbers, C);
      }
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int b = tile + i * kBlock + tid;
        if (b < half) {
          store_pixel(acc[i], b, S, npix, g, nr_stations, spheroidal, aterms,
                      out);
          store_pixel(acc[NB + i], npix - 1 - b, S, npix, g, nr_stations,
                      spheroidal, aterms, out);
        }
      }
    }
    return;
  }

  // General path (odd S or w_offset != 0): every pixel its own phase.
  for (int tile = 0; tile < npix; tile += kBlock * PPT) {
    float l[PPT], m[PPT], n[PPT], poff[PPT], acc[PPT][8];
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const int p = min(tile + i * kBlock + tid, npix - 1);
      pixel_geometry(p, S, image_size, g, l[i], m[i], n[i], poff[i]);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = 0.0f;
    }
    for (int t = 0; t < g.nr_timesteps; ++t) {
      const long long row = g.time_offset + t;
      const idg::UVWCoordinate<float> c = uvw[row];
      const float4 *vrow =
          reinterpret_cast<const float4 *>(visibilities + row * C * 4);
      timestep_general<PPT, CB>(l, m, n, poff, acc, c, vrow, wavenumbers, C);
    }
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const int p = tile + i * kBlock + tid;
      if (p < npix)
        store_pixel(acc[i], p, S, npix, g, nr_stations, spheroidal, aterms,
                    out);
    }
  }
}

// The two-kernel form of the device entries (select_gridder; DESIGN.md
// §4.1).  Each path gets the register allocation of its own code alone:
//
// kernel_gridder_mirror_mi355x: grid = nr_subgrids, one workgroup per
//   subgrid as kernel_gridder_mi355x; a mirror-eligible subgrid (even S,
//   w_offset = 0, w = 0 on every timestep) is gridded on the mirror GEMMs,
//   any other is pushed onto the general queue (device.hpp: queue_push) and
//   left.
// kernel_gridder_general_mi355x: a resident grid (occupancy x CUs) that
//   takes the queued subgrids one at a time from the queue's take counter,
//   the next index requested while the current subgrid runs, and grids each
//   on the fused single-pixel GEMMs.  With `all` set it takes subgrids
//   0 .. nr_subgrids-1 and there is no mirror launch: the launch layer sets
//   it when no subgrid can be mirror-eligible (odd S, or w_step_in_lambda
//   != 0, which makes every w_offset non-zero).  Dynamic, not a fixed range
//   per workgroup: with fixed ranges the slowest CU set the time (w-term
//   batch +7-9 %).  On a batch without w-terms the queue is empty and every
//   workgroup returns at once.
// queue: device.hpp queue_ints(nr_subgrids) ints of stream-ordered
// workspace, its counters zeroed before the launches.
// SPLIT > 1 (S = 64: four passes of 512 base pixels): grid = SPLIT x
// nr_subgrids, workgroup (s, q) takes pass q of subgrid s.  The SPLIT
// workgroups of a subgrid are consecutive in the XCD-contiguous order, so
// they run side by side on one XCD and all but the first read the subgrid's
// visibilities from its L2 -- one pass after another in one workgroup
// re-streamed them from memory each pass (2.0x the algorithmic bytes,
// profiles/r04/kernels_s64).  Each workgroup forms the same scale from the
// same first fill, so the output is the one-workgroup kernel's as long as no
// later fill rescales: in the one-workgroup kernel a rescale in pass q
// carries into passes q+1.. (the scale e lives across the pass loop), while
// each split workgroup restarts from the prologue's e.  On data where a late
// fill grows more than 8x past the first the two forms then differ in their
// f16 splits, both within the parity bar
// (tests/test_gpu.py::test_s64_split_forms_with_a_late_loud_timestep).
template <int S_CT, int CB, int PT, bool FFT = false, int PREC = kPrecTail,
          int SPLIT = 1>
__global__ void __launch_bounds__(64 * IDG_GRID_NW, IDG_GRID_WAVES)
    kernel_gridder_mirror_mi355x(
        const int grid_size, int subgrid_size, float image_size,
        float w_step_in_lambda, int nr_channels, int nr_stations,
        const idg::UVWCoordinate<float> *__restrict__ uvw,
        const float *__restrict__ wavenumbers,
        const float2 *__restrict__ visibilities,
        const float *__restrict__ spheroidal,
        const float2 *__restrict__ aterms,
        const idg::Metadata *__restrict__ metadata,
        float2 *__restrict__ subgrids, int *__restrict__ queue) {
  constexpr int NW = IDG_GRID_NW;
  __shared__ unsigned lds[MfmaLds<2 * PT, NW>::kWords];
  const int S = S_CT > 0 ? S_CT : subgrid_size;
  const int npix = S * S;
  const int wg = xcd_subgrid(blockIdx.x, gridDim.x);
  const int s = SPLIT > 1 ? wg / SPLIT : wg;
  const int q = SPLIT > 1 ? wg % SPLIT : 0;
  const int tid = threadIdx.x;
  const SubgridSetup g = setup_subgrid(metadata, s, grid_size, S, image_size,
                                       w_step_in_lambda);
  float *red = reinterpret_cast<float *>(lds + MfmaLds<2 * PT, NW>::kRedOff);
  const bool mirror =
      __syncthreads_or(prologue_scan<NW>(g, nr_channels, uvw, visibilities,
                                         red)) == 0 &&
      S % 2 == 0 && g.w_offset == 0.0f;
  if (!mirror) {
    if constexpr (SPLIT > 1) {
      if (tid == 0 && q == 0)
        queue_push(queue, gridDim.x / SPLIT, s, s % kQueueShards);
    } else {
      if (tid == 0) queue_push(queue, gridDim.x, s);
    }
    return;
  }
  constexpr int kPass = NW * 16 * PT;
  // SPLIT workgroups of kPass base pixels each cover the S_CT subgrid's
  // S^2/2 base pixels exactly once, none of them idle
  static_assert(SPLIT == 1 || (S_CT > 0 && SPLIT * kPass >= S_CT * S_CT / 2 &&
                               (SPLIT - 1) * kPass < S_CT * S_CT / 2),
                "mirror_split(S) does not match the pass size");
  grid_mfma<S_CT, PT, CB, NW, true, FFT, PREC, true>(
      g, S, npix, image_size, nr_channels, nr_stations, uvw, wavenumbers,
      visibilities, spheroidal, aterms,
      subgrids + static_cast<size_t>(s) * 4 * npix, lds,
      prologue_max<NW>(red), SPLIT > 1 ? q * kPass : 0,
      SPLIT > 1 ? (q + 1) * kPass : 1 << 30);
}

// The persistent form of the mirror kernel (A/B builds, -DIDG_GRID_PERSIST=1;
// round 6, the review's N = 8 item): a resident grid (occupancy x CUs, at
// most nr_subgrids) whose workgroups take subgrids 0 .. nr_subgrids-1 from a
// take counter in the queue workspace (kQueueMirror), the next index
// requested while the current subgrid runs, and grid each exactly as
// kernel_gridder_mirror_mi355x does (bit for bit: the same grid_mfma on the
// same subgrid).  The last workgroup to leave zeroes the counter and its
// exit count (kQueueMirrorExit) for the next launch.
template <int S_CT, int CB, int PT, bool FFT = false, int PREC = kPrecTail>
__global__ void __launch_bounds__(64 * IDG_GRID_NW, IDG_GRID_WAVES)
    kernel_gridder_mirror_persist_mi355x(
        const int grid_size, int subgrid_size, float image_size,
        float w_step_in_lambda, int nr_channels, int nr_stations,
        const idg::UVWCoordinate<float> *__restrict__ uvw,
        const float *__restrict__ wavenumbers,
        const float2 *__restrict__ visibilities,
        const float *__restrict__ spheroidal,
        const float2 *__restrict__ aterms,
        const idg::Metadata *__restrict__ metadata,
        float2 *__restrict__ subgrids, int *__restrict__ queue,
        int nr_subgrids) {
  constexpr int NW = IDG_GRID_NW;
  __shared__ unsigned lds[MfmaLds<2 * PT, NW>::kWords];
  __shared__ int take;
  const int S = S_CT > 0 ? S_CT : subgrid_size;
  const int npix = S * S;
  const int tid = threadIdx.x;
  if (tid == 0) take = atomicAdd(queue + kQueueMirror, 1);
  __syncthreads();
  int i = __builtin_amdgcn_readfirstlane(take);
  while (i < nr_subgrids) {
    __syncthreads();  // every thread has read `take`
    if (tid == 0) take = atomicAdd(queue + kQueueMirror, 1);  // lands later
    const int s = i;
    const SubgridSetup g = setup_subgrid(metadata, s, grid_size, S,
                                         image_size, w_step_in_lambda);
    float *red = reinterpret_cast<float *>(lds + MfmaLds<2 * PT, NW>::kRedOff);
    const bool mirror =
        __syncthreads_or(prologue_scan<NW>(g, nr_channels, uvw, visibilities,
                                           red)) == 0 &&
        S % 2 == 0 && g.w_offset == 0.0f;
    if (!mirror) {
      if (tid == 0) queue_push(queue, nr_subgrids, s, s % kQueueShards);
    } else {
      grid_mfma<S_CT, PT, CB, NW, true, FFT, PREC, true, true>(
          g, S, npix, image_size, nr_channels, nr_stations, uvw, wavenumbers,
          visibilities, spheroidal, aterms,
          subgrids + static_cast<size_t>(s) * 4 * npix, lds,
          prologue_max<NW>(red), 0, 1 << 30);
    }
    __syncthreads();  // `take` has landed; the subgrid's LDS is consumed
    i = __builtin_amdgcn_readfirstlane(take);
  }
  if (tid == 0 && atomicAdd(queue + kQueueMirrorExit, 1) ==
                      static_cast<int>(gridDim.x) - 1) {
    queue[kQueueMirror] = 0;
    queue[kQueueMirrorExit] = 0;
  }
}

template <int S_CT, int CB, int PT, bool FFT = false, int PREC = kPrecTail>
__global__ void __launch_bounds__(64 * IDG_GRID_NW, IDG_GRID_WAVES_GENERAL)
    kernel_gridder_general_mi355x(
        const int grid_size, int subgrid_size, float image_size,
        float w_step_in_lambda, int nr_channels, int nr_stations,
        const idg::UVWCoordinate<float> *__restrict__ uvw,
        const float *__restrict__ wavenumbers,
        const float2 *__restrict__ visibilities,
        const float *__restrict__ spheroidal,
        const float2 *__restrict__ aterms,
        const idg::Metadata *__restrict__ metadata,
        float2 *__restrict__ subgrids, int *__restrict__ queue,
        int nr_subgrids, int all) {
  constexpr int NW = IDG_GRID_NW;
  __shared__ unsigned lds[general_lds_words<S_CT, NW, 2 * PT>()];
  const int S = S_CT > 0 ? S_CT : subgrid_size;
  const int npix = S * S;
  const int tid = threadIdx.x;
  const QueueView qv = queue_view(queue, nr_subgrids);
  const int count = all ? nr_subgrids : qv.count();
  // An empty queue (every subgrid took the mirror path: the benchmark data)
  // leaves every counter at zero, so no workgroup takes a position or
  // retires: all return before any atomic (the resident grid's serialized
  // take and exit atomics were most of this launch's 15 us).
  if (count == 0) return;
  // the next queue position, taken by thread 0 and passed on through lds[0]
  // (between subgrids, where grid_mfma uses no LDS)
  if (tid == 0)
    lds[0] = static_cast<unsigned>(atomicAdd(queue + kQueueNext, 1));
  __syncthreads();
  int i = static_cast<int>(__builtin_amdgcn_readfirstlane(lds[0]));
  __syncthreads();
  while (i < count) {
    int next = 0;
    if (tid == 0) next = atomicAdd(queue + kQueueNext, 1);  // lands later
    const int s = all ? i : qv.at(i);
    const SubgridSetup g = setup_subgrid(metadata, s, grid_size, S,
                                         image_size, w_step_in_lambda);
    grid_mfma<S_CT, IDG_GRID_FUSED_GENERAL ? 2 * PT : PT, CB, NW, false, FFT,
              PREC>(
        g, S, npix, image_size, nr_channels, nr_stations, uvw, wavenumbers,
        visibilities, spheroidal, aterms,
        subgrids + static_cast<size_t>(s) * 4 * npix, lds);
    if (tid == 0) lds[0] = static_cast<unsigned>(next);
    __syncthreads();
    i = static_cast<int>(__builtin_amdgcn_readfirstlane(lds[0]));
    __syncthreads();
  }
  if (tid == 0) queue_retire(queue);
}

// The MFMA kernels of one (S, FFT epilogue, precision): the combined
// kernel (13-argument ABI) and the two-kernel form's mirror and general
// kernels.
struct GridderSet {
  const void *combined, *mirror, *general;
};
// The mirror kernel's workgroups per subgrid: the four S = 64 passes on
// four workgroups (IDG_GRID_SPLIT64=0: one, the A/B).
#ifndef IDG_GRID_SPLIT64
#define IDG_GRID_SPLIT64 1
#endif
// IDG_GRID_PERSIST=1 (A/B builds): the S = 32 mirror kernel in its
// persistent form (kernel_gridder_mirror_persist_mi355x).
#ifndef IDG_GRID_PERSIST
#define IDG_GRID_PERSIST 0
#endif
constexpr int mirror_split(int S) {
  return S == 64 && IDG_GRID_SPLIT64 ? 4 : 1;
}
template <int S_, bool FFT_, int PREC_>
const void *mirror_kernel() {
  if constexpr (IDG_GRID_PERSIST && S_ == 32)
    return reinterpret_cast<const void *>(
        &kernel_gridder_mirror_persist_mi355x<S_, 16, IDG_GRID_PT, FFT_,
                                              PREC_>);
  else
    return reinterpret_cast<const void *>(
        &kernel_gridder_mirror_mi355x<S_, 16, IDG_GRID_PT, FFT_, PREC_,
                                      mirror_split(S_)>);
}
template <int S_, int PPT_, bool FFT_, int PREC_>
GridderSet gridder_set() {
  return {reinterpret_cast<const void *>(
              &kernel_gridder_mi355x<S_, PPT_, 16, 1, IDG_GRID_PT, FFT_, PREC_>),
          mirror_kernel<S_, FFT_, PREC_>(),
          reinterpret_cast<const void *>(
              &kernel_gridder_general_mi355x<S_, 16, IDG_GRID_PT, FFT_, PREC_>)};
}
template <int S_, int PPT_, bool FFT_>
GridderSet gridder_set_for(int prec) {
  // the alternating tail replaces the every-phasor one in the gridder (the
  // degridder reads kPrecTail alone)
  if (prec & kPrecTailAlt) prec &= ~kPrecTail;
  if constexpr (S_ == 32) {
    switch (prec) {
      case 0: return gridder_set<S_, PPT_, FFT_, 0>();
      case kPrecTail | kPrecFlush:
        return gridder_set<S_, PPT_, FFT_, kPrecTail | kPrecFlush>();
      case kPrecFlush: return gridder_set<S_, PPT_, FFT_, kPrecFlush>();
      case kPrecTailAlt: return gridder_set<S_, PPT_, FFT_, kPrecTailAlt>();
      case kPrecTailAlt | kPrecFlush:
        return gridder_set<S_, PPT_, FFT_, kPrecTailAlt | kPrecFlush>();
      default: return gridder_set<S_, PPT_, FFT_, kPrecTail>();
    }
  } else {
    // no flush off S = 32 (the master needs a one-pass subgrid slot)
    if (prec & kPrecTailAlt) return gridder_set<S_, PPT_, FFT_, kPrecTailAlt>();
    return (prec & kPrecTail) ? gridder_set<S_, PPT_, FFT_, kPrecTail>()
                              : gridder_set<S_, PPT_, FFT_, 0>();
  }
}
#define IDG_GRIDDER_VALU(S_, PPT_)                                        \
  reinterpret_cast<const void *>(                                         \
      &kernel_gridder_mi355x<S_, PPT_, 16, 0, IDG_GRID_PT>)

// IDG_GRID_SPLIT=0: the device entries launch the one combined MFMA kernel
// (A/B of the two-launch form).
#ifndef IDG_GRID_SPLIT
#define IDG_GRID_SPLIT 1
#endif

// IDG_GRIDDER_IMPL=valu selects the VALU mirror path (A/B comparisons);
// IDG_GRIDDER_IMPL=sequential the order-preserving kernel, bit-exact to the
// reference's CPU output (sequential_mi355x.hip.cpp).
static int gridder_impl() {
  const char *v = std::getenv("IDG_GRIDDER_IMPL");
  if (v && std::string(v) == "sequential") return 2;
  return (v && std::string(v) == "valu") ? 0 : 1;
}

KernelChoice select_gridder(const Problem &p) {
  KernelChoice k;
  k.grid = p.nr_subgrids;
  if (gridder_impl() == 2) {
    k.func = sequential_gridder(p.subgrid_size);
    k.block = sequential_block();
    k.name = p.subgrid_size == 32   ? "gridder_sequential_mi355x_s32"
             : p.subgrid_size == 64 ? "gridder_sequential_mi355x_s64"
                                    : "gridder_sequential_mi355x_generic";
    return k;  // no FFT epilogue: launch() runs launch_subgrid_fft after it
  }
  const bool mfma = gridder_impl() == 1;
  k.block = mfma ? 64 * IDG_GRID_NW : kBlock;
  // the options the selected kernel is built with (reported by
  // idg_precision_options / bench.py): the alternating tail replaces the
  // every-phasor one, blocked summation exists at S = 32 only, and the VALU
  // kernel has none of them
  k.prec = precision_for(Direction::kGridder, p);
  if (k.prec & kPrecTailAlt) k.prec &= ~kPrecTail;
  if (p.subgrid_size != 32) k.prec &= ~kPrecFlush;
  if (!mfma) k.prec = 0;
  // the FFT in the gridder's epilogue (S = 32, MFMA; IDG_GRID_FFT=0: the
  // launch layer runs launch_subgrid_fft after the plain gridder instead)
  const char *fenv = std::getenv("IDG_GRID_FFT");
  const bool fft_epilogue = p.fft_out && mfma && p.subgrid_size == 32 &&
                            !(fenv != nullptr && fenv[0] == '0');
  GridderSet set{};
  switch (p.subgrid_size) {
    case 32:
      set = fft_epilogue ? gridder_set_for<32, 4, true>(k.prec)
                         : gridder_set_for<32, 4, false>(k.prec);
      k.name = fft_epilogue ? "gridder_fft_mi355x_s32"
                            : (mfma ? "gridder_mi355x_s32"
                                    : "gridder_mi355x_s32_valu");
      k.fft_in_kernel = fft_epilogue;
      if (!mfma) set.combined = IDG_GRIDDER_VALU(32, 4);
      break;
    case 64:
      set = gridder_set_for<64, 4, false>(k.prec);
      k.name = mfma ? "gridder_mi355x_s64" : "gridder_mi355x_s64_valu";
      if (!mfma) set.combined = IDG_GRIDDER_VALU(64, 4);
      break;
    default:
      set = gridder_set_for<0, 2, false>(k.prec);
      k.name = mfma ? "gridder_mi355x_generic" : "gridder_mi355x_generic_valu";
      // odd S has no mirror pairs: one general-only launch
      if (p.subgrid_size % 2 != 0) set.mirror = nullptr;
      if (!mfma) set.combined = IDG_GRIDDER_VALU(0, 2);
      break;
  }
  k.func = set.combined;
  if (mfma && IDG_GRID_SPLIT && two_kernel_form(p.nr_subgrids)) {
    if (set.mirror)
      k.parts[0] = {set.mirror, k.block, KernelChoice::kMirror,
                    p.subgrid_size == 64 ? mirror_split(64)
                    : IDG_GRID_PERSIST && p.subgrid_size == 32 ? 0
                                                               : 1};
    k.parts[1] = {set.general, k.block, KernelChoice::kGeneral};
    // no subgrid mirror-eligible: the combined kernel, one workgroup per
    // subgrid (2.7 % faster on a w-term batch than the queue-fed kernel)
    k.all_general = {k.func, k.block, KernelChoice::kPlain};
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
  // func = nullptr: c_run_gridder_ selects the MI355X kernel for the
  // problem (S, C, IDG_GRIDDER_IMPL) and launches it with that kernel's own
  // block size, so no thread count is passed.
  c_run_gridder_(nr_subgrids, grid_size, subgrid_size, image_size,
                 w_step_in_lambda, nr_channels, nr_stations, uvw, wavenumbers,
                 visibilities, spheroidal, aterms, metadata, subgrids, nullptr,
                 0);
}

}  // namespace hip

#if defined(IDG_WG_TIMELINE) && IDG_WG_TIMELINE
// Debug builds only: the last combined-gridder launch's workgroup stamps
// (tools/debug/wg_timeline.py).
extern "C" int idg_debug_timeline_gridder_copy(void *host, int n) {
  return hipMemcpyFromSymbol(
      host, HIP_SYMBOL(idg_mi355x::idg_debug_timeline_gridder),
      sizeof(WgStamp) * std::min(n, kTimelineMax));
}
#endif
