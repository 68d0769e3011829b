// degridder_mi355x.hip.cpp -- IDG degridder for MI355X (gfx950).
//
// Replaces the reference's app/HIP/kernels/degridder_*.hip.cpp behind the same
// kernel-TU contract (hip::p_run_degridder, hip::c_run_degridder; harness
// declarations tests/degridder_common.cpp:13-31) and 13-argument kernel ABI
// (grid = nr_subgrids; block = 256 = 4 wave64, or 512 = 8 wave64 for
// launches below kDegridSmallLaunch subgrids, select_degridder).  It computes
// cpu::kernel_degridder_reference
// (app/CPU/kernels/degridder_reference.cpp:6-129):
//
//   P'(y,x) = A1 * (sph * P(y,x)) * A2^H
//   V_p(t,c) = sum_{y,x} P'_p(y,x) * exp(i*phase),
//   phase    = fl(phase_index(t,y,x) * k_c - phase_offset(y,x))   [one FMA]
//
// Design:
//  * one workgroup per subgrid; default (MODE 1): per channel a real f16
//    two-term-split GEMM timesteps x pixel pairs x correlation components
//    on v_mfma_f32_16x16x32_f16 (degrid_mfma below); B (the A-termed,
//    tapered pixels) is built once per subgrid into LDS;
//  * the fp32 phase is formed exactly as the reference rounds it and reduced
//    as fma(phase, 1/2pi_hi, -m) + c with an integer m per (timestep, pixel,
//    16-channel block) and c the k * phase_index part of the tail of
//    1/2pi_hi; its phase_offset part is applied to the pixels (device.hpp:
//    kPhaseTail, phase_tail, tail_k_rev);
//  * mirror pixels (even S, w = 0, w_offset = 0): phase(S-1-y, S-1-x) =
//    -phase(y, x) exactly, so each sin/cos pair serves a pixel pair;
//  * IDG_DEGRIDDER_IMPL=valu (MODE 0): the all-VALU kernel, a lane per
//    (timestep, channel group) unit, 16 v_fma_f32 per (pixel, t, c), phase
//    anchored per channel group with a Dekker-split 1/(2*pi) (A/B reference).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <string>

#include "../util.hpp"
#include "device.hpp"
#include "lib-hip.hpp"
#include "mfma.hpp"

// waves-per-SIMD launch bound of the MFMA degridder (tuning knob)
// channels per MFMA pass (accumulators per wave) and per phase anchor
#ifndef IDG_DEGRID_CT
#define IDG_DEGRID_CT 16
#endif
#ifndef IDG_DEGRID_CB
#define IDG_DEGRID_CB 16
#endif
#ifndef IDG_DEGRID_WAVES
#define IDG_DEGRID_WAVES 4
#endif
// A subgrid of several K-chunks (S = 64; the general path of the combined
// kernel) takes its f16 scale per chunk, from the chunk's own entries, as a
// single-chunk subgrid does (round 5).  IDG_DEGRID_CHUNK_SCALE=0: one scale
// per subgrid from a pass over every pixel entry before the first chunk --
// whose bytes the later chunks then re-read from beyond L2 (configs[4]
// degridder 29.43 -> 29.0 ms, 11.86 -> 10.08 GB per launch; DESIGN.md
// §5.000).
#ifndef IDG_DEGRID_CHUNK_SCALE
#define IDG_DEGRID_CHUNK_SCALE 1
#endif

namespace idg_mi355x {

constexpr int kChunk = 1024;  // general path: pixels per LDS table chunk
// below this many subgrids the MFMA degridder runs 8-wave workgroups
#ifndef IDG_DEGRID_SMALL
#define IDG_DEGRID_SMALL 4096
#endif
constexpr int kDegridSmallLaunch = IDG_DEGRID_SMALL;
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

// A pixel entry's 4 correlations (pa = xx|xy, pb = yx|yy) times (c, s).
__device__ __forceinline__ void rotate_entry(float4 &pa, float4 &pb, float c,
                                             float s) {
  float v[8] = {pa.x, pa.y, pa.z, pa.w, pb.x, pb.y, pb.z, pb.w};
  rotate4(v, c, s);
  pa = make_float4(v[0], v[1], v[2], v[3]);
  pb = make_float4(v[4], v[5], v[6], v[7]);
}

// ---------------------------------------------------------------------------
// MFMA mirror path (even S, w = 0 for every timestep, w_offset = 0).
//
// A base pixel b and its mirror m have exactly negated phases, so their
// contribution to a visibility is
//   P'_b e^{i phi} + P'_m e^{-i phi} = cos(phi) * S + i sin(phi) * D,
//   S = P'_b + P'_m,  D = P'_b - P'_m,
// a real GEMM per channel over pixel pairs:
//   O[t][col] += sum_k A[t][k] * B[k][col]             (v_mfma_f32_16x16x32_f16)
//   A rows = 16 timesteps (lane l%16), K-block of lane group g = 2 pixel
//   pairs (p0, p1) as [c0_h, c1_h, c0_l, c1_l, s0_h, s1_h, s0_l, s1_l],
//   B rows = (Bc0, Bc1, Bc0, Bc1, Bs0, Bs1, Bs0, Bs1) with cos row
//   Bc = (S.re | S.im) and sin row Bs = (-D.im | D.re) per correlation,
//   columns [8 components hi | 8 lo] of the f16 split.
// B does not depend on the timestep or channel: its fragments -- 2 dwords
// (x = Bc pair, y = Bs pair) per lane per K-step of 8 pairs -- and the pair
// geometry are built ONCE per chunk of KP pairs (the whole subgrid when
// npix/2 <= KP) and reused by every timestep block and channel tile.
// Per phasor: 1 packed phase instruction, v_sin + v_cos, 3 split
// instructions, half an MFMA.
// ---------------------------------------------------------------------------
#ifndef IDG_DEGRID_BSCALE
#define IDG_DEGRID_BSCALE 13
#endif

template <int KP>
struct DegridMfmaLds {
  static constexpr int kGeoWords = KP * 4;              // l | m | poff | n
  static constexpr int kBfrWords = (KP / 8) * 64 * 2;   // uint2 per lane
  // 40 KiB at KP = 512: four workgroups per CU (the scale reduction reuses
  // the start of the geometry area before the first build)
  static constexpr int kWords = kGeoWords + kBfrWords;
};

// Revolutions of the phases of one pixel at the channel pair kp = (k_j,
// k_j+1):  fma(fma(p, k, o), 1/2pi_hi, -m) + c  with p, o, -m and c taken
// from half H of their (pixel 0, pixel 1) VGPR pairs and broadcast to both
// lanes by op_sel, so no operand is duplicated into a register pair (hipcc
// otherwise materialises the broadcasts or splits the packed FMA into two).
// The constant is the inline 1/(2 pi) = kInv2PiHi; m is the integer
// revolution count of the anchor block, c the k * phase_index part of the
// reduction's tail at the block's first channel (device.hpp: kPhaseTail,
// tail_k_rev).  A dependent packed-f32 VALU pair gets one wait state
// (s_nop 0), as hipcc pads its own; the output is read by compiler code,
// which pads after the asm itself.
// TAIL = false: the same without c (two v_pk_fma_f32).
template <int H, bool TAIL = true>
__device__ __forceinline__ floatx2 phase_rev_bcast(floatx2 p, floatx2 kp,
                                                   floatx2 o, floatx2 nm,
                                                   floatx2 cr) {
  floatx2 r;
  if constexpr (!TAIL && H == 0)
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,0]\n\t"
        "s_nop 0\n\t"
        "v_pk_fma_f32 %0, %0, 0.15915494, %4 op_sel_hi:[1,0,0]"
        : "=&v"(r)
        : "v"(p), "s"(kp), "v"(o), "v"(nm));
  else if constexpr (!TAIL)
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,1] op_sel_hi:[1,1,1]\n\t"
        "s_nop 0\n\t"
        "v_pk_fma_f32 %0, %0, 0.15915494, %4 op_sel:[0,0,1] "
        "op_sel_hi:[1,0,1]"
        : "=&v"(r)
        : "v"(p), "s"(kp), "v"(o), "v"(nm));
  else if constexpr (H == 0)
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,0]\n\t"
        "s_nop 0\n\t"
        "v_pk_fma_f32 %0, %0, 0.15915494, %4 op_sel_hi:[1,0,0]\n\t"
        "s_nop 0\n\t"
        "v_pk_add_f32 %0, %0, %5 op_sel_hi:[1,0]"
        : "=&v"(r)
        : "v"(p), "s"(kp), "v"(o), "v"(nm), "v"(cr));
  else
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,1] op_sel_hi:[1,1,1]\n\t"
        "s_nop 0\n\t"
        "v_pk_fma_f32 %0, %0, 0.15915494, %4 op_sel:[0,0,1] "
        "op_sel_hi:[1,0,1]\n\t"
        "s_nop 0\n\t"
        "v_pk_add_f32 %0, %0, %5 op_sel:[0,1] op_sel_hi:[1,1]"
        : "=&v"(r)
        : "v"(p), "s"(kp), "v"(o), "v"(nm), "v"(cr));
  return r;
}
static_assert(kInv2PiHi == 0.15915494f, "phase_rev_bcast's inline constant");

// KS: K split -- the workgroup's waves form KS groups of NW / KS waves;
// every group covers all timesteps and channel tiles, each over its own
// share of the chunk's K-steps (KS = 2: the 16-wave S = 64 mirror kernel,
// whose eight timestep waves would otherwise leave half the workgroup idle
// at T = 128).  Group 1 stores its partial sums, the workgroup barrier
// orders them (same CU: one L1), group 0 adds its own on top: p1 + p0, the
// same float as the two-chunk form's p0 + p1 (two-term addition commutes).
template <int S_CT, int CT, int CB, int KP, bool MIRROR, int NW,
          bool TAIL = true, int KS = 1>
__device__ __forceinline__ void degrid_mfma(
    const SubgridSetup &g, int S, int npix, float image_size, int C,
    int nr_stations, const idg::UVWCoordinate<float> *__restrict__ uvw,
    const float *__restrict__ wavenumbers, float2 *__restrict__ visibilities,
    const float *__restrict__ spheroidal, const float2 *__restrict__ aterms,
    const float2 *__restrict__ sg, unsigned *lds) {
  static_assert(CT % CB == 0 && CB % 2 == 0,
                "channel tiles hold whole, even anchor blocks");
  static_assert(KP % 32 == 0, "chunks hold whole 8-pair K-steps, 4 per pass");
  using L = DegridMfmaLds<KP>;
  constexpr int kThreads = 64 * NW;
  // General path: an opaque copy of the thread index, so values derived
  // from it are formed per call, not hoisted out of the general kernel's
  // loop over subgrids and kept live (spilled) across it (scratch 408 -> 160
  // B/lane gridder, 168 -> 68 degridder at S = 32; the mirror path, one
  // subgrid per workgroup, is better without it).
  int tid = threadIdx.x;
  if constexpr (!MIRROR) asm volatile("" : "+v"(tid));
  const int lane = tid & 63, wave = tid >> 6;
  const int grp = lane >> 4, col = lane & 15;
  static_assert(NW % KS == 0 && KS <= 2, "whole wave groups per K group");
  constexpr int kTWaves = NW / KS;  // waves per timestep pass
  const int wave_t = wave % kTWaves, wave_k = wave / kTWaves;
  // MIRROR: K runs over pixel pairs (b, npix-1-b); general: over single
  // pixels, as pairs whose mirror term is zero (S = D = P'), w-term on.
  const int half = MIRROR ? npix / 2 : npix;
  const int nt = g.nr_timesteps;

  // pair geometry, structure of arrays: l[KP], m[KP], phase_offset[KP]
  float *geo_l = reinterpret_cast<float *>(lds);
  float *geo_m = geo_l + KP;
  float *geo_o = geo_m + KP;
  float *geo_n = geo_o + KP;
  uint2 *bfr = reinterpret_cast<uint2 *>(lds + L::kGeoWords);
  const bool single = half <= KP;
  // the workgroup max of |P'| lands in red[] (the first geometry words,
  // before any geometry is written)
  float *red = reinterpret_cast<float *>(lds);
  auto block_max = [&](float v) {
    for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off));
    if (lane == 0) red[wave] = v;
    __syncthreads();
#pragma unroll
    for (int w = 0; w < NW; ++w) v = fmaxf(v, red[w]);
    __syncthreads();  // red[] is geometry space from here on
    return v;
  };
  auto absmax = [](const float4 &a, const float4 &b) {
    return fmaxf(fmaxf(fmaxf(fabsf(a.x), fabsf(a.y)),
                       fmaxf(fabsf(a.z), fabsf(a.w))),
                 fmaxf(fmaxf(fabsf(b.x), fabsf(b.y)),
                       fmaxf(fabsf(b.z), fabsf(b.w))));
  };

  // Pixel entries P' (and geometry) of pairs pc0 + 2q + h, h = 0, 1, of
  // K-block q: base in pa/pb, mirror in ma/mb (zero on general subgrids).
  struct Block {
    float4 pa[2], pb[2], ma[2], mb[2], geo[2];
  };
  auto entries = [&](int pc0, int q, Block &k) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int b = pc0 + 2 * q + h;
      const float4 z = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
      k.pa[h] = k.pb[h] = k.ma[h] = k.mb[h] = k.geo[h] = z;
      if (b < half) {
        pixel_entry(b, S, npix, image_size, g, nr_stations, spheroidal,
                    aterms, sg, k.pa[h], k.pb[h], k.geo[h]);
        // the phase tail of the reduction (device.hpp: kPhaseTail): the
        // pixel times exp(-i phase_offset eps), its mirror (phase_offset
        // exactly negated) times exp(+i phase_offset eps)
        float tc, ts;
        phase_tail(k.geo[h].w, &tc, &ts);
        rotate_entry(k.pa[h], k.pb[h], tc, -ts);
        if constexpr (MIRROR) {
          float4 mgeo;
          pixel_entry(npix - 1 - b, S, npix, image_size, g, nr_stations,
                      spheroidal, aterms, sg, k.ma[h], k.mb[h], mgeo);
          rotate_entry(k.ma[h], k.mb[h], tc, ts);
        }
      }
    }
  };
  // S = P'_b + P'_m and D = P'_b - P'_m of K-block q, scaled, split, and
  // written as the 16 column lanes' B fragments; the pairs' geometry too.
  auto store_block = [&](int q, const Block &k, float scale) {
    float sre[2][4], sim[2][4], dre[2][4], dim[2][4];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float pr[4] = {k.pa[h].x, k.pa[h].z, k.pb[h].x, k.pb[h].z};
      const float pi[4] = {k.pa[h].y, k.pa[h].w, k.pb[h].y, k.pb[h].w};
      const float mr[4] = {k.ma[h].x, k.ma[h].z, k.mb[h].x, k.mb[h].z};
      const float mi[4] = {k.ma[h].y, k.ma[h].w, k.mb[h].y, k.mb[h].w};
#pragma unroll
      for (int cr = 0; cr < 4; ++cr) {
        sre[h][cr] = (pr[cr] + mr[cr]) * scale;
        sim[h][cr] = (pi[cr] + mi[cr]) * scale;
        dre[h][cr] = (pr[cr] - mr[cr]) * scale;
        dim[h][cr] = (pi[cr] - mi[cr]) * scale;
      }
      geo_l[2 * q + h] = k.geo[h].x;
      geo_m[2 * q + h] = k.geo[h].y;
      geo_o[2 * q + h] = k.geo[h].w;
      if constexpr (!MIRROR) geo_n[2 * q + h] = k.geo[h].z;
    }
    // lane (g, col) of K-step ks: ks = q / 4, g = q % 4
    uint2 *dst = bfr + (q >> 2) * 64 + (q & 3) * 16;
#pragma unroll
    for (int cl = 0; cl < 16; ++cl) {
      const int cr = (cl & 7) >> 1;
      const bool im = cl & 1;
      const float bc0 = im ? sim[0][cr] : sre[0][cr];
      const float bc1 = im ? sim[1][cr] : sre[1][cr];
      const float bs0 = im ? dre[0][cr] : -dim[0][cr];
      const float bs1 = im ? dre[1][cr] : -dim[1][cr];
      dst[cl] = (cl & 8) ? make_uint2(split_lo(bc0, bc1), split_lo(bs0, bs1))
                         : make_uint2(split_hi(bc0, bc1), split_hi(bs0, bs1));
    }
  };

  // Per-chunk power-of-two scale: |S|, |D| <= 2 max|P'| stay in f16 range
  // (below 2^IDG_DEGRID_BSCALE: high in the range keeps the split's lo part
  // a normal f16 for all but the smallest pixels).
  auto scale_exp = [](float vmax) {
    int e = 0;
    if (vmax > 0.0f && vmax <= 3.0e38f) frexpf(vmax, &e);
    return e;
  };
  int e = 0;
  static_assert(KP / 2 <= kThreads, "one K-block per thread in a single chunk");
  constexpr bool kChunkScale = IDG_DEGRID_CHUNK_SCALE != 0;
  if (single) {
    // one chunk: every thread computes its K-block's entries once (NW = 8:
    // the upper half repeats the last K-block, for the max only), the
    // workgroup max sets the scale, and the same registers are split
    Block k;
    const bool has_block = tid < KP / 2;
    entries(0, has_block ? tid : KP / 2 - 1, k);
    float v = 0.0f;
#pragma unroll
    for (int h = 0; h < 2; ++h)
      v = fmaxf(v, fmaxf(absmax(k.pa[h], k.pb[h]), absmax(k.ma[h], k.mb[h])));
    e = scale_exp(2.0f * block_max(v));
    if (has_block) store_block(tid, k, ldexpf(1.0f, IDG_DEGRID_BSCALE - e));
    __syncthreads();
  } else if constexpr (!kChunkScale) {
    float v = 0.0f;
    for (int p = tid; p < npix; p += kThreads) {
      float4 pa, pb, geo;
      pixel_entry(p, S, npix, image_size, g, nr_stations, spheroidal, aterms,
                  sg, pa, pb, geo);
      v = fmaxf(v, absmax(pa, pb));
    }
    e = scale_exp(2.0f * block_max(v));
  }
  float scale = ldexpf(1.0f, IDG_DEGRID_BSCALE - e),
        unscale = ldexpf(1.0f, e - IDG_DEGRID_BSCALE);
  // B fragments and geometry of pairs [pc0, pc0 + KP): one thread per
  // K-block (2 pairs), writing all 16 column lanes of it.
  auto build = [&](int pc0) {
    if constexpr (kChunkScale) {
      // the chunk's own scale: every thread's K-block entries (the last
      // K-block again past KP/2, for the maximum only), the workgroup
      // maximum, then the split -- the single chunk's steps, per chunk
      Block k;
      const bool has_block = tid < KP / 2;
      entries(pc0, has_block ? tid : KP / 2 - 1, k);
      float v = 0.0f;
#pragma unroll
      for (int h = 0; h < 2; ++h)
        v = fmaxf(v, fmaxf(absmax(k.pa[h], k.pb[h]), absmax(k.ma[h], k.mb[h])));
      const int ec = scale_exp(2.0f * block_max(v));
      scale = ldexpf(1.0f, IDG_DEGRID_BSCALE - ec);
      unscale = ldexpf(1.0f, ec - IDG_DEGRID_BSCALE);
      if (has_block) store_block(tid, k, scale);
      return;
    }
    // an opaque copy of tid per call: the addresses derived from it are
    // formed here, not hoisted out of the chunk loop and kept live across
    // the MFMA loops (they were spilled: scratch 92 -> 36 B/lane at S = 32,
    // degridder counter traffic 2.95 -> 2.70 GB per launch)
    int q0 = tid;
    asm volatile("" : "+v"(q0));
    for (int q = q0; q < KP / 2; q += kThreads) {
      Block k;
      entries(pc0, q, k);
      store_block(q, k, scale);
    }
  };

  // Chunks of KP pairs are the outermost loop so that building the next
  // chunk never overlaps live accumulators (no spills); each chunk's partial
  // sums are added to the visibilities its own lanes wrote for the previous
  // chunk (same lane, same address: ordered, no atomics).
  for (int pc0 = 0; pc0 < half; pc0 += KP) {
    if (!single) {
      __syncthreads();
      build(pc0);
      __syncthreads();
    }
    // kTWaves waves x 16 timesteps per pass
    for (int t0 = 0; t0 < nt; t0 += 16 * kTWaves) {
      const int t_row = t0 + wave_t * 16 + col;  // this lane's A row timestep
      const idg::UVWCoordinate<float> c =
          uvw[g.time_offset + min(t_row, nt - 1)];
      for (int cg0 = 0; cg0 < C; cg0 += CT) {
        float kk[CT];
#pragma unroll
        for (int j = 0; j < CT; ++j) kk[j] = wavenumbers[min(cg0 + j, C - 1)];
        floatx4 acc[CT];
#pragma unroll
        for (int j = 0; j < CT; ++j) acc[j] = floatx4{0.0f, 0.0f, 0.0f, 0.0f};
        {
        const int nks = (min(KP, half - pc0) + 7) / 8;
        // this wave's K group's K-steps
        const int ks_per = (nks + KS - 1) / KS;
        const int ks_end = min(nks, (wave_k + 1) * ks_per);
        for (int ks = wave_k * ks_per; ks < ks_end; ++ks) {
          const int pp = 8 * ks + 2 * grp;
          const float2 gl = *reinterpret_cast<const float2 *>(geo_l + pp);
          const float2 gm = *reinterpret_cast<const float2 *>(geo_m + pp);
          const float2 go = *reinterpret_cast<const float2 *>(geo_o + pp);
          const uint2 bb = bfr[ks * 64 + lane];
          const half8 bf = pack4(bb.x, bb.x, bb.y, bb.y);
          // phase_index = fma(u, l, v*m) + w*n (w = 0 on mirror subgrids)
          floatx2 pidx = {fma_(c.u, gl.x, c.v * gm.x),
                          fma_(c.u, gl.y, c.v * gm.y)};
          if constexpr (!MIRROR) {
            const float2 gn = *reinterpret_cast<const float2 *>(geo_n + pp);
            pidx.x = pidx.x + c.w * gn.x;
            pidx.y = pidx.y + c.w * gn.y;
          }
          const floatx2 npoff = {-go.x, -go.y};
#pragma unroll
          for (int jb = 0; jb < CT; jb += CB) {
            // -m: the whole revolutions of the block's first-channel phase
            const floatx2 A = __builtin_elementwise_fma(
                pidx, floatx2{kk[jb], kk[jb]}, npoff);
            const floatx2 t = A * floatx2{kInv2PiHi, kInv2PiHi};
            const floatx2 nm = {-__builtin_rintf(t.x), -__builtin_rintf(t.y)};
            // the k * phase_index part of the reduction's tail at the
            // block's first channel (phase = k * phase_index - poff here)
            floatx2 cr = {0.0f, 0.0f};
            if constexpr (TAIL) cr = tail_k_rev(pidx, kk[jb]);
            // Packed over channel pairs (j, j+1) per pixel: the wavenumber
            // pair is one SGPR pair and the pixel's terms are broadcast from
            // their halves of the (pixel 0, pixel 1) pairs by op_sel, so the
            // phase chain is three v_pk_* per two phasors (same
            // fma(pidx, k, -poff) rounding as the scalar form).
#pragma unroll
            for (int j = jb; j < jb + CB; j += 2) {
              const floatx2 kp = {kk[j], kk[j + 1]};
              const floatx2 rx =
                  phase_rev_bcast<0, TAIL>(pidx, kp, npoff, nm, cr);
              const floatx2 ry =
                  phase_rev_bcast<1, TAIL>(pidx, kp, npoff, nm, cr);
              float s0, c0, s1, c1, s2, c2, s3, c3;
              sincos_rev(rx.x, &s0, &c0);  // channel j,   pixel 0
              sincos_rev(ry.x, &s1, &c1);  // channel j,   pixel 1
              sincos_rev(rx.y, &s2, &c2);  // channel j+1, pixel 0
              sincos_rev(ry.y, &s3, &c3);  // channel j+1, pixel 1
              half8 a01, a23;  // one asm block (one pair of pads) for both
              split_oct(c0, c1, s0, s1, c2, c3, s2, s3, &a01, &a23);
              acc[j] = mfma16(a01, bf, acc[j]);
              acc[j + 1] = mfma16(a23, bf, acc[j + 1]);
            }
          }
          // one K-step's MFMAs stay in their iteration
          IDG_KSTEP_FENCE();
        }
      }

      // D rows = timesteps wave*16 + grp*4 + r, col = component (hi | lo).
      // hi + lo: row_ror:8 adds lane col+8 to lane col (and col to col+8),
      // so both half-rows hold the component sums; lanes col < 8 take
      // channel j's, lanes col >= 8 channel j+1's, and each 16-lane group
      // writes the two adjacent 32-byte visibilities (t, j), (t, j+1) as one
      // contiguous 64-byte store -- no LDS shuffle, no inactive lanes.
      const bool full_tc = t0 + 16 * kTWaves <= nt && cg0 + CT <= C;
      auto store = [&](bool add) {
      if (full_tc) {
        float *vrow = reinterpret_cast<float *>(visibilities) +
                      (static_cast<size_t>(g.time_offset + t0 + wave_t * 16 +
                                           grp * 4) * C + cg0) * 8 + col;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float *dst = vrow + static_cast<size_t>(r) * C * 8;
#pragma unroll
          for (int j = 0; j < CT; j += 2) {
            const float v0 = acc[j][r], v1 = acc[j + 1][r];
            const float s0 = v0 + row_ror8(v0);
            const float s1 = v1 + row_ror8(v1);
            const float out = (col < 8 ? s0 : s1) * unscale;
            if (!add)
              dst[8 * j] = out;
            else
              dst[8 * j] += out;
          }
        }
      } else {
#pragma unroll
      for (int j = 0; j < CT; ++j) {
        const int ch = cg0 + j;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = acc[j][r];
          const float other = __shfl_xor(v, 8);
          const int t = t0 + wave_t * 16 + grp * 4 + r;
          if (col < 8 && t < nt && ch < C) {
            float *dst = reinterpret_cast<float *>(
                visibilities + ((g.time_offset + t) * C + ch) * 4);
            const float out = (v + other) * unscale;
            dst[col] = !add ? out : dst[col] + out;
          }
        }
      }
      }
      };
      if constexpr (KS == 1) {
        store(pc0 != 0);
      } else {
        // group 1's partial sums first, then group 0's added on top
        if (wave_k == 1) store(pc0 != 0);
        __syncthreads();
        if (wave_k == 0) store(true);
      }
    }
  }
  }
}

}  // namespace

#if defined(IDG_WG_TIMELINE) && IDG_WG_TIMELINE
__device__ WgStamp idg_debug_timeline_degridder[kTimelineMax];
#endif

// CG: channels per lane (VALU paths).
// MODE: 0 = VALU kernel, 1 = MFMA kernel (mirror GEMMs on eligible
//       subgrids, single-pixel GEMMs with the w-term on the others).
// CT: channels per MFMA pass.
// NW: waves per workgroup of the MFMA kernel (4; 8 for small launches, whose
//     drain is then half as long: select_degridder).
// (One launch over every subgrid, each on its path: the reference's launch
// shape.  The device entries launch the two-kernel form instead:
// kernel_degridder_mirror_mi355x + kernel_degridder_general_mi355x.)
template <int S_CT, int CG, int MODE, int CT, int NW, bool TAIL = true>
__global__ void __launch_bounds__(MODE == 1 ? 64 * NW : kBlock,
                                  MODE == 1 ? IDG_DEGRID_WAVES : 1)
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
  const int S = S_CT > 0 ? S_CT : subgrid_size;
  const int npix = S * S;
  const int s = xcd_subgrid(blockIdx.x, gridDim.x);
  const int tid = threadIdx.x;
  const SubgridSetup g = setup_subgrid(metadata, s, grid_size, S, image_size,
                                       w_step_in_lambda);
  const float2 *sg = subgrids + static_cast<size_t>(s) * 4 * npix;
  const int C = nr_channels;

  if constexpr (MODE == 1) {
    // chunks of 512 K-pairs (the whole S = 32 subgrid on mirror subgrids)
    constexpr int KP = 512;
    __shared__ unsigned lds[DegridMfmaLds<KP>::kWords];
    // Subgrid-uniform mirror eligibility: even S, w_offset = 0 and w = 0 on
    // every timestep.  Reduced through lds[0] rather than __syncthreads_or,
    // whose library implementation adds 256 B of LDS and would cost the
    // fourth workgroup per CU.
    if (tid == 0) lds[0] = 0u;
    __syncthreads();
    bool w_nonzero = false;
    for (int t = tid; t < g.nr_timesteps; t += 64 * NW)
      w_nonzero |= uvw[g.time_offset + t].w != 0.0f;
    if (w_nonzero) atomicOr(&lds[0], 1u);
    __syncthreads();
    const bool eligible = lds[0] == 0u && S % 2 == 0 && g.w_offset == 0.0f;
    __syncthreads();
#if defined(IDG_WG_TIMELINE) && IDG_WG_TIMELINE
    timeline_start(idg_debug_timeline_degridder);
#endif
    if (eligible)
      degrid_mfma<S_CT, CT, IDG_DEGRID_CB, KP, true, NW, TAIL>(
          g, S, npix, image_size, C, nr_stations, uvw, wavenumbers,
          visibilities, spheroidal, aterms, sg, lds);
    else
      degrid_mfma<S_CT, CT, IDG_DEGRID_CB, KP, false, NW, TAIL>(
          g, S, npix, image_size, C, nr_stations, uvw, wavenumbers,
          visibilities, spheroidal, aterms, sg, lds);
#if defined(IDG_WG_TIMELINE) && IDG_WG_TIMELINE
    timeline_end(idg_debug_timeline_degridder);
#endif
    return;
  }

  // general: [pixel][0..1] = P' (xx, xy | yx, yy), [pixel][2] = (l,m,n,poff)
  // mirror : [pair][0..1] = P'(base), [pair][2..3] = P'(mirror),
  //          [pair][4] = geometry of the base pixel
  __shared__ float4 table[kChunk * 3];
  static_assert(kPairChunk * 5 <= kChunk * 3, "table size");
  constexpr int CGV = CG;
  const int ncg = (C + CGV - 1) / CGV;
  const int nunits = g.nr_timesteps * ncg;
  const bool mirror_ok = (S % 2 == 0) && g.w_offset == 0.0f;

  for (int ubase = 0; ubase < nunits; ubase += kBlock) {
    const int unit = min(ubase + tid, nunits - 1);
    const bool active = ubase + tid < nunits;
    const int t = unit / ncg;
    const int c0 = (unit - t * ncg) * CGV;
    const long long row = g.time_offset + t;
    const idg::UVWCoordinate<float> c = uvw[row];
    float k[CGV];
#pragma unroll
    for (int j = 0; j < CGV; ++j) k[j] = wavenumbers[min(c0 + j, C - 1)];
    float acc[CGV][8];
#pragma unroll
    for (int j = 0; j < CGV; ++j)
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
          for (int j = 0; j < CGV; ++j) {
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
          for (int j = 0; j < CGV; ++j) {
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
      for (int j = 0; j < CGV; ++j) {
        if (c0 + j < C) {
          dst[2 * j] = make_float4(acc[j][0], acc[j][1], acc[j][2], acc[j][3]);
          dst[2 * j + 1] =
              make_float4(acc[j][4], acc[j][5], acc[j][6], acc[j][7]);
        }
      }
    }
  }
}

// The two-kernel form of the device entries (select_degridder; DESIGN.md
// §4.2), as the gridder's (gridder_mi355x.hip.cpp): the mirror kernel,
// grid = nr_subgrids, degrids the mirror-eligible subgrids and queues the
// others (device.hpp: queue_push); the general kernel, a resident grid of
// 8-wave workgroups, takes the queued subgrids one at a time from the
// queue's take counter (all subgrids, with no mirror launch, when `all` is
// set: odd S or w_step_in_lambda != 0) and degrids each with chunks of
// KP = 1,024 single pixels (one thread per
// K-block of the 512), so an S = 32 subgrid is one chunk and its
// visibilities are written once (the combined kernel's 512-pixel chunks
// read them back and wrote them again).
// IDG_DEGRID_KP64=512: the S = 64 8-wave mirror kernel keeps 512-pair
// chunks (A/B); the two-kernel form takes the 8-wave one at S = 64
#ifndef IDG_DEGRID_KP64
#define IDG_DEGRID_KP64 1024
#endif
constexpr int mirror_kp64() { return IDG_DEGRID_KP64; }

// KPX > 0: pairs per chunk (else as below); KS: K split (degrid_mfma).
// The S = 64 single-chunk form (round 6): KPX = 2,048 -- the whole
// subgrid's pairs, 160 KB of LDS, one 16-wave workgroup per CU in two K
// groups of 8 waves -- so the visibilities are written once
// instead of written, read back and written again (the two-chunk form's
// 2.08x the algorithmic bytes, profiles/r05/kernels_s64).
template <int S_CT, int CT, int NW, bool TAIL = true, int KPX = 0,
          int KS = 1>
__global__ void __launch_bounds__(64 * NW, IDG_DEGRID_WAVES)
    kernel_degridder_mirror_mi355x(
        const int grid_size, int subgrid_size, float image_size,
        float w_step_in_lambda, int nr_channels, int nr_stations,
        const idg::UVWCoordinate<float> *__restrict__ uvw,
        const float *__restrict__ wavenumbers,
        float2 *__restrict__ visibilities,
        const float *__restrict__ spheroidal,
        const float2 *__restrict__ aterms,
        const idg::Metadata *__restrict__ metadata,
        const float2 *__restrict__ subgrids, int *__restrict__ queue) {
  // S = 64 on 8 waves: 1,024-pair chunks (80 KB of LDS, two workgroups per
  // CU: the occupancy of four 4-wave ones), so a subgrid is two chunks, not
  // four, and its visibilities are written, read back and written again
  // once instead of three times (profiles/r04/kernels_s64: 18.7 GB per
  // launch against 4.85 GB algorithmic)
  constexpr int KP =
      KPX > 0 ? KPX : (S_CT == 64 && NW == 8) ? mirror_kp64() : 512;
  __shared__ unsigned lds[DegridMfmaLds<KP>::kWords];
  const int S = S_CT > 0 ? S_CT : subgrid_size;
  const int npix = S * S;
  const int s = xcd_subgrid(blockIdx.x, gridDim.x);
  const int tid = threadIdx.x;
  const SubgridSetup g = setup_subgrid(metadata, s, grid_size, S, image_size,
                                       w_step_in_lambda);
  // eligibility reduced through lds[0] (see kernel_degridder_mi355x)
  if (tid == 0) lds[0] = 0u;
  __syncthreads();
  bool w_nonzero = false;
  for (int t = tid; t < g.nr_timesteps; t += 64 * NW)
    w_nonzero |= uvw[g.time_offset + t].w != 0.0f;
  if (w_nonzero) atomicOr(&lds[0], 1u);
  __syncthreads();
  const bool eligible = lds[0] == 0u && S % 2 == 0 && g.w_offset == 0.0f;
  __syncthreads();
  if (!eligible) {
    if (tid == 0) queue_push(queue, gridDim.x, s);
    return;
  }
  degrid_mfma<S_CT, CT, IDG_DEGRID_CB, KP, true, NW, TAIL, KS>(
      g, S, npix, image_size, nr_channels, nr_stations, uvw, wavenumbers,
      visibilities, spheroidal, aterms,
      subgrids + static_cast<size_t>(s) * 4 * npix, lds);
}

// IDG_DEGRID_S64=1: the S = 64 mirror kernel of the two-kernel form in the
// single-chunk form above; 2 (default): the two-chunk form (8 waves,
// 1,024-pair chunks).  Measured on one box (profiles/r06/s64_single/): the
// single chunk moves 7.01 GB per launch against 10.09 (5.23 GB with the
// channel groups split instead of K, at 33.7 ms) but runs 32.5 ms against
// 29.3: with one workgroup per CU nothing overlaps its chunk build and the
// partial-sum hand-over, which the two-chunk form's second workgroup hides.
#ifndef IDG_DEGRID_S64
#define IDG_DEGRID_S64 2
#endif
template <bool TAIL>
const void *degridder_mirror_s64_single() {
  return reinterpret_cast<const void *>(
      &kernel_degridder_mirror_mi355x<64, IDG_DEGRID_CT, 16, TAIL, 2048, 2>);
}

template <int S_CT, int CT, bool TAIL = true>
__global__ void __launch_bounds__(512, IDG_DEGRID_WAVES)
    kernel_degridder_general_mi355x(
        const int grid_size, int subgrid_size, float image_size,
        float w_step_in_lambda, int nr_channels, int nr_stations,
        const idg::UVWCoordinate<float> *__restrict__ uvw,
        const float *__restrict__ wavenumbers,
        float2 *__restrict__ visibilities,
        const float *__restrict__ spheroidal,
        const float2 *__restrict__ aterms,
        const idg::Metadata *__restrict__ metadata,
        const float2 *__restrict__ subgrids, int *__restrict__ queue,
        int nr_subgrids, int all) {
  constexpr int NW = 8, KP = 1024;
  __shared__ unsigned lds[DegridMfmaLds<KP>::kWords];
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
  // (between subgrids, where degrid_mfma uses no LDS)
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
    degrid_mfma<S_CT, CT, IDG_DEGRID_CB, KP, false, NW, TAIL>(
        g, S, npix, image_size, nr_channels, nr_stations, uvw, wavenumbers,
        visibilities, spheroidal, aterms,
        subgrids + static_cast<size_t>(s) * 4 * npix, lds);
    __syncthreads();  // every wave is done with the LDS tables
    if (tid == 0) lds[0] = static_cast<unsigned>(next);
    __syncthreads();
    i = static_cast<int>(__builtin_amdgcn_readfirstlane(lds[0]));
    __syncthreads();
  }
  if (tid == 0) queue_retire(queue);
}

// The general path alone, one 8-wave workgroup per subgrid with KP = 1,024
// (grid = nr_subgrids, the 13-argument ABI): the device entries' launch
// when no subgrid can be mirror-eligible (odd S, or w_step_in_lambda != 0:
// every w_offset is then non-zero).  The general path is the generic
// computation, valid for any subgrid.  On a w-term batch this runs 2-3 %
// faster than the queue-fed general kernel above, whose workgroups loop
// over subgrids.
template <int S_CT, int CT, bool TAIL = true>
__global__ void __launch_bounds__(512, IDG_DEGRID_WAVES)
    kernel_degridder_general_direct_mi355x(
        const int grid_size, int subgrid_size, float image_size,
        float w_step_in_lambda, int nr_channels, int nr_stations,
        const idg::UVWCoordinate<float> *__restrict__ uvw,
        const float *__restrict__ wavenumbers,
        float2 *__restrict__ visibilities,
        const float *__restrict__ spheroidal,
        const float2 *__restrict__ aterms,
        const idg::Metadata *__restrict__ metadata,
        const float2 *__restrict__ subgrids) {
  constexpr int NW = 8, KP = 1024;
  __shared__ unsigned lds[DegridMfmaLds<KP>::kWords];
  const int S = S_CT > 0 ? S_CT : subgrid_size;
  const int npix = S * S;
  const int s = xcd_subgrid(blockIdx.x, gridDim.x);
  const SubgridSetup g = setup_subgrid(metadata, s, grid_size, S, image_size,
                                       w_step_in_lambda);
  degrid_mfma<S_CT, CT, IDG_DEGRID_CB, KP, false, NW, TAIL>(
      g, S, npix, image_size, nr_channels, nr_stations, uvw, wavenumbers,
      visibilities, spheroidal, aterms,
      subgrids + static_cast<size_t>(s) * 4 * npix, lds);
}

#define IDG_DEGRIDDER_VALU(S_, CG_)                                       \
  reinterpret_cast<const void *>(                                         \
      &kernel_degridder_mi355x<S_, CG_, 0, IDG_DEGRID_CT, 4>)

// The MFMA kernels of one (S, waves per workgroup, tail): the combined
// kernel and the two-kernel form's mirror, queue-fed general and direct
// all-general kernels.
struct DegridderSet {
  const void *combined, *mirror, *general, *general_direct;
};
template <int S_, int NW_, bool TAIL_>
DegridderSet degridder_set() {
  return {reinterpret_cast<const void *>(
              &kernel_degridder_mi355x<S_, 4, 1, IDG_DEGRID_CT, NW_, TAIL_>),
          reinterpret_cast<const void *>(
              &kernel_degridder_mirror_mi355x<S_, IDG_DEGRID_CT, NW_, TAIL_>),
          reinterpret_cast<const void *>(
              &kernel_degridder_general_mi355x<S_, IDG_DEGRID_CT, TAIL_>),
          reinterpret_cast<const void *>(
              &kernel_degridder_general_direct_mi355x<S_, IDG_DEGRID_CT,
                                                      TAIL_>)};
}
template <int S_>
DegridderSet degridder_set_for(bool nw8, bool tail) {
  if (nw8)
    return tail ? degridder_set<S_, 8, true>() : degridder_set<S_, 8, false>();
  return tail ? degridder_set<S_, 4, true>() : degridder_set<S_, 4, false>();
}

// IDG_DEGRID_SPLIT=0: the device entries launch the one combined MFMA
// kernel (A/B of the two-launch form).
#ifndef IDG_DEGRID_SPLIT
#define IDG_DEGRID_SPLIT 1
#endif

// IDG_DEGRIDDER_IMPL=valu selects the VALU mirror path (A/B comparisons).
static int degridder_impl() {
  const char *v = std::getenv("IDG_DEGRIDDER_IMPL");
  if (v && std::string(v) == "sequential") return 2;
  return (v && std::string(v) == "valu") ? 0 : 1;
}

KernelChoice select_degridder(const Problem &p) {
  KernelChoice k;
  k.grid = p.nr_subgrids;
  if (degridder_impl() == 2) {  // bit-exact to the reference's CPU output
    k.func = sequential_degridder(p.subgrid_size);
    k.block = sequential_block();
    k.name = p.subgrid_size == 32   ? "degridder_sequential_mi355x_s32"
             : p.subgrid_size == 64 ? "degridder_sequential_mi355x_s64"
                                    : "degridder_sequential_mi355x_generic";
    return k;
  }
  k.block = kBlock;
  const int C = p.nr_channels;
  const bool cg8 = C % 8 == 0 || (C % 4 != 0 && C >= 8);
  const bool s32 = p.subgrid_size == 32, s64 = p.subgrid_size == 64;
  const bool mfma = degridder_impl() == 1;
  // Small launches (a shard of the batch: 3,063 subgrids at N = 8) take
  // 8-wave workgroups: half the workgroup duration, so half the drain of
  // the last round (0.926 vs 0.935 ms at 3,063 subgrids); large ones keep
  // 4 waves (7.18 vs 7.21-7.26 ms at 24,500).  Same
  // arithmetic, bitwise identical outputs.
  bool nw8 = mfma && p.nr_subgrids < kDegridSmallLaunch;
  // IDG_DEGRID_NW=4 / 8 forces the workgroup size (tests; read per call)
  if (const char *v = std::getenv("IDG_DEGRID_NW"))
    nw8 = mfma && std::string(v) == "8";
  if (mfma) {
    k.prec = precision_for(Direction::kDegridder, p);
    const bool tail = (k.prec & kPrecTail) != 0;
    const DegridderSet set = s32   ? degridder_set_for<32>(nw8, tail)
                             : s64 ? degridder_set_for<64>(nw8, tail)
                                   : degridder_set_for<0>(nw8, tail);
    // the MFMA kernel has no CG
    k.func = set.combined;
    k.block = nw8 ? 512 : 256;
    if (IDG_DEGRID_SPLIT && two_kernel_form(p.nr_subgrids)) {
      // mirror-eligible subgrids (even S only), then the others on 8-wave
      // workgroups with 1,024-pixel chunks
      if (s64 && IDG_DEGRID_S64 == 1)  // 16 waves, one 2,048-pair chunk
        k.parts[0] = {tail ? degridder_mirror_s64_single<true>()
                           : degridder_mirror_s64_single<false>(),
                      1024, KernelChoice::kMirror};
      else if (s64 && mirror_kp64() > 512)  // 8 waves, 1,024-pair chunks
        k.parts[0] = {degridder_set_for<64>(true, tail).mirror, 512,
                      KernelChoice::kMirror};
      else if (p.subgrid_size % 2 == 0)
        k.parts[0] = {set.mirror, k.block, KernelChoice::kMirror};
      k.parts[1] = {set.general, 512, KernelChoice::kGeneral};
      k.all_general = {set.general_direct, 512, KernelChoice::kPlain};
    }
  } else {
    k.func = s32   ? (cg8 ? IDG_DEGRIDDER_VALU(32, 8) : IDG_DEGRIDDER_VALU(32, 4))
             : s64 ? (cg8 ? IDG_DEGRIDDER_VALU(64, 8) : IDG_DEGRIDDER_VALU(64, 4))
                   : (cg8 ? IDG_DEGRIDDER_VALU(0, 8) : IDG_DEGRIDDER_VALU(0, 4));
  }
  if (mfma)
    k.name = s32 ? "degridder_mi355x_s32"
                 : (s64 ? "degridder_mi355x_s64" : "degridder_mi355x_generic");
  else
    k.name = s32 ? "degridder_mi355x_s32_valu"
                 : (s64 ? "degridder_mi355x_s64_valu"
                        : "degridder_mi355x_generic_valu");
  return k;
}

}  // namespace idg_mi355x

namespace hip {

void p_run_degridder() {
  idg_mi355x::Problem p;
  p.subgrid_size = static_cast<int>(get_env_var("SUBGRID_SIZE", 32));
  p.nr_channels = static_cast<int>(get_env_var("NR_CHANNELS", 16));
  // the batch run_performance builds (the kernel choice depends on its size)
  const int nr_stations = static_cast<int>(get_env_var("NR_STATIONS", 50));
  p.nr_subgrids = nr_stations * (nr_stations - 1) / 2 *
                  static_cast<int>(get_env_var("NR_TIMESLOTS", 20));
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

#if defined(IDG_WG_TIMELINE) && IDG_WG_TIMELINE
// Debug builds only: the last combined-degridder launch's workgroup stamps
// (tools/debug/wg_timeline.py).
extern "C" int idg_debug_timeline_degridder_copy(void *host, int n) {
  return hipMemcpyFromSymbol(
      host, HIP_SYMBOL(idg_mi355x::idg_debug_timeline_degridder),
      sizeof(WgStamp) * std::min(n, kTimelineMax));
}
#endif
