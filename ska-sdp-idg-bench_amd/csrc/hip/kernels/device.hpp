// device.hpp -- gfx950 device helpers shared by the gridder and degridder.
//
// Compiled with -ffp-contract=off: every fused multiply-add below is an
// explicit __builtin_fmaf, so the phase arithmetic rounds exactly as the
// reference build does (oracle/idg_oracle.c).
#pragma once

#include <hip/hip_runtime.h>

#include "common/math.hpp"
#include "common/types.hpp"

namespace idg_mi355x {

constexpr int kBlock = 256;  // 4 wave64 per workgroup

typedef float floatx2 __attribute__((ext_vector_type(2)));  // as mfma.hpp

// 1/(2*pi) split into a float head and tail: head + tail = 1/(2*pi) to ~2^-52.
constexpr float kInv2PiHi = 0x1.45f306p-3f;
constexpr float kInv2PiLo = 0x1.b9391p-28f;

__device__ __forceinline__ float fma_(float a, float b, float c) {
  return __builtin_fmaf(a, b, c);
}

// Revolutions of the fp32 angle x (radians), reduced to [-0.5, 0.5] plus a
// tail: x/(2*pi) - k with |error| <~ 3e-8 revolutions for |x| < 2^20.
// The head product's rounding error is recovered exactly with an FMA
// (Dekker), so no precision is lost to the ~3e3-radian phases of IDG
// (|phase| = |phase_offset| + |phase_index * k| reaches ~525 revolutions,
// where a plain x * (1/2pi) would be off by ~3e-5 revolutions).
__device__ __forceinline__ float revolutions(float x) {
  const float hi = x * kInv2PiHi;
  float lo = fma_(x, kInv2PiHi, -hi);
  lo = fma_(x, kInv2PiLo, lo);
  return (hi - __builtin_rintf(hi)) + lo;
}

// kPhaseTail = 1 - 2*pi*kInv2PiHi: the MFMA kernels reduce a phase x to
// revolutions as r = fma(x, kInv2PiHi, -m), m an integer (the product is
// exact inside the FMA, |r| < 1, one rounding), which is x/(2*pi) - m minus
// x * kPhaseTail/(2*pi).  Splitting x = phase_offset - k * phase_index (the
// degridder's phase is the negative), the phase_offset part of that tail is
// a constant per pixel and is restored exactly as one phasor
// exp(i * phase_offset * kPhaseTail) per pixel (phase_tail below, applied
// after the gridder's sum or to the degridder's pixels).  The k *
// phase_index part (<= 1.5e-6 rad at C = 256) is added to r in revolutions,
// evaluated at the first channel k_b of the r's 16-channel block
// (tail_k_rev: one packed multiply per block, one packed add per two
// phasors); what remains, (k - k_b) * phase_index * kPhaseTail, is below
// 1e-7 rad.  Left out (round 2), it put the gridder as far from exact
// accumulation as the reference's own f32 sum at C = 256 (1.3e-5 in the
// reference metric, tests/test_gpu_accuracy.py).
constexpr float kPhaseTail = 0x1.5a892p-25f;  // 4.034206e-8

// c = k_b * (-phase_index) * (1/2pi - kInv2PiHi) in revolutions for a
// packed pair of -phase_index (the gridder's sign; the degridder passes
// +phase_index for its phase = k * phase_index - phase_offset).
#ifndef IDG_TAIL_K
#define IDG_TAIL_K 1
#endif
__device__ __forceinline__ floatx2 tail_k_rev(floatx2 neg_pidx, float kb) {
  const float f = IDG_TAIL_K ? kb * kInv2PiLo : 0.0f;
  return neg_pidx * floatx2{f, f};
}

// Precision options of the MFMA kernels (template PREC, chosen per launch by
// util.cpp precision_for): kPrecTail adds tail_k_rev to every phasor's
// revolutions; kPrecTailAlt (gridder) adds 4 x tail_k_rev to the first
// channel of every channel quad and nothing to the other three -- the same
// correction summed over each quad, for a quarter of the adds: the gridder
// sums over channels, so the +3c / -c pattern cancels in every coherent sum
// to first order (tests/emul/tail_mean_emul.py); kPrecFlush
// (gridder, S = 32) sums the accumulator tiles into an f32 master every
// kFlushFills fills (at most 32 K-steps each).
constexpr int kPrecTail = 1, kPrecFlush = 2, kPrecTailAlt = 4;
// Every 16 fills (round 5; 8 in round 4): C = 256 gridder 3.35e-6 from the
// exact sum against 2.74e-6 (the reference's own output: 1.27e-5), its
// counter traffic 7.90 -> 6.63 GB at NR_TIMESLOTS = 4 (1.49x -> 1.25x the
// algorithmic bytes); 32 fills (5.97 GB) put a configs[2] sample at 6.98e-6
// (profiles/r05/flush/).
#ifndef IDG_FLUSH_FILLS
#define IDG_FLUSH_FILLS 16
#endif
constexpr int kFlushFills = IDG_FLUSH_FILLS;

// exp(i * phase_offset * kPhaseTail), |angle| <= 1.4e-4: cos = 1 - a^2/2
// (the a^4 term is below 1e-16), sin = a (the a^3 term below 5e-13).
__device__ __forceinline__ void phase_tail(float phase_offset, float *c,
                                           float *s) {
  const float a = phase_offset * kPhaseTail;
  *c = fma_(-0.5f * a, a, 1.0f);
  *s = a;
}

// The value of lane (l + 8) mod 16 of the lane's 16-lane row (DPP
// row_ror:8).  Call it on a named scalar: applied to the elements of an
// ext_vector in a loop, this hipcc emitted one DPP move of element 0 for
// all of them (tools/probes/dpp_vector_probe.hip).
__device__ __forceinline__ float row_ror8(float x) {
  return __builtin_bit_cast(
      float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x128,
                                         0xF, 0xF, false));
}

// The 4 correlations (re, im interleaved) times the phasor (c, s).
__device__ __forceinline__ void rotate4(float (&v)[8], float c, float s) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float re = v[2 * q], im = v[2 * q + 1];
    v[2 * q] = fma_(re, c, -(im * s));
    v[2 * q + 1] = fma_(re, s, im * c);
  }
}

// sin / cos of 2*pi*r for r in revolutions.  v_sin_f32 / v_cos_f32 take
// their argument in revolutions and are exact enough once r is small
// (measured on MI355X: tools/probes); the range
// reduction is done by revolutions() / the anchored update in the kernels,
// never by the hardware's own [-256, 256] fold of a large, already-rounded
// argument (the trap of __sinf/__cosf).
__device__ __forceinline__ void sincos_rev(float r, float *s, float *c) {
#if IDG_SINCOS_POLY
  // Minimax-free fallback: quadrant split + Cody-Waite style polynomials.
  const float q = __builtin_rintf(4.0f * r);
  const float g = fma_(q, -0.25f, r);  // |g| <= 1/8 revolution, exact
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
#else
  *s = __builtin_amdgcn_sinf(r);
  *c = __builtin_amdgcn_cosf(r);
#endif
}

// Subgrid of workgroup `orig` among nwg: blocks are dealt round-robin over
// the 8 XCDs (blocks b and b + 8 share one L2), so the bijective remap below
// gives each XCD a contiguous run of subgrids (MI355X_MICROARCH.md, XCD
// placement; cdna_hip_programming.md T1).  Neighbouring subgrids share
// stations, so their A-term reads hit the same L2.  A speed choice only:
// any placement computes the same outputs.
__device__ __forceinline__ int xcd_subgrid(int orig, int nwg) {
#ifdef IDG_NO_XCD_REMAP
  return orig;
#else
  const int q = nwg / 8, r = nwg % 8, x = orig % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + orig / 8;
#endif
}

// The general-subgrid queue of the two-kernel launch (util.hpp
// KernelChoice::parts): the mirror kernel pushes the subgrids it leaves,
// the general kernel takes them from a shared counter.  8 shards, one per
// XCD (the pushing workgroup's blockIdx % 8, so at most ceil(NS / 8) pushes
// each), each a count on a 128-byte line of its own (a single count took
// 0.28 ms of serialized atomics for 24,500 pushes) and a list; then one take
// counter.  Layout in ints: counts at 32 x, take counter at kQueueNext,
// shard x's list at kQueueHead + x * queue_cap(ns); then the general
// kernel's exit counter at kQueueExit.  The counters (ints [0, kQueueExit])
// are zero before a launch pair: zeroed when the workspace is allocated, and
// zeroed again by the general kernel's last workgroup to finish
// (queue_retire), so a workspace cached per stream needs no clear per launch.
// (A persistent mirror kernel's take counter and exit count sit at
// kQueueMirror / kQueueMirrorExit, zeroed by its own last workgroup.)
constexpr int kQueueShards = 8, kQueueNext = 256, kQueueExit = 257,
              kQueueMirror = 264, kQueueMirrorExit = 272, kQueueHead = 288;

__host__ __device__ inline int queue_cap(int ns) {
  return (ns + kQueueShards - 1) / kQueueShards;
}
__host__ __device__ inline size_t queue_ints(int ns) {
  return kQueueHead + static_cast<size_t>(kQueueShards) * queue_cap(ns);
}

// One thread of the pushing workgroup; shard x (default: the workgroup's
// XCD, blockIdx % 8).  A shard takes at most queue_cap(ns) entries: a
// launch with several workgroups per subgrid pushes into shard s % 8.
__device__ __forceinline__ void queue_push(int *queue, int ns, int s,
                                           int shard = -1) {
  const int x = shard >= 0 ? shard : static_cast<int>(blockIdx.x) % kQueueShards;
  queue[kQueueHead + x * queue_cap(ns) + atomicAdd(queue + 32 * x, 1)] = s;
}

// The queue's entries in shard order: count() of them, at(i) the i-th.
struct QueueView {
  const int *q;
  int cap, pre[kQueueShards + 1];
  __device__ int count() const { return pre[kQueueShards]; }
  __device__ int at(int i) const {
    int x = 0;
#pragma unroll
    for (int k = 1; k < kQueueShards; ++k) x += i >= pre[k] ? 1 : 0;
    return q[kQueueHead + x * cap + (i - pre[x])];
  }
};

// Thread 0 of a general-kernel workgroup, after its last take: the last
// workgroup of the grid to get here (every other one has read the counts
// and made its last take) zeroes the counters for the next launch pair.
__device__ __forceinline__ void queue_retire(int *queue) {
  if (atomicAdd(queue + kQueueExit, 1) == static_cast<int>(gridDim.x) - 1) {
#pragma unroll
    for (int x = 0; x < kQueueShards; ++x) queue[32 * x] = 0;
    queue[kQueueNext] = 0;
    queue[kQueueExit] = 0;
  }
}

__device__ __forceinline__ QueueView queue_view(const int *queue, int ns) {
  QueueView v;
  v.q = queue;
  v.cap = queue_cap(ns);
  v.pre[0] = 0;
#pragma unroll
  for (int x = 0; x < kQueueShards; ++x)
    v.pre[x + 1] = v.pre[x] + __builtin_amdgcn_readfirstlane(queue[32 * x]);
  return v;
}

// Per-subgrid constants, evaluated exactly as the reference does
// (gridder_reference.cpp:15-39): offsets in double, rounded to float.
struct SubgridSetup {
  long long time_offset;
  int nr_timesteps, aterm_index, station1, station2;
  float u_offset, v_offset, w_offset;
};

__device__ __forceinline__ SubgridSetup
setup_subgrid(const idg::Metadata *__restrict__ metadata, int s,
              int grid_size, int subgrid_size, float image_size,
              float w_step_in_lambda) {
  const idg::Metadata m = metadata[s];
  const int bo0 = metadata[0].baseline_offset;
  SubgridSetup g;
  g.time_offset = static_cast<long long>(m.baseline_offset - bo0) +
                  m.time_offset;
  g.nr_timesteps = m.nr_timesteps;
  g.aterm_index = m.aterm_index;
  g.station1 = static_cast<int>(m.baseline.station1);
  g.station2 = static_cast<int>(m.baseline.station2);
  const double scale = 2.0 * 3.14159265358979323846 /
                       static_cast<double>(image_size);
  g.u_offset = static_cast<float>(
      static_cast<double>(m.coordinate.x + subgrid_size / 2 - grid_size / 2) *
      scale);
  g.v_offset = static_cast<float>(
      static_cast<double>(m.coordinate.y + subgrid_size / 2 - grid_size / 2) *
      scale);
  const float w_lambda = static_cast<float>(
      static_cast<double>(w_step_in_lambda) *
      (static_cast<double>(m.coordinate.z) + 0.5));
  g.w_offset = static_cast<float>(2.0 * 3.14159265358979323846 *
                                  static_cast<double>(w_lambda));
  return g;
}

// Pointer to the 2x2 A-term of (slot, station, y, x).
__device__ __forceinline__ const float4 *aterm_ptr(const float2 *aterms,
                                                   int nr_stations, int S,
                                                   int slot, int station,
                                                   int y, int x) {
  const size_t idx =
      ((static_cast<size_t>(slot) * nr_stations + station) * S + y) * S + x;
  return reinterpret_cast<const float4 *>(aterms + idx * 4);
}

__device__ __forceinline__ void load_jones(const float4 *p, idg::cfloat *j) {
  const float4 a = p[0], b = p[1];
  j[0] = {a.x, a.y};
  j[1] = {a.z, a.w};
  j[2] = {b.x, b.y};
  j[3] = {b.z, b.w};
}

}  // namespace idg_mi355x

// Debug builds only (-DIDG_WG_TIMELINE=1, tools/debug/wg_timeline.py): per
// workgroup wall-clock start / end (s_memrealtime, 100 MHz), HW_ID and
// XCC_ID of the combined kernels, written by thread 0 with vector stores.
#if defined(IDG_WG_TIMELINE) && IDG_WG_TIMELINE
constexpr int kTimelineMax = 32768;
struct WgStamp {
  unsigned long long t0, t1;
  unsigned hw_id, xcc_id;
};
__device__ __forceinline__ void timeline_start(WgStamp *tl) {
  if (threadIdx.x == 0 && blockIdx.x < kTimelineMax) {
    WgStamp w;
    w.t0 = static_cast<unsigned long long>(wall_clock64());
    w.t1 = 0;
    w.hw_id = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    w.xcc_id = __builtin_amdgcn_s_getreg((31 << 11) | 20);
    tl[blockIdx.x] = w;
  }
}
__device__ __forceinline__ void timeline_end(WgStamp *tl) {
  __syncthreads();
  if (threadIdx.x == 0 && blockIdx.x < kTimelineMax)
    tl[blockIdx.x].t1 = static_cast<unsigned long long>(wall_clock64());
}
#endif
