// pipeline_mi355x.hip.cpp -- the IDG steps either side of the gridder and
// degridder: batched subgrid FFT, adder
// (subgrids -> uv grid) and splitter (uv grid -> subgrids).
//
// None of these is in the reference (its `Grid` type, types.hpp:358-370, is
// never used), so their conventions are pinned by the path they complete
// (tests/test_pipeline*.py):
//
//   gridding:   gridder -> FFT(sign +1, scale 1) -> adder
//   degridding: splitter -> FFT(sign -1, scale 1/S^2) -> degridder
//
// with, for subgrid pixel (y, x) at grid cell (coordinate.y + y,
// coordinate.x + x) and FFT index ((y + S/2) % S, (x + S/2) % S),
//   adder:    grid  += exp(+i pi ((x + y)(S + 1)/S - 1)) * F
//   splitter: F      = exp(-i pi ((x + y)(S + 1)/S - 1)) * grid
// so that one unit visibility whose uv lies exactly on a grid cell grids to
// S^2 at that cell, and a unit grid cell degrids to 1 for a visibility at it
// (checked against the C oracle's gridder/degridder).
//
// The grid is [nr_w_layers][4][G][G] complex64; a subgrid goes to layer
// coordinate.z (w-stacking).  A subgrid that does not lie wholly inside the
// grid is skipped by the adder and zero-filled by the splitter.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>

#include "../util.hpp"
#include "common/types.hpp"
#include "device.hpp"
#include "fft.hpp"  // unit_phasor, cmulf, fft_dif_registers, bit_reverse

namespace idg_mi355x {

namespace {

// Adder/splitter phasor of subgrid pixel (y, x): exp(i sgn pi ((x + y)(S + 1)
// / S - 1)) = exp(2 pi i sgn ((x + y)(S + 1) - S) / (2 S)).
__device__ __forceinline__ float2 shift_phasor(int x, int y, int S, float sgn) {
  return unit_phasor((x + y) * (S + 1) - S, 2 * S, sgn);
}

// (v + S/2) % S for 0 <= v < S, without an integer division (S is a
// runtime value): the fftshift index of subgrid row/column v.
__device__ __forceinline__ int half_shift(int v, int S) {
  const int w = v + S / 2;
  return w >= S ? w - S : w;
}

// Stores of the FFT and splitter outputs (0.8 GB at configs[1], consumed by
// a later kernel): non-temporal, so they do not sit dirty in L2 / MALL and
// the next kernel does not pay for their write-back (measured: splitter
// 0.266 -> 0.256 ms and the inverse FFT after it 0.306 -> 0.270 ms).
#ifndef IDG_PIPE_NT
#define IDG_PIPE_NT 1
#endif
__device__ __forceinline__ void store_stream(float2 *p, float2 v) {
#if IDG_PIPE_NT
  typedef float f2 __attribute__((ext_vector_type(2)));
  __builtin_nontemporal_store(f2{v.x, v.y}, reinterpret_cast<f2 *>(p));
#else
  *p = v;
#endif
}
__device__ __forceinline__ void store_stream(float4 *p, float4 v) {
#if IDG_PIPE_NT
  typedef float f4 __attribute__((ext_vector_type(4)));
  __builtin_nontemporal_store(f4{v.x, v.y, v.z, v.w},
                              reinterpret_cast<f4 *>(p));
#else
  *p = v;
#endif
}

__device__ __forceinline__ bool fits(const idg::Metadata &m, int G, int S,
                                     int nr_w_layers) {
  return m.coordinate.x >= 0 && m.coordinate.x + S <= G &&
         m.coordinate.y >= 0 && m.coordinate.y + S <= G &&
         m.coordinate.z >= 0 && m.coordinate.z < nr_w_layers;
}

}  // namespace

// 2-D DFT of one S x S correlation plane per workgroup, in place:
//   out[k][l] = scale * sum_{y,x} in[y][x] exp(sign 2 pi i (k y + l x) / S)
// as a row pass then a column pass through LDS, twiddles from a per-plane
// table (exact integer argument reduction).  Unnormalised for scale = 1
// (numpy: sign -1 -> fft2, sign +1 -> ifft2 * S^2).  Dynamic LDS:
// (2 S^2 + S) float2.
__global__ void __launch_bounds__(256)
    kernel_subgrid_dft(float2 *__restrict__ planes, int S, float sign,
                       float scale) {
  extern __shared__ float2 dft_lds[];
  float2 *a = dft_lds;
  float2 *b = a + S * S;
  float2 *tw = b + S * S;
  float2 *plane = planes + static_cast<size_t>(blockIdx.x) * S * S;
  const int tid = threadIdx.x;
  const int npix = S * S;
  for (int i = tid; i < S; i += blockDim.x) tw[i] = unit_phasor(i, S, sign);
  for (int i = tid; i < npix; i += blockDim.x) a[i] = plane[i];
  __syncthreads();
  // rows: b[y][l] = sum_x a[y][x] tw[(x l) mod S]
  for (int i = tid; i < npix; i += blockDim.x) {
    const int y = i / S, l = i - y * S;
    float re = 0.0f, im = 0.0f;
    int idx = 0;
    for (int x = 0; x < S; ++x) {
      const float2 v = a[y * S + x], w = tw[idx];
      re = fma_(v.x, w.x, fma_(-v.y, w.y, re));
      im = fma_(v.x, w.y, fma_(v.y, w.x, im));
      idx += l;
      if (idx >= S) idx -= S;
    }
    b[i] = make_float2(re, im);
  }
  __syncthreads();
  // columns: out[k][l] = scale * sum_y b[y][l] tw[(y k) mod S]
  for (int i = tid; i < npix; i += blockDim.x) {
    const int k = i / S, l = i - k * S;
    float re = 0.0f, im = 0.0f;
    int idx = 0;
    for (int y = 0; y < S; ++y) {
      const float2 v = b[y * S + l], w = tw[idx];
      re = fma_(v.x, w.x, fma_(-v.y, w.y, re));
      im = fma_(v.x, w.y, fma_(v.y, w.x, im));
      idx += k;
      if (idx >= S) idx -= S;
    }
    plane[i] = make_float2(re * scale, im * scale);
  }
}

// The home sort: subgrids counting-sorted by their home tile, the grid tile
// (TW x TH, w-layer major, then tile rows) holding their corner, with the
// subgrids not wholly inside the grid last.  offset[key] is the first
// position of key's subgrids in order[] (entries {s, x, y, z}, z = -1 when
// not wholly inside the grid), offset[nkeys] = nr_subgrids.  Both
// the adder and the splitter read it:
//  * the adder's tile finds the subgrids overlapping it in the home tiles up
//    to ceil((S - 1) / TW) tiles left and ceil((S - 1) / TH) tiles up of
//    itself: one contiguous range of order[] per tile row;
//  * the splitter processes subgrids in this order, so consecutive
//    workgroups of one XCD (xcd_subgrid) read overlapping grid windows,
//    which stay in that XCD's L2, instead of every subgrid pulling its
//    32 KB window from the Infinity Cache.
// The order within a home tile is that of the atomics; neither output
// depends on it (the adder sorts its list by subgrid index, the splitter
// writes every subgrid from its own workgroup).
#ifndef IDG_ADD_TW
#define IDG_ADD_TW 16
#endif
#ifndef IDG_ADD_TH
#define IDG_ADD_TH 16
#endif
#ifndef IDG_ADD_U
#define IDG_ADD_U 4
#endif
#ifndef IDG_ADD_MASKED
#define IDG_ADD_MASKED 1
#endif
constexpr int kTW = IDG_ADD_TW;  // grid tile width (pixels)
constexpr int kTH = IDG_ADD_TH;  // grid tile height
constexpr int kAddPix = kTW * kTH / 256;  // tile pixels per thread
constexpr int kAddMaxTable = 256;  // shift phasors kept in LDS for S <= 128
constexpr int kAddListCap = 1536;  // candidate entries sorted in LDS
constexpr int kAddMaxRows = 64;    // home-tile rows a tile gathers from
constexpr int kSortLdsKeys = 19 * 1024;  // LDS: 2 x 76 KB (place kernel)
constexpr int kSortMaxChunks = 16;       // workgroups of the LDS sort
static_assert(kTW * kTH == 256 * kAddPix && (kTW & (kTW - 1)) == 0,
              "tile = block x pixels, power-of-two width");

struct TileGrid {
  int ntx, nty;
  __host__ __device__ TileGrid(int G)
      : ntx(G > 0 ? (G + kTW - 1) / kTW : 0),
        nty(G > 0 ? (G + kTH - 1) / kTH : 0) {}
  __host__ __device__ int nkeys(int nr_w_layers) const {
    return nr_w_layers * nty * ntx + 1;
  }
};

__device__ __forceinline__ int home_key(const idg::Metadata &m, int G, int S,
                                        int nr_w_layers, const TileGrid &tg) {
  return fits(m, G, S, nr_w_layers)
             ? (m.coordinate.z * tg.nty + m.coordinate.y / kTH) * tg.ntx +
                   m.coordinate.x / kTW
             : nr_w_layers * tg.nty * tg.ntx;
}

// Exclusive scan of the n values v[0, n) held by one workgroup of 1,024:
// each thread takes `per` consecutive values, the waves scan their thread
// totals by shuffles, the 16 wave totals go through LDS.  Returns this
// thread's exclusive prefix; the caller walks its `per` values from it.
__device__ __forceinline__ int block_scan_1024(int t, int *wave_sum) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int incl = t;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int o = __shfl_up(incl, d);
    if (lane >= d) incl += o;
  }
  if (lane == 63) wave_sum[wave] = incl;
  __syncthreads();
  int before = incl - t;
#pragma unroll
  for (int w = 0; w < 16; ++w) before += w < wave ? wave_sum[w] : 0;
  return before;
}

// The home sort in two launches of nwg workgroups of 1,024, each workgroup
// owning a contiguous chunk of subgrids, with its counters in LDS (no
// device-scope atomics, which cross the XCDs: a counting pass of 24,500 of
// them took 19 us; one workgroup sorting everything took 47 us):
//  count: key, rank within the chunk's home tile and corner -> slot[s], the
//         chunk's histogram -> hist[key][w];
//  place: every workgroup scans the nwg histograms itself (its own base per
//         key: the keys before it, then the earlier chunks of the same key),
//         then scatters its chunk as entries {s, x, y, z} (z = -1: not
//         wholly inside the grid), so the adder and splitter read a
//         subgrid's corner with its index, not through its metadata;
//         workgroup 0 writes offset[].
// nkeys <= kSortLdsKeys, nwg <= kSortMaxChunks.
__global__ void __launch_bounds__(1024)
    kernel_home_count(const idg::Metadata *__restrict__ metadata,
                      int nr_subgrids, int G, int S, int nr_w_layers,
                      int chunk, int *__restrict__ hist,
                      int4 *__restrict__ slot) {
  extern __shared__ int lhist[];
  const int tid = threadIdx.x;
  const TileGrid tg(G);
  const int nkeys = tg.nkeys(nr_w_layers);
  for (int i = tid; i < nkeys; i += 1024) lhist[i] = 0;
  __syncthreads();
  const int s0 = blockIdx.x * chunk;
  const int s1 = min(nr_subgrids, s0 + chunk);
  // U subgrids per step, every metadata load issued before the first atomic
  constexpr int U = 4;
  for (int b = s0; b < s1; b += 1024 * U) {
    int key[U], cx[U], cy[U];
#pragma unroll
    for (int h = 0; h < U; ++h) {
      const int s = b + 1024 * h + tid;
      key[h] = -1;
      if (s < s1) {
        const idg::Metadata m = metadata[s];
        key[h] = home_key(m, G, S, nr_w_layers, tg);
        cx[h] = m.coordinate.x;
        cy[h] = m.coordinate.y;
      }
    }
#pragma unroll
    for (int h = 0; h < U; ++h)
      if (key[h] >= 0)
        slot[b + 1024 * h + tid] =
            make_int4(key[h], atomicAdd(&lhist[key[h]], 1), cx[h], cy[h]);
  }
  __syncthreads();
  // key-major rows of kSortMaxChunks counts: the place kernel reads a key's
  // row as four 16-byte loads
  for (int i = tid; i < nkeys; i += 1024)
    hist[static_cast<size_t>(i) * kSortMaxChunks + blockIdx.x] = lhist[i];
}

__global__ void __launch_bounds__(1024)
    kernel_home_place(const int *__restrict__ hist, int nwg, int nkeys,
                      int keys_per_layer, int nr_subgrids, int chunk,
                      const int4 *__restrict__ slot,
                      int *__restrict__ offset, int4 *__restrict__ order) {
  extern __shared__ int base[];  // [nkeys] bases, then [nkeys] earlier parts
  int *pre = base + nkeys;
  __shared__ int wave_sum[16];
  const int tid = threadIdx.x, w = blockIdx.x;
  static_assert(kSortMaxChunks == 16, "a key's row is four int4");
  // per key: the total over the chunks and the part in earlier chunks
#pragma unroll 4
  for (int k = tid; k < nkeys; k += 1024) {
    const int4 *row =
        reinterpret_cast<const int4 *>(hist + static_cast<size_t>(k) * 16);
    int tot = 0, p = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int4 v = row[q];
      const int vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int c = 4 * q + u;
        const int x = c < nwg ? vv[u] : 0;
        tot += x;
        p += c < w ? x : 0;
      }
    }
    base[k] = tot;
    pre[k] = p;
  }
  __syncthreads();
  // scan of the totals over the keys (a thread takes `per` consecutive)
  const int per = (nkeys + 1023) / 1024;
  int t = 0;
  for (int j = 0; j < per; ++j) {
    const int k = tid * per + j;
    t += k < nkeys ? base[k] : 0;
  }
  int e = block_scan_1024(t, wave_sum);
  for (int j = 0; j < per; ++j) {
    const int k = tid * per + j;
    if (k < nkeys) {
      const int tot = base[k];
      if (w == 0) offset[k] = e;
      base[k] = e + pre[k];
      e += tot;
    }
  }
  if (w == 0 && tid == 0) offset[nkeys] = nr_subgrids;
  __syncthreads();
  const int s0 = w * chunk, s1 = min(nr_subgrids, s0 + chunk);
  for (int b = s0; b < s1; b += 1024 * 4) {
    int4 k[4];
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const int s = b + 1024 * h + tid;
      k[h] = s < s1 ? slot[s] : make_int4(-1, 0, 0, 0);
    }
#pragma unroll
    for (int h = 0; h < 4; ++h)
      if (k[h].x >= 0)
        order[base[k[h].x] + k[h].y] = make_int4(
            b + 1024 * h + tid, k[h].z, k[h].w,
            k[h].x < nkeys - 1 ? k[h].x / keys_per_layer : -1);
  }
}

// The same sort for more keys than LDS holds: count (pass 0) or scatter
// (pass 1) with device-scope atomics, one thread per subgrid ...
__global__ void __launch_bounds__(256)
    kernel_home_key(const idg::Metadata *__restrict__ metadata,
                    int nr_subgrids, int G, int S, int nr_w_layers, int pass,
                    int *__restrict__ count, int *__restrict__ cursor,
                    int4 *__restrict__ order) {
  const int s = blockIdx.x * 256 + threadIdx.x;
  if (s >= nr_subgrids) return;
  const idg::Metadata m = metadata[s];
  const int key = home_key(m, G, S, nr_w_layers, TileGrid(G));
  if (pass == 0)
    atomicAdd(count + key, 1);
  else
    order[atomicAdd(cursor + key, 1)] =
        make_int4(s, m.coordinate.x, m.coordinate.y,
                  fits(m, G, S, nr_w_layers) ? m.coordinate.z : -1);
}

// ... and the exclusive scan between the passes (one workgroup of 1,024, in
// chunks of 4,096 counts): offset = cursor = the running sum, offset[n] =
// the total.
__global__ void __launch_bounds__(1024)
    kernel_home_scan(const int *__restrict__ count, int n,
                     int *__restrict__ offset, int *__restrict__ cursor) {
  __shared__ int wave_sum[16];
  const int tid = threadIdx.x;
  int running = 0;
  for (int base = 0; base < n; base += 4096) {
    int v[4], t = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = base + 4 * tid + j;
      v[j] = i < n ? count[i] : 0;
      t += v[j];
    }
    int e = running + block_scan_1024(t, wave_sum);
    int total = 0;
#pragma unroll
    for (int w = 0; w < 16; ++w) total += wave_sum[w];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = base + 4 * tid + j;
      if (i < n) {
        offset[i] = e;
        cursor[i] = e;
      }
      e += v[j];
    }
    running += total;
    __syncthreads();  // wave_sum is rewritten by the next chunk
  }
  if (tid == 0) offset[n] = running;
}

// grid[z][pol][cy + y][cx + x] += shift_phasor(x, y) * F[s][pol][ys][xs],
// ys = (y + S/2) % S, xs = (x + S/2) % S.
//
// A gather, not a scatter: one workgroup owns one TW x TH tile of one
// w-layer, adds the pixels of the subgrids overlapping it into registers in
// ascending subgrid order and read-modify-writes the tile once.  Every
// subgrid pixel is read exactly once over the whole launch, there are no
// atomics on the grid, and the summation order -- hence every bit of the
// grid -- is deterministic.  The overlapping subgrids are gathered from the
// home sort's ranges and sorted in LDS; a candidate list larger than the
// LDS list falls back to an ordered scan of all the metadata, which yields
// the same order.
//
// Crowded tiles (round 4): one workgroup per tile serialises a crowded uv
// centre onto a few CUs (24,500 subgrids around the centre: 0.2 -> 6.6 ms,
// DESIGN.md §11).  A tile whose candidate rows hold more than kAddSegLen
// subgrids (an upper bound of its list, from the home sort's offsets
// alone) is summed in segments of kAddSegLen list entries instead, in
// three launches that need no cross-workgroup waits or fences (each kernel
// boundary orders the next one's reads):
//   kernel_adder_crowd   one thread per tile: the crowded tiles, their
//                        segment count and partial slots;
//   kernel_adder         the segment workgroups first in the grid (so they
//                        start at once), each segment into its own partial
//                        tile; then one workgroup per uncrowded tile, as
//                        before and bit for bit;
//   kernel_adder_combine each crowded tile's partials added to the grid in
//                        segment order.
// Deterministic: a segment's sum and the order of the partials depend on
// the data only.
constexpr int kAddSegLen = 256;   // list entries per segment
constexpr int kAddWorkers = 256;  // segment workgroups
constexpr int kAddCombiners = 64;
// counters, each on its own 128-byte line; zero between launches (the
// combine kernel's last workgroup clears them)
constexpr int kSegHeavy = 0, kSegTotal = 32, kSegExit = 64, kSegHdrInts = 96;
constexpr size_t kAddPartialFloat2 = static_cast<size_t>(kAddPix) * 4 * 256;

// The segment workspace (util.hpp WorkspaceLease, cached per stream):
// counters | partial [slot][pixel j][pol][thread] | heavy {tile, z, nseg,
// base} | owner (crowded tile of each partial slot) | tile_seg (per tile:
// its crowded index, or -1).  Sized for the worst case of the batch: a
// subgrid is a candidate of at most tps tiles, so the bounds sum to at most
// T = nr_subgrids * tps, at most T / kAddSegLen tiles are crowded, and
// their segments number at most 2 T / kAddSegLen + 1.
struct AdderSeg {
  int *hdr = nullptr;
  float2 *partial = nullptr;
  int4 *heavy = nullptr;
  int *owner = nullptr;
  int *tile_seg = nullptr;
  int heavy_cap = 0, slot_cap = 0;
};

struct AdderSegCaps {
  int heavy, slots;
  size_t bytes;
};
inline AdderSegCaps adder_seg_caps(int nr_subgrids, int S, int ntiles_all) {
  const long long cols_x = (S - 1 + kTW - 1) / kTW + 1;
  const long long cols_y = (S - 1 + kTH - 1) / kTH + 1;
  const long long entries =
      static_cast<long long>(nr_subgrids) * cols_x * cols_y;
  const long long per = (entries + kAddSegLen - 1) / kAddSegLen;
  AdderSegCaps c;
  c.heavy = static_cast<int>(std::min<long long>(ntiles_all, per + 1));
  c.slots = static_cast<int>(2 * per + 1);
  c.bytes = kSegHdrInts * sizeof(int) +
            static_cast<size_t>(c.slots) *
                (kAddPartialFloat2 * sizeof(float2) + sizeof(int)) +
            static_cast<size_t>(c.heavy) * sizeof(int4) +
            static_cast<size_t>(ntiles_all) * sizeof(int);
  return c;
}

__global__ void __launch_bounds__(256)
    kernel_adder_crowd(const int *__restrict__ offset, int G, int S,
                       int nr_w_layers, AdderSeg sw) {
  const TileGrid tg(G);
  const int ntiles = tg.ntx * tg.nty;
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= ntiles * nr_w_layers) return;
  const int z = t / ntiles, tl = t - z * ntiles;
  const int tx = tl % tg.ntx, ty = tl / tg.ntx;
  const int DX = (S - 1 + kTW - 1) / kTW, DY = (S - 1 + kTH - 1) / kTH;
  const int nrows = min(DY, ty) + 1;
  const int hx0 = max(0, tx - DX);
  int bound = 0;
  if (nrows <= kAddMaxRows)
    for (int r = 0; r < nrows; ++r) {
      const int k0 = (z * tg.nty + ty - r) * tg.ntx;
      bound += offset[k0 + tx + 1] - offset[k0 + hx0];
    }
  int h = -1;
  if (bound > kAddSegLen) {
    const int ns = (bound + kAddSegLen - 1) / kAddSegLen;
    h = atomicAdd(sw.hdr + kSegHeavy, 1);
    const int b = atomicAdd(sw.hdr + kSegTotal, ns);
    const bool ok = h < sw.heavy_cap && b + ns <= sw.slot_cap;  // (sized: always)
    if (ok) sw.heavy[h] = make_int4(tl, z, ns, b);
    // every slot below the total gets an owner (-1: skipped by the segment
    // workgroups; the tile then takes the one-workgroup path)
    for (int s = 0; s < ns && b + s < sw.slot_cap; ++s)
      sw.owner[b + s] = ok ? h : -1;
    if (!ok) h = -1;
  }
  sw.tile_seg[t] = h;
}

// Each crowded tile's partials, in segment order, onto the grid; the last
// workgroup to finish clears the counters for the next launch.
__global__ void __launch_bounds__(256)
    kernel_adder_combine(float2 *__restrict__ grid, int G, AdderSeg sw) {
  const int tid = threadIdx.x;
  const TileGrid tg(G);
  const int nh = min(sw.hdr[kSegHeavy], sw.heavy_cap);
  for (int h = blockIdx.x; h < nh; h += gridDim.x) {
    const int4 he = sw.heavy[h];  // {tile, z, nseg, base}
    const int tx0 = (he.x % tg.ntx) * kTW, ty0 = (he.x / tg.ntx) * kTH;
    float2 *gz = grid + static_cast<size_t>(he.y) * 4 * G * G;
    const float2 *p0 =
        sw.partial + static_cast<size_t>(he.w) * kAddPartialFloat2;
#pragma unroll
    for (int j = 0; j < kAddPix; ++j) {
      const int i = tid + 256 * j;
      const int gx = tx0 + (i & (kTW - 1)), gy = ty0 + i / kTW;
      if (gx >= G || gy >= G) continue;
#pragma unroll
      for (int pol = 0; pol < 4; ++pol) {
        const int k = (j * 4 + pol) * 256 + tid;
        float2 sum = p0[k];
        for (int q = 1; q < he.z; ++q) {
          const float2 v = p0[static_cast<size_t>(q) * kAddPartialFloat2 + k];
          sum.x += v.x;
          sum.y += v.y;
        }
        float2 *o = gz + static_cast<size_t>(pol) * G * G +
                    static_cast<size_t>(gy) * G + gx;
        const float2 v = *o;
        *o = make_float2(v.x + sum.x, v.y + sum.y);
      }
    }
  }
  __syncthreads();
  if (tid == 0 && atomicAdd(sw.hdr + kSegExit, 1) ==
                      static_cast<int>(gridDim.x) - 1) {
    sw.hdr[kSegHeavy] = 0;
    sw.hdr[kSegTotal] = 0;
    sw.hdr[kSegExit] = 0;
  }
}

__global__ void __launch_bounds__(256)
    kernel_adder(const idg::Metadata *__restrict__ metadata, int nr_subgrids,
                 const int *__restrict__ offset, const int4 *__restrict__ order,
                 const float2 *__restrict__ subgrids,
                 float2 *__restrict__ grid, int G, int S, int nr_w_layers,
                 AdderSeg sw, int nworkers) {
  // the list (subgrid ids ascending, their corners relative to the tile
  // packed as (y - ty0 + S) << 16 | (x - tx0 + S), both in (0, S + T)) and
  // the candidates staged for it
  __shared__ int keys[kAddListCap], corner[kAddListCap];
  __shared__ int cand_key[kAddListCap], cand_corner[kAddListCap];
  __shared__ int row_begin[kAddMaxRows], row_pre[kAddMaxRows + 1];
  __shared__ int wave_count[4];
  __shared__ float2 table[kAddMaxTable];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const TileGrid tg(G);
  const int ntiles = tg.ntx * tg.nty;
  const int npix = S * S;
  const bool tabled = 2 * S - 1 <= kAddMaxTable;
  // shift phasor depends on x + y only
  if (tabled)
    for (int k = tid; k < 2 * S - 1; k += 256)
      table[k] = unit_phasor(k * (S + 1) - S, 2 * S, 1.0f);

  // Tile tl of layer z: the whole list onto the grid (seg < 0), or list
  // entries [seg kAddSegLen, (seg + 1) kAddSegLen) into partial slot `slot`.
  auto add_tile = [&](int tl, int z, int seg, int slot) {
    const int tx = tl % tg.ntx, ty = tl / tg.ntx;
    const int tx0 = tx * kTW, ty0 = ty * kTH;

    // candidates: home tiles (tx - dx, ty - dy), dx <= DX, dy <= DY, one
    // contiguous range of order[] per home-tile row
    const int DX = (S - 1 + kTW - 1) / kTW, DY = (S - 1 + kTH - 1) / kTH;
    const int nrows = min(DY, ty) + 1;
    const int hx0 = max(0, tx - DX);
    __syncthreads();  // the previous tile's LDS is consumed
    if (wave == 0 && nrows <= kAddMaxRows) {
      int len = 0;
      if (lane < nrows) {
        const int k0 = (z * tg.nty + ty - lane) * tg.ntx;
        const int b = offset[k0 + hx0];
        len = offset[k0 + tx + 1] - b;
        row_begin[lane] = b;
      }
      int incl = len;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int o = __shfl_up(incl, d);
        if (lane >= d) incl += o;
      }
      if (lane < nrows) row_pre[lane + 1] = incl;
      if (lane == 0) row_pre[0] = 0;
    }

    float2 acc[kAddPix][4];
#pragma unroll
    for (int j = 0; j < kAddPix; ++j)
#pragma unroll
      for (int pol = 0; pol < 4; ++pol) acc[j][pol] = make_float2(0.0f, 0.0f);

    // add the entries [e0, e1) of the LDS list, in list order; U entries
    // per step with every load issued before the first add (lanes outside
    // an entry's subgrid load its pixel 0 and drop it)
    constexpr int U = IDG_ADD_U;
    auto add_list = [&](int e0, int e1) {
      for (int e = e0; e < e1; e += U) {
        float2 v[U][kAddPix][4];
        float2 ph[U][kAddPix];
        bool ok[U][kAddPix];
#pragma unroll
        for (int hh = 0; hh < U; ++hh) {
          const int ee = min(e + hh, e1 - 1);
          const int2 c = make_int2(tx0 - S + (corner[ee] & 0xffff),
                                   ty0 - S + (corner[ee] >> 16));
          const float2 *sg =
              subgrids + static_cast<size_t>(keys[ee]) * 4 * npix;
#pragma unroll
          for (int j = 0; j < kAddPix; ++j) {
            const int i = tid + 256 * j;
            const int x = tx0 + (i & (kTW - 1)) - c.x;
            const int y = ty0 + i / kTW - c.y;
            ok[hh][j] = e + hh < e1 && x >= 0 && x < S && y >= 0 && y < S;
            const int src =
                ok[hh][j] ? half_shift(y, S) * S + half_shift(x, S) : 0;
            ph[hh][j] = !ok[hh][j] ? make_float2(0.0f, 0.0f)
                        : tabled   ? table[x + y]
                                   : shift_phasor(x, y, S, 1.0f);
#if IDG_ADD_MASKED
            // lanes outside the entry's subgrid issue no load (a wave with
            // none inside skips the entry's loads)
            if (ok[hh][j]) {
#pragma unroll
              for (int pol = 0; pol < 4; ++pol)
                v[hh][j][pol] = sg[pol * npix + src];
            } else {
#pragma unroll
              for (int pol = 0; pol < 4; ++pol)
                v[hh][j][pol] = make_float2(0.f, 0.f);
            }
#else
#pragma unroll
            for (int pol = 0; pol < 4; ++pol)
              v[hh][j][pol] = sg[pol * npix + src];
#endif
          }
        }
#pragma unroll
        for (int hh = 0; hh < U; ++hh)
#pragma unroll
          for (int j = 0; j < kAddPix; ++j) {
            if (!ok[hh][j]) continue;
#pragma unroll
            for (int pol = 0; pol < 4; ++pol) {
              const float2 w = cmulf(ph[hh][j], v[hh][j][pol]);
              acc[j][pol].x += w.x;
              acc[j][pol].y += w.y;
            }
          }
      }
    };
    auto pack_corner = [&](int cx, int cy) {
      return (cy - ty0 + S) << 16 | (cx - tx0 + S);
    };
    auto overlaps = [&](int cx, int cy) {
      return cx < tx0 + kTW && cx + S > tx0 && cy < ty0 + kTH && cy + S > ty0;
    };

    __syncthreads();
    // Compact the candidates that overlap the tile into the staging list
    // (in any order: LDS atomic slots), so the list's cap bounds the
    // overlapping subgrids, not every subgrid homed in the candidate rows;
    // then sort them ascending by rank (subgrid indices are distinct: each
    // entry's rank = the entries below it).  More overlaps than the cap
    // take the ordered scan below.  The count is exact either way.
    if (tid == 0) wave_count[0] = 0;
    __syncthreads();
    if (nrows <= kAddMaxRows) {
      const int n = row_pre[nrows];
      for (int i = tid; i < n; i += 256) {
        int r = 0;
        while (row_pre[r + 1] <= i) ++r;
        const int4 e = order[row_begin[r] + i - row_pre[r]];  // {s, x, y, z}
        if (!overlaps(e.y, e.z)) continue;
        const int slot = atomicAdd(&wave_count[0], 1);
        if (slot < kAddListCap) {
          cand_key[slot] = e.x;
          cand_corner[slot] = pack_corner(e.y, e.z);
        }
      }
    }
    __syncthreads();
    const int m = nrows <= kAddMaxRows ? wave_count[0] : kAddListCap + 1;

    const bool split = seg >= 0;
    const int lo = split ? seg * kAddSegLen : 0;
    const int hi = split ? lo + kAddSegLen : 0x7fffffff;

    if (m <= kAddListCap) {
      for (int i = tid; i < m; i += 256) {
        const int k = cand_key[i];
        int rank = 0;
        for (int j = 0; j < m; ++j) rank += cand_key[j] < k;
        keys[rank] = k;
        corner[rank] = cand_corner[i];
      }
      __syncthreads();
      add_list(lo, min(hi, m));
    } else {
      // ordered scan of all the metadata, 256 subgrids at a time, until
      // the range is covered
      int seen = 0;
      for (int mb = 0; mb < nr_subgrids && seen < hi; mb += 256) {
        const int s = mb + tid;
        bool hit = false;
        int cx = 0, cy = 0;
        if (s < nr_subgrids) {
          const idg::Metadata md = metadata[s];
          cx = md.coordinate.x;
          cy = md.coordinate.y;
          hit = fits(md, G, S, nr_w_layers) && md.coordinate.z == z &&
                overlaps(cx, cy);
        }
        const unsigned long long mask = __ballot(hit);
        __syncthreads();  // the previous chunk's list is consumed
        if (lane == 0) wave_count[wave] = __popcll(mask);
        __syncthreads();
        int pos = 0, total = 0;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          pos += w < wave ? wave_count[w] : 0;
          total += wave_count[w];
        }
        if (hit) {
          pos += __popcll(mask & ((1ull << lane) - 1ull));  // ordered
          keys[pos] = s;
          corner[pos] = pack_corner(cx, cy);
        }
        __syncthreads();
        const int a = max(lo - seen, 0), b = min(hi - seen, total);
        if (a < b) add_list(a, b);
        seen += total;
      }
    }

    float2 *gz = grid + static_cast<size_t>(z) * 4 * G * G;
    if (!split) {
#pragma unroll
      for (int j = 0; j < kAddPix; ++j) {
        const int i = tid + 256 * j;
        const int gx = tx0 + (i & (kTW - 1)), gy = ty0 + i / kTW;
        if (gx >= G || gy >= G) continue;
#pragma unroll
        for (int pol = 0; pol < 4; ++pol) {
          float2 *o = gz + static_cast<size_t>(pol) * G * G +
                      static_cast<size_t>(gy) * G + gx;
          const float2 v = *o;
          *o = make_float2(v.x + acc[j][pol].x, v.y + acc[j][pol].y);
        }
      }
      return;
    }
    // a segment: its partial tile (kernel_adder_combine adds the partials)
    float2 *pp = sw.partial + static_cast<size_t>(slot) * kAddPartialFloat2;
#pragma unroll
    for (int j = 0; j < kAddPix; ++j)
#pragma unroll
      for (int pol = 0; pol < 4; ++pol)
        pp[(j * 4 + pol) * 256 + tid] = acc[j][pol];
  };

  // segment workgroups first (kernel_adder_crowd listed the slots before
  // this launch), one per slot in turn; layer row 0 only
  if (static_cast<int>(blockIdx.x) < nworkers) {
    if (blockIdx.y != 0) return;
    const int total = min(sw.hdr[kSegTotal], sw.slot_cap);
    for (int p = blockIdx.x; p < total; p += nworkers) {
      const int h = sw.owner[p];
      if (h < 0) continue;
      const int4 he = sw.heavy[h];  // {tile, z, nseg, base}
      add_tile(he.x, he.y, p - he.w, p);
    }
    return;
  }
  // XCD-contiguous tiles (device.hpp: xcd_subgrid): horizontal neighbours,
  // whose subgrid reads share cache lines, run on the same XCD's L2
  const int tl = xcd_subgrid(blockIdx.x - nworkers, ntiles);
  if (nworkers > 0 && sw.tile_seg[blockIdx.y * ntiles + tl] >= 0)
    return;  // crowded: its segments and kernel_adder_combine
  add_tile(tl, blockIdx.y, -1, 0);
}

// F[s][pol][ys][xs] = conj(shift_phasor(x, y)) * grid[z][pol][cy + y][cx + x]
// (zero when the subgrid does not lie inside the grid).
__global__ void __launch_bounds__(256)
    kernel_splitter(const int4 *__restrict__ order,
                    const float2 *__restrict__ grid,
                    float2 *__restrict__ subgrids, int G, int S) {
  __shared__ float2 table[kAddMaxTable];
  // the home sort's entry {s, x, y, z}, z = -1 when not inside the grid
  const int4 e = order[xcd_subgrid(blockIdx.x, gridDim.x)];
  const int s = e.x;
  const int tid = threadIdx.x, nt = blockDim.x;
  const bool inside = e.w >= 0;
  const int npix = S * S;
  float2 *sg = subgrids + static_cast<size_t>(s) * 4 * npix;
  const float2 *gz =
      grid + static_cast<size_t>(inside ? e.w : 0) * 4 * G * G;
  // the shift phasor depends on x + y only: 2S - 1 values per subgrid
  const bool tabled = 2 * S - 1 <= kAddMaxTable;
  if (tabled)
    for (int k = tid; k < 2 * S - 1; k += nt)
      table[k] = unit_phasor(k * (S + 1) - S, 2 * S, -1.0f);
  __syncthreads();
  // pixel (y, x) of i = tid + nt * j, advanced without integer division
  const int dy = nt / S, dx = nt - (nt / S) * S;
  int y = tid / S, x = tid - (tid / S) * S;
  for (int i = tid; i < npix; i += nt) {
    const int dst = half_shift(y, S) * S + half_shift(x, S);
    const float2 ph = tabled ? table[x + y] : shift_phasor(x, y, S, -1.0f);
    const size_t src =
        static_cast<size_t>(e.z + y) * G + e.y + x;
#pragma unroll
    for (int pol = 0; pol < 4; ++pol)
      store_stream(&sg[pol * npix + dst],
                   inside ? cmulf(ph, gz[static_cast<size_t>(pol) * G * G + src])
                          : make_float2(0.0f, 0.0f));
    x += dx;
    y += dy;
    if (x >= S) {
      x -= S;
      ++y;
    }
  }
}

// The splitter for S = 32 / 64 (S/2 even): a thread owns PR pixel pairs
// (x, x + 1) of one row, whose fftshifted destinations are adjacent too
// (x + S/2 is even, so a pair never straddles the wrap), so each pair is one
// 16-byte store per correlation; every grid load of the thread is issued
// before its first store.  The same arithmetic as kernel_splitter.
template <int S>
__global__ void __launch_bounds__(256)
    kernel_splitter_pairs(const int4 *__restrict__ order,
                          const float2 *__restrict__ grid,
                          float4 *__restrict__ subgrids, int G) {
  static_assert(S % 4 == 0 && (S * S / 2) % 256 == 0, "whole pair rows");
  constexpr int PR = S * S / 2 / 256;  // pairs per thread
  constexpr int npix = S * S;
  __shared__ float2 table[2 * S - 1];
  // the home sort's entry {s, x, y, z}, z = -1 when not inside the grid
  const int4 e = order[xcd_subgrid(blockIdx.x, gridDim.x)];
  const int s = e.x;
  const int tid = threadIdx.x;
  const bool inside = e.w >= 0;
  for (int k = tid; k < 2 * S - 1; k += 256)
    table[k] = unit_phasor(k * (S + 1) - S, 2 * S, -1.0f);
  __syncthreads();
  float4 *sg = subgrids + static_cast<size_t>(s) * 4 * npix / 2;
  if (!inside) {
#pragma unroll
    for (int j = 0; j < PR; ++j)
#pragma unroll
      for (int pol = 0; pol < 4; ++pol)
        store_stream(&sg[pol * npix / 2 + tid + 256 * j],
                     make_float4(0.f, 0.f, 0.f, 0.f));
    return;
  }
  const float2 *gz = grid + static_cast<size_t>(e.w) * 4 * G * G;
  float2 v[PR][4][2];
#pragma unroll
  for (int j = 0; j < PR; ++j) {
    const int p = tid + 256 * j;
    const int y = p / (S / 2), x = 2 * (p % (S / 2));
    const size_t src =
        static_cast<size_t>(e.z + y) * G + e.y + x;
#pragma unroll
    for (int pol = 0; pol < 4; ++pol) {
      v[j][pol][0] = gz[static_cast<size_t>(pol) * G * G + src];
      v[j][pol][1] = gz[static_cast<size_t>(pol) * G * G + src + 1];
    }
  }
#pragma unroll
  for (int j = 0; j < PR; ++j) {
    const int p = tid + 256 * j;
    const int y = p / (S / 2), x = 2 * (p % (S / 2));
    const int dst = half_shift(y, S) * S + half_shift(x, S);  // even
    const float2 p0 = table[x + y], p1 = table[x + 1 + y];
#pragma unroll
    for (int pol = 0; pol < 4; ++pol) {
      const float2 a = cmulf(p0, v[j][pol][0]), b = cmulf(p1, v[j][pol][1]);
      store_stream(&sg[(pol * npix + dst) / 2],
                   make_float4(a.x, a.y, b.x, b.y));
    }
  }
}

// Power-of-two S: radix-2 Stockham FFT (log2 S stages per direction, natural
// order in and out) through two LDS buffers, the same transform as
// kernel_subgrid_dft.  Twiddles w^k = exp(sign 2 pi i k / S), k < S/2, from
// an LDS table.  Dynamic LDS: (2 S^2 + S/2) float2.
__global__ void __launch_bounds__(256)
    kernel_subgrid_fft2(float2 *__restrict__ planes, int S, int log2S,
                        float sign, float scale) {
  extern __shared__ float2 fft_lds[];
  float2 *buf0 = fft_lds;
  float2 *buf1 = buf0 + S * S;
  float2 *tw = buf1 + S * S;
  float2 *plane = planes + static_cast<size_t>(blockIdx.x) * S * S;
  const int tid = threadIdx.x, nthr = blockDim.x;
  const int npix = S * S, half = S / 2;
  for (int i = tid; i < half; i += nthr) tw[i] = unit_phasor(i, S, sign);
  for (int i = tid; i < npix; i += nthr) buf0[i] = plane[i];
  __syncthreads();
  float2 *src = buf0, *dst = buf1;
  // pass 0: rows (element stride 1, sequence stride S); pass 1: columns
#pragma unroll 1
  for (int pass = 0; pass < 2; ++pass) {
    const int es = pass == 0 ? 1 : S, ss = pass == 0 ? S : 1;
#pragma unroll 1
    for (int st = 0; st < log2S; ++st) {
      const int ns = 1 << st;           // current sub-transform length
      const int tstep = half >> st;     // twiddle index step S/(2 ns)
      for (int b = tid; b < npix / 2; b += nthr) {
        // consecutive lanes take consecutive elements (rows) or consecutive
        // sequences (columns): unit LDS stride, no bank conflicts
        int seq, j;
        if (pass == 0) {
          seq = b / half;
          j = b - seq * half;
        } else {
          j = b / S;
          seq = b - j * S;
        }
        const int k = j & (ns - 1);
        const int base = seq * ss;
        const float2 a0 = src[base + j * es];
        const float2 a1 = cmulf(src[base + (j + half) * es], tw[k * tstep]);
        const int d = ((j - k) << 1) + k;
        dst[base + d * es] = make_float2(a0.x + a1.x, a0.y + a1.y);
        dst[base + (d + ns) * es] = make_float2(a0.x - a1.x, a0.y - a1.y);
      }
      __syncthreads();
      float2 *t = src;
      src = dst;
      dst = t;
    }
  }
  for (int i = tid; i < npix; i += nthr)
    plane[i] = make_float2(src[i].x * scale, src[i].y * scale);
}

// S = 32 or 64: each thread owns one whole row, then one whole column, of a
// plane and transforms it in registers (radix-2 decimation in frequency,
// fully unrolled, so the bit-reversed output order is a compile-time register
// renaming); the planes pass through LDS once for the transpose (rows padded
// to N + 1 complex: conflict-free column reads).  A workgroup of 128 threads
// takes 128 / N planes, loaded and stored coalesced.  Same transform as
// kernel_subgrid_dft.
template <int N>
__global__ void __launch_bounds__(128)
    kernel_subgrid_fft_reg(float2 *__restrict__ planes, int nr_planes,
                           float sign, float scale) {
  constexpr int P = 128 / N;          // planes per workgroup
  constexpr int RS = N + 1;           // padded LDS row stride (complex)
  __shared__ float2 lds[P * N * RS];
  const int tid = threadIdx.x;
  const int p0 = blockIdx.x * P;
  const int np = min(P, nr_planes - p0);
  float2 *base = planes + static_cast<size_t>(p0) * N * N;

  // coalesced load of the workgroup's planes (contiguous), all loads of a
  // thread in flight before the first LDS write
  if (np == P) {
    constexpr int K = P * N * N / 2 / 128;  // float4 (2 complex) per thread
    const float4 *b4 = reinterpret_cast<const float4 *>(base);
    float4 v[K];
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = b4[tid + 128 * k];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int i = 2 * (tid + 128 * k);  // complex index, even
      const int pp = i / (N * N), r = i - pp * N * N;
      float2 *d = lds + pp * N * RS + (r / N) * RS + (r % N);
      d[0] = make_float2(v[k].x, v[k].y);
      d[1] = make_float2(v[k].z, v[k].w);
    }
  } else {
    for (int i = tid; i < np * N * N; i += 128) {
      const int pp = i / (N * N), r = i - pp * N * N;
      lds[pp * N * RS + (r / N) * RS + (r % N)] = base[i];
    }
  }
  float2 tw[N / 2];
#pragma unroll
  for (int k = 0; k < N / 2; ++k) tw[k] = unit_phasor(k, N, sign);
  __syncthreads();

  const int p = tid / N, q = tid % N;  // plane, row (then column)
  float2 x[N];
  // rows
#pragma unroll
  for (int i = 0; i < N; ++i) x[i] = lds[p * N * RS + q * RS + i];
  fft_dif_registers<N>(x, tw);
#pragma unroll
  for (int i = 0; i < N; ++i)
    lds[p * N * RS + q * RS + bit_reverse<N>(i)] = x[i];
  __syncthreads();
  // columns
#pragma unroll
  for (int i = 0; i < N; ++i) x[i] = lds[p * N * RS + i * RS + q];
  fft_dif_registers<N>(x, tw);
  if (p < np) {
    float2 *out = base + static_cast<size_t>(p) * N * N;
#pragma unroll
    for (int i = 0; i < N; ++i)
      store_stream(&out[bit_reverse<N>(i) * N + q],
                   make_float2(x[i].x * scale, x[i].y * scale));
  }
}

// The splitter and the degridding FFT (sign -1, scale 1/S^2) in one pass,
// for S = 32 / 64: the uv-domain subgrid never goes to HBM.  A unit of work
// is P = 128 / N correlation planes of one subgrid (a whole S = 32 subgrid,
// half an S = 64 one), taken in the home sort's order.  Persistent: a
// resident grid (a multiple of 8 workgroups of 128 threads), the workgroups
// of one XCD (blockIdx % 8) walking one contiguous eighth of the units, so
// they read overlapping grid windows from that XCD's L2 (0.259 against
// 0.271 ms for a workgroup per unit; loading the next unit's window behind
// the current transform took 256 VGPRs and spilled, 0.271 ms).  Every
// thread keeps one window column x (128 is a multiple of N), so each
// wave-load reads whole grid-row segments; the splitter's value
// cmulf(conj shift phasor, grid) goes straight to its fftshifted place in
// the padded LDS planes, and the rest is kernel_subgrid_fft_reg's transform
// (fft.hpp): the same operations in the same order as kernel_splitter_pairs
// followed by kernel_subgrid_fft_reg, so the output is bit for bit theirs.
// A subgrid not wholly inside the grid transforms zeros, as the two-kernel
// path does (its window is read at the grid's origin, in bounds as G >= N,
// and dropped).
template <int N>
__global__ void __launch_bounds__(128)
    kernel_splitter_fft(const int4 *__restrict__ order,
                        const float2 *__restrict__ grid,
                        float2 *__restrict__ subgrids, int G, int nunits,
                        float sign, float scale) {
  constexpr int P = 128 / N;   // planes per unit
  constexpr int WPS = 4 / P;   // units per subgrid
  constexpr int RS = N + 1;    // padded LDS row stride (complex)
  constexpr int K = P * N * N / 128;  // window values per thread
  __shared__ float2 lds[P * N * RS];
  __shared__ float2 table[2 * N - 1];
  const int tid = threadIdx.x;
  const int x = tid % N, y0 = tid / N, xs = half_shift(x, N);
  const int J = gridDim.x / 8;             // workgroups per XCD
  const int per = (nunits + 7) / 8;        // units per XCD
  const int xcd = blockIdx.x % 8;
  const int u1 = min(nunits, (xcd + 1) * per);
  for (int k = tid; k < 2 * N - 1; k += 128)
    table[k] = unit_phasor(k * (N + 1) - N, 2 * N, -1.0f);
  float2 tw[N / 2];
#pragma unroll
  for (int k = 0; k < N / 2; ++k) tw[k] = unit_phasor(k, N, sign);
  // a wave-uniform base per row k plus the lane's 32-bit byte offset
  const unsigned lane_off = static_cast<unsigned>((x + y0 * G) * 8);
  __syncthreads();  // table
  for (int u = xcd * per + blockIdx.x / 8; u < u1; u += J) {
    // the home sort's entry {s, x, y, z}, z = -1 when not inside the grid
    const int4 o = order[u / WPS];
    const int4 e = make_int4(__builtin_amdgcn_readfirstlane(o.x),
                             __builtin_amdgcn_readfirstlane(o.y),
                             __builtin_amdgcn_readfirstlane(o.z),
                             __builtin_amdgcn_readfirstlane(o.w));
    const int pol0 = (u % WPS) * P;
    const bool inside = e.w >= 0;
    const char *gz = reinterpret_cast<const char *>(
        grid + (static_cast<size_t>(inside ? e.w : 0) * 4 + pol0) * G * G +
        static_cast<size_t>(inside ? e.z : 0) * G + (inside ? e.y : 0));
    // rows r = y0 + P k: plane P k / N, row P k % N + y0 (y0 < P | N); every
    // load of the thread in flight before the first LDS write
    float2 v[K];
#pragma unroll
    for (int k = 0; k < K; ++k)
      v[k] = *reinterpret_cast<const float2 *>(
          gz + (static_cast<size_t>(P * k / N) * G * G +
                static_cast<size_t>(P * k % N) * G) * 8 + lane_off);
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int r = y0 + P * k, pp = r / N, y = r % N;
      lds[pp * N * RS + half_shift(y, N) * RS + xs] =
          inside ? cmulf(table[x + y], v[k]) : make_float2(0.0f, 0.0f);
    }
    __syncthreads();
    float2 f[N];
    fft2_planes_lds<N>(lds, tid, 128, tw, f);
    const int p = tid / N, q = tid % N;
    float2 *out = subgrids + (static_cast<size_t>(e.x) * 4 + pol0 + p) * N * N;
#pragma unroll
    for (int i = 0; i < N; ++i)
      store_stream(&out[bit_reverse<N>(i) * N + q],
                   make_float2(f[i].x * scale, f[i].y * scale));
    __syncthreads();  // the planes are rewritten by the next unit
  }
}

hipError_t launch_subgrid_fft(int nr_subgrids, int subgrid_size, int sign,
                              float scale, void *d_subgrids,
                              hipStream_t stream) {
  if (nr_subgrids <= 0) return hipSuccess;
  const int S = subgrid_size;
  const float sgn = sign >= 0 ? 1.0f : -1.0f;
  const int nplanes = 4 * nr_subgrids;
  if (S == 32) {
    hipLaunchKernelGGL(kernel_subgrid_fft_reg<32>, dim3((nplanes + 3) / 4),
                       dim3(128), 0, stream, static_cast<float2 *>(d_subgrids),
                       nplanes, sgn, scale);
    return hipGetLastError();
  }
  if (S == 64) {
    hipLaunchKernelGGL(kernel_subgrid_fft_reg<64>, dim3((nplanes + 1) / 2),
                       dim3(128), 0, stream, static_cast<float2 *>(d_subgrids),
                       nplanes, sgn, scale);
    return hipGetLastError();
  }
  if ((S & (S - 1)) == 0 && S >= 2) {
    int log2S = 0;
    while ((1 << log2S) < S) ++log2S;
    const size_t lds = (2 * static_cast<size_t>(S) * S + S / 2) *
                       sizeof(float2);
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    hipLaunchKernelGGL(kernel_subgrid_fft2, dim3(4 * nr_subgrids), dim3(256),
                       lds, stream, static_cast<float2 *>(d_subgrids), S,
                       log2S, sgn, scale);
    return hipGetLastError();
  }
  const size_t lds = (2 * static_cast<size_t>(S) * S + S) * sizeof(float2);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  hipLaunchKernelGGL(kernel_subgrid_dft, dim3(4 * nr_subgrids), dim3(256),
                     lds, stream, static_cast<float2 *>(d_subgrids), S, sgn,
                     scale);
  return hipGetLastError();
}

namespace {

// The home sort's workspace (util.hpp WorkspaceLease, cached per stream
// and held until the kernels that read it are enqueued): hist (16 nkeys,
// LDS form) | slot (2 ns) | offset (nkeys + 1) | order (ns) | count,
// cursor (nkeys each, multi-kernel form).  Every launch rewrites what it
// reads.
struct HomeSort {
  WorkspaceLease lease;
  int *ws = nullptr;
  int *offset = nullptr;
  int4 *order = nullptr;  // entries {s, x, y, z or -1}
};

// Dynamic LDS per workgroup the current device grants (cached per device):
// the LDS form of the home sort needs 2 x 4 nkeys bytes (kernel_home_place),
// sized for gfx950's 160 KB; a part with less takes the multi-kernel form.
size_t device_lds_per_block() {
  static std::mutex mu;
  static std::map<int, size_t> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  std::lock_guard<std::mutex> lock(mu);
  auto it = cache.find(dev);
  if (it != cache.end()) return it->second;
  int v = 0;
  if (hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerBlock,
                            dev) != hipSuccess)
    v = 0;
  cache[dev] = static_cast<size_t>(v);
  return cache[dev];
}

hipError_t home_sort(const idg::Metadata *md, int ns, int G, int S, int W,
                     hipStream_t stream, HomeSort *hs) {
  const TileGrid tg(G);
  const int nkeys = tg.nkeys(W);
  // IDG_HOME_SORT=multi forces the multi-kernel form (tests)
  const char *form = std::getenv("IDG_HOME_SORT");
  const bool multi = (form != nullptr && std::strcmp(form, "multi") == 0) ||
                     nkeys > kSortLdsKeys ||
                     2 * nkeys * sizeof(int) > device_lds_per_block();
  const int nwg = std::min(kSortMaxChunks, (ns + 3071) / 3072);
  const int chunk = (ns + nwg - 1) / nwg;
  const size_t ints =
      static_cast<size_t>(nkeys) + 1 + 8 * static_cast<size_t>(ns) +
      (multi ? 2 * static_cast<size_t>(nkeys)
             : static_cast<size_t>(kSortMaxChunks) * nkeys);
  hipError_t err =
      hs->lease.acquire(stream, kWorkspaceHomeSort, ints * sizeof(int));
  if (err != hipSuccess) return err;
  hs->ws = static_cast<int *>(hs->lease.ptr);
  // hist rows (64 B) first, then the 16-byte slot[] and order[] entries
  int *hist = hs->ws;
  int4 *slot = reinterpret_cast<int4 *>(
      hist + (multi ? 0 : static_cast<size_t>(kSortMaxChunks) * nkeys));
  hs->order = slot + ns;
  hs->offset = reinterpret_cast<int *>(hs->order + ns);
  int *rest = hs->offset + nkeys + 1;
  if (!multi) {
    hipLaunchKernelGGL(kernel_home_count, dim3(nwg), dim3(1024),
                       nkeys * sizeof(int), stream, md, ns, G, S, W, chunk,
                       hist, slot);
    hipLaunchKernelGGL(kernel_home_place, dim3(nwg), dim3(1024),
                       2 * nkeys * sizeof(int), stream, hist, nwg, nkeys,
                       tg.ntx * tg.nty, ns, chunk, slot, hs->offset,
                       hs->order);
    return hipGetLastError();
  }
  int *count = rest, *cursor = rest + nkeys;
  err = hipMemsetAsync(count, 0, nkeys * sizeof(int), stream);
  if (err != hipSuccess) return err;
  const int nb = (ns + 255) / 256;
  hipLaunchKernelGGL(kernel_home_key, dim3(nb), dim3(256), 0, stream, md, ns,
                     G, S, W, 0, count, cursor, hs->order);
  hipLaunchKernelGGL(kernel_home_scan, dim3(1), dim3(1024), 0, stream, count,
                     nkeys, hs->offset, cursor);
  hipLaunchKernelGGL(kernel_home_key, dim3(nb), dim3(256), 0, stream, md, ns,
                     G, S, W, 1, count, cursor, hs->order);
  return hipGetLastError();
}

// (the lease returns the workspace to the stream's cache when `hs` goes
// out of scope, after every kernel reading it is enqueued)
hipError_t free_home_sort(const HomeSort &hs, hipError_t err,
                          hipStream_t stream) {
  (void)hs;
  (void)stream;
  return err;
}

}  // namespace

hipError_t launch_adder(int nr_subgrids, int grid_size, int subgrid_size,
                        int nr_w_layers, const void *d_metadata,
                        const void *d_subgrids, void *d_grid,
                        hipStream_t stream) {
  if (nr_subgrids <= 0 || nr_w_layers <= 0 || grid_size <= 0)
    return hipSuccess;
  const auto *md = static_cast<const idg::Metadata *>(d_metadata);
  const TileGrid tg(grid_size);
  HomeSort hs;
  hipError_t err = home_sort(md, nr_subgrids, grid_size, subgrid_size,
                             nr_w_layers, stream, &hs);
  // crowded tiles split into segments (IDG_ADD_SEG=0: one workgroup per
  // tile whatever its list, the round-3 form)
  const char *segenv = std::getenv("IDG_ADD_SEG");
  const bool segmented = !(segenv != nullptr && segenv[0] == '0');
  AdderSeg sw;
  WorkspaceLease slease;
  int nworkers = 0;
  if (err == hipSuccess && segmented) {
    const AdderSegCaps caps =
        adder_seg_caps(nr_subgrids, subgrid_size, tg.ntx * tg.nty * nr_w_layers);
    err = slease.acquire(stream, kWorkspaceAdderSeg, caps.bytes);
    if (err == hipSuccess) {
      char *b = static_cast<char *>(slease.ptr);
      sw.heavy_cap = caps.heavy;
      sw.slot_cap = caps.slots;
      sw.hdr = reinterpret_cast<int *>(b);
      b += kSegHdrInts * sizeof(int);
      sw.partial = reinterpret_cast<float2 *>(b);
      b += static_cast<size_t>(caps.slots) * kAddPartialFloat2 * sizeof(float2);
      sw.heavy = reinterpret_cast<int4 *>(b);
      b += static_cast<size_t>(caps.heavy) * sizeof(int4);
      sw.owner = reinterpret_cast<int *>(b);
      b += static_cast<size_t>(caps.slots) * sizeof(int);
      sw.tile_seg = reinterpret_cast<int *>(b);
      // zero when new or after a failed launch; else left zero by
      // kernel_adder_combine's last workgroup
      if (!slease.clean)
        err = hipMemsetAsync(sw.hdr, 0, kSegHdrInts * sizeof(int), stream);
      nworkers = kAddWorkers;
    }
  }
  const int ntiles_all = tg.ntx * tg.nty * nr_w_layers;
  if (err == hipSuccess && nworkers > 0) {
    hipLaunchKernelGGL(kernel_adder_crowd, dim3((ntiles_all + 255) / 256),
                       dim3(256), 0, stream, hs.offset, grid_size,
                       subgrid_size, nr_w_layers, sw);
    err = hipGetLastError();
  }
  if (err == hipSuccess) {
    hipLaunchKernelGGL(kernel_adder,
                       dim3(nworkers + tg.ntx * tg.nty, nr_w_layers),
                       dim3(256), 0, stream, md, nr_subgrids, hs.offset,
                       hs.order, static_cast<const float2 *>(d_subgrids),
                       static_cast<float2 *>(d_grid), grid_size,
                       subgrid_size, nr_w_layers, sw, nworkers);
    err = hipGetLastError();
  }
  if (err == hipSuccess && nworkers > 0) {
    hipLaunchKernelGGL(kernel_adder_combine, dim3(kAddCombiners), dim3(256),
                       0, stream, static_cast<float2 *>(d_grid), grid_size,
                       sw);
    err = hipGetLastError();
  }
  slease.leave_clean = err == hipSuccess && nworkers > 0;
  return free_home_sort(hs, err, stream);
}

hipError_t launch_splitter(int nr_subgrids, int grid_size, int subgrid_size,
                           int nr_w_layers, const void *d_metadata,
                           const void *d_grid, void *d_subgrids,
                           hipStream_t stream) {
  if (nr_subgrids <= 0) return hipSuccess;
  const auto *md = static_cast<const idg::Metadata *>(d_metadata);
  HomeSort hs;
  hipError_t err = home_sort(md, nr_subgrids, grid_size, subgrid_size,
                             std::max(0, nr_w_layers), stream, &hs);
  if (err == hipSuccess) {
    if (subgrid_size == 32 || subgrid_size == 64)
      hipLaunchKernelGGL(subgrid_size == 32 ? kernel_splitter_pairs<32>
                                            : kernel_splitter_pairs<64>,
                         dim3(nr_subgrids), dim3(256), 0, stream, hs.order,
                         static_cast<const float2 *>(d_grid),
                         static_cast<float4 *>(d_subgrids), grid_size);
    else
      hipLaunchKernelGGL(kernel_splitter, dim3(nr_subgrids), dim3(256), 0,
                         stream, hs.order,
                         static_cast<const float2 *>(d_grid),
                         static_cast<float2 *>(d_subgrids), grid_size,
                         subgrid_size);
    err = hipGetLastError();
  }
  return free_home_sort(hs, err, stream);
}

hipError_t launch_splitter_fft(int nr_subgrids, int grid_size,
                               int subgrid_size, int nr_w_layers,
                               const void *d_metadata, const void *d_grid,
                               void *d_subgrids, hipStream_t stream) {
  if (nr_subgrids <= 0) return hipSuccess;
  const int S = subgrid_size;
  const float scale = 1.0f / static_cast<float>(S * S);
  // IDG_SPLIT_FFT=0: the two launches (A/B and tests)
  const char *env = std::getenv("IDG_SPLIT_FFT");
  // the fused kernel's static LDS (S = 64: ~66.5 KB, sized for gfx950's
  // 160 KB) against what the device grants a workgroup
  bool fits = true;
  if (S == 32 || S == 64) {
    hipFuncAttributes fa{};
    const void *f = S == 32 ? reinterpret_cast<const void *>(&kernel_splitter_fft<32>)
                            : reinterpret_cast<const void *>(&kernel_splitter_fft<64>);
    fits = hipFuncGetAttributes(&fa, f) == hipSuccess &&
           fa.sharedSizeBytes <= device_lds_per_block();
  }
  if ((S != 32 && S != 64) || !fits || (env != nullptr && env[0] == '0')) {
    const hipError_t err =
        launch_splitter(nr_subgrids, grid_size, S, nr_w_layers, d_metadata,
                        d_grid, d_subgrids, stream);
    if (err != hipSuccess) return err;
    return launch_subgrid_fft(nr_subgrids, S, -1, scale, d_subgrids, stream);
  }
  const auto *md = static_cast<const idg::Metadata *>(d_metadata);
  HomeSort hs;
  hipError_t err = home_sort(md, nr_subgrids, grid_size, S,
                             std::max(0, nr_w_layers), stream, &hs);
  if (err == hipSuccess) {
    const int nunits = nr_subgrids * (S == 32 ? 1 : 2);
    const void *func = S == 32
                           ? reinterpret_cast<const void *>(
                                 &kernel_splitter_fft<32>)
                           : reinterpret_cast<const void *>(
                                 &kernel_splitter_fft<64>);
    // a multiple of 8 workgroups (whole XCD rows), at most the resident
    // grid and at most one per unit (rounded up to the multiple of 8)
    const int resident = std::max(8, resident_workgroups(func, 128) / 8 * 8);
    const int nwg = std::min(resident, (nunits + 7) / 8 * 8);
    int G = grid_size;
    float sign = -1.0f, sc = scale;
    const int4 *order = hs.order;
    int nu = nunits;
    void *args[] = {&order, const_cast<void **>(&d_grid), &d_subgrids, &G,
                    &nu,    &sign,                         &sc};
    err = hipLaunchKernel(func, dim3(nwg), dim3(128), args, 0, stream);
  }
  return free_home_sort(hs, err, stream);
}

}  // namespace idg_mi355x
