// traffic_probe.hip -- calibrates rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950
// for the access shapes the IDG kernels use (DESIGN EVIDENCE).
//
// Each kernel moves exactly 1 GiB once; the counters of each dispatch are
// divided by 2^30 to give the factor to apply to the hot kernels' readings.
//   k_sload_x8   wave-uniform 32-B scalar loads (gridder visibilities)
//   k_load_x2    8 B/lane coalesced global loads (degridder subgrid reads)
//   k_load_x4    16 B/lane coalesced global loads (the guide's "1/2" case)
//   k_store_rows 16 x 16 B per lane, lanes 256 B apart (degridder stores)
//   k_store_x2   8 B/lane coalesced stores (gridder subgrid stores)
//   k_fill_gather the gridder's B-fragment fill (round 2): 4 B per lane,
//                SGPR base + fixed lane offset; a wave reads 4 rows x 4
//                items x 32 B per K-step, every word by two lanes
//   rocprofv3 --pmc FETCH_SIZE -- ./traffic_probe ; ... --pmc WRITE_SIZE ...
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr size_t kBytes = size_t(1) << 30;

__global__ void __launch_bounds__(256) k_sload_x8(const float4 *__restrict__ in,
                                                  float *out) {
  // one workgroup streams a contiguous 64 KiB chunk through the scalar unit
  const float4 *p = in + static_cast<size_t>(blockIdx.x) * 4096;
  float acc = 0.0f;
  for (int i = 0; i < 4096; i += 2) {
    const float4 a = p[i], b = p[i + 1];
    acc += a.x + a.y + a.z + a.w + b.x + b.y + b.z + b.w;
  }
  if (acc == 1234.5f) out[threadIdx.x] = acc;
}

__global__ void __launch_bounds__(256) k_load_x2(const float2 *__restrict__ in,
                                                 float *out) {
  const size_t i = static_cast<size_t>(blockIdx.x) * 256 + threadIdx.x;
  const float2 v = in[i];
  if (v.x + v.y == 1234.5f) out[threadIdx.x] = v.x;
}

__global__ void __launch_bounds__(256) k_load_x4(const float4 *__restrict__ in,
                                                 float *out) {
  const size_t i = static_cast<size_t>(blockIdx.x) * 256 + threadIdx.x;
  const float4 v = in[i];
  if (v.x + v.y + v.z + v.w == 1234.5f) out[threadIdx.x] = v.x;
}

__global__ void __launch_bounds__(256) k_store_rows(float4 *__restrict__ out) {
  const size_t lane = static_cast<size_t>(blockIdx.x) * 256 + threadIdx.x;
  float4 *p = out + lane * 16;
  for (int j = 0; j < 16; ++j) p[j] = make_float4(lane, j, 0, 1);
}

__global__ void __launch_bounds__(256) k_store_x2(float2 *__restrict__ out) {
  const size_t i = static_cast<size_t>(blockIdx.x) * 256 + threadIdx.x;
  out[i] = make_float2(i, 1);
}

__global__ void __launch_bounds__(256) k_fill_gather(const float *__restrict__ in,
                                                     float *out) {
  // rows of 16 items x 8 floats (C = 16); one wave = one quad of rows,
  // four K-steps of 4 items (the fill of gridder_mi355x.hip.cpp)
  constexpr int C = 16;
  const int lane = threadIdx.x & 63, grp = lane >> 4, col = lane & 15;
  const int bpol = (col & 7) >> 1;
  const int w_c = 2 * bpol + (col & 1), w_s = 2 * bpol + 1 - (col & 1);
  const size_t quad = static_cast<size_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const float *rows = in + quad * 4 * C * 8;
  const unsigned off_c = (grp * C * 8 + w_c) * 4u;
  const unsigned off_s = (grp * C * 8 + w_s) * 4u;
  float acc = 0.0f;
  for (int j = 0; j < C / 4; ++j) {
    const char *blk = reinterpret_cast<const char *>(rows + 4 * j * 8);
#pragma unroll
    for (int u = 0; u < 4; ++u)
      acc += *reinterpret_cast<const float *>(blk + off_c + 32 * u) +
             *reinterpret_cast<const float *>(blk + off_s + 32 * u);
  }
  if (acc == 1234.5f) out[threadIdx.x] = acc;
}

int main() {
  void *buf, *out;
  if (hipMalloc(&buf, kBytes) != hipSuccess || hipMalloc(&out, 4096)) return 1;
  (void)hipMemset(buf, 0, kBytes);
  (void)hipDeviceSynchronize();
  hipLaunchKernelGGL(k_sload_x8, dim3(kBytes / 65536), dim3(256), 0, 0,
                     (const float4 *)buf, (float *)out);
  hipLaunchKernelGGL(k_load_x2, dim3(kBytes / 8 / 256), dim3(256), 0, 0,
                     (const float2 *)buf, (float *)out);
  hipLaunchKernelGGL(k_load_x4, dim3(kBytes / 16 / 256), dim3(256), 0, 0,
                     (const float4 *)buf, (float *)out);
  hipLaunchKernelGGL(k_fill_gather, dim3(kBytes / (4 * 4 * 16 * 32)), dim3(256),
                     0, 0, (const float *)buf, (float *)out);
  hipLaunchKernelGGL(k_store_rows, dim3(kBytes / 256 / 256), dim3(256), 0, 0,
                     (float4 *)buf);
  hipLaunchKernelGGL(k_store_x2, dim3(kBytes / 8 / 256), dim3(256), 0, 0,
                     (float2 *)buf);
  const hipError_t e = hipDeviceSynchronize();
  std::printf("traffic probe: %s, each kernel moves %zu bytes\n",
              hipGetErrorString(e), kBytes);
  return e == hipSuccess ? 0 : 1;
}
