// mall_probe.hip -- does rocprofv3's FETCH_SIZE (TCC_EA0_RDREQ) count reads
// that the Infinity Cache (MALL, 256 MiB) serves?  (DESIGN EVIDENCE for the
// traffic figures in profiles/traffic.json.)
//
// k_read sweeps a buffer once per launch with 16-B coalesced loads, every
// workgroup a contiguous slice.  Each buffer size is swept kPasses times
// back to back:
//   64 MiB, 128 MiB  larger than the 32 MiB of L2, smaller than the MALL:
//                    from the second pass on, every line a MALL hit;
//   2 GiB            larger than the MALL: every pass from HBM.
// If FETCH_SIZE per launch stays at the buffer size for the MALL-resident
// sweeps, it counts MALL hits; if it drops towards zero, it does not.  The
// per-launch time (printed) shows where the bytes came from either way.
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace -- ./mall_probe
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kPasses = 6;

__global__ void __launch_bounds__(256) k_read(const float4 *__restrict__ in,
                                              size_t n4, float *out) {
  const size_t per = n4 / gridDim.x;
  const float4 *p = in + static_cast<size_t>(blockIdx.x) * per;
  float acc = 0.0f;
  for (size_t i = threadIdx.x; i < per; i += 256) {
    const float4 a = p[i];
    acc += a.x + a.y + a.z + a.w;
  }
  if (acc == 1234.5f) out[threadIdx.x] = acc;
}

int main() {
  const size_t sizes[] = {size_t(64) << 20, size_t(128) << 20,
                          size_t(2) << 30};
  float *out = nullptr;
  if (hipMalloc(&out, 1024 * sizeof(float)) != hipSuccess) return 2;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (size_t bytes : sizes) {
    float4 *buf = nullptr;
    if (hipMalloc(&buf, bytes) != hipSuccess) return 2;
    (void)hipMemset(buf, 0, bytes);
    (void)hipDeviceSynchronize();
    const size_t n4 = bytes / sizeof(float4);
    const int grid = 4096;  // 16 per CU; slices of bytes / 4096
    for (int pass = 0; pass < kPasses; ++pass) {
      (void)hipEventRecord(e0, 0);
      hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, buf, n4, out);
      (void)hipEventRecord(e1, 0);
      (void)hipEventSynchronize(e1);
      float ms = 0.0f;
      (void)hipEventElapsedTime(&ms, e0, e1);
      printf("bytes %zu pass %d ms %.4f TB/s %.2f\n", bytes, pass, ms,
             bytes / (ms * 1e-3) / 1e12);
    }
    (void)hipFree(buf);
  }
  (void)hipFree(out);
  return 0;
}
