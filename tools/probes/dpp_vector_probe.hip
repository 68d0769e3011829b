// dpp_vector_probe.hip -- a hipcc (ROCm 7.2) miscompile the gridder's
// blocked summation ran into: a DPP row_ror:8 move applied
// to each element of an ext_vector float4 in a loop is emitted as ONE DPP
// move of element 0, reused for all four (v_mov_b32_dpp v4, v0 row_ror:8;
// v_pk_add_f32 ... op_sel_hi:[1,0]) when the builtin is written inline in
// the loop (loop_form).  Through the row_ror8 helper (device.hpp) on named
// scalars it is four moves (scalar_form).  Compile-only check (tests/test_isa.py):
//   hipcc --offload-arch=gfx950 -O3 --cuda-device-only -S dpp_vector_probe.hip
#include <hip/hip_runtime.h>

#include "hip/kernels/device.hpp"

typedef float floatx4 __attribute__((ext_vector_type(4)));

__global__ void loop_form(floatx4 *p, float4 *o) {
  floatx4 a = p[threadIdx.x], v;
#pragma unroll
  for (int r = 0; r < 4; ++r)
    v[r] = a[r] + __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
                                                0, __builtin_bit_cast(int, a[r]),
                                                0x128, 0xF, 0xF, false));
  o[threadIdx.x] = make_float4(v[0], v[1], v[2], v[3]);
}

__global__ void scalar_form(floatx4 *p, float4 *o) {
  const floatx4 a = p[threadIdx.x];
  const float a0 = a[0], a1 = a[1], a2 = a[2], a3 = a[3];
  o[threadIdx.x] = make_float4(a0 + idg_mi355x::row_ror8(a0),
                               a1 + idg_mi355x::row_ror8(a1),
                               a2 + idg_mi355x::row_ror8(a2),
                               a3 + idg_mi355x::row_ror8(a3));
}
