/*
 * idg_oracle.h -- CPU oracle for the IDG gridder / degridder hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product library
 * (ska-sdp-idg-bench_amd/) includes, links or calls this file.  It is used by
 * tests/, by __graft_entry__.smoke() and by bench.py's cpu_baseline leg, always
 * as the checker, never as the thing measured or shipped.
 *
 * Plain-C restatement of
 *   cpu::kernel_gridder_reference    app/CPU/kernels/gridder_reference.cpp:6-114
 *   cpu::kernel_degridder_reference  app/CPU/kernels/degridder_reference.cpp:6-129
 * of ska-telescope/ska-sdp-idg-bench.  Pinned against golden vectors generated
 * from the reference's own CPU path (tests/golden/, oracle/make_golden.sh).
 */
#ifndef IDG_ORACLE_H_
#define IDG_ORACLE_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Same 36-byte layout as idg::Metadata (app/common/types.hpp:11-26). */
typedef struct oracle_metadata {
  int32_t baseline_offset;
  int32_t time_offset;
  int32_t nr_timesteps;
  int32_t aterm_index;
  uint32_t station1;
  uint32_t station2;
  int32_t x, y, z;
} oracle_metadata;

/*
 * Array layouts (all row-major, complex = interleaved {re, im} float):
 *   uvw           [rows][3]                 float  (u, v, w)
 *   wavenumbers   [nr_channels]             float
 *   visibilities  [rows][nr_channels][4]    complex
 *   spheroidal    [S][S]                    float
 *   aterms        [slots][nr_stations][S][S][4] complex
 *   metadata      [nr_subgrids]
 *   subgrids      [nr_subgrids][4][S][S]    complex
 * `nthreads` <= 1 runs single-threaded (the reference as built: its OpenMP
 * pragma is inert, CMakeLists.txt:42 has no -fopenmp).
 */
void oracle_gridder(int nr_subgrids, int grid_size, int subgrid_size,
                    float image_size, float w_step_in_lambda, int nr_channels,
                    int nr_stations, const float *uvw, const float *wavenumbers,
                    const float *visibilities, const float *spheroidal,
                    const float *aterms, const oracle_metadata *metadata,
                    float *subgrids, int nthreads);

void oracle_degridder(int nr_subgrids, int grid_size, int subgrid_size,
                      float image_size, float w_step_in_lambda,
                      int nr_channels, int nr_stations, const float *uvw,
                      const float *wavenumbers, float *visibilities,
                      const float *spheroidal, const float *aterms,
                      const oracle_metadata *metadata, const float *subgrids,
                      int nthreads);

/*
 * Exact-accumulation twins of the two kernels (a measuring instrument, no
 * reference counterpart): the reference's f32 phase exactly as above, then
 * cos/sin of it and every product, sum, A-term and taper in double.
 * Outputs are double [re, im] pairs with the layouts above.
 */
void oracle_gridder_exact(int nr_subgrids, int grid_size, int subgrid_size,
                          float image_size, float w_step_in_lambda,
                          int nr_channels, int nr_stations, const float *uvw,
                          const float *wavenumbers, const float *visibilities,
                          const float *spheroidal, const float *aterms,
                          const oracle_metadata *metadata, double *subgrids,
                          int nthreads);

void oracle_degridder_exact(int nr_subgrids, int grid_size, int subgrid_size,
                            float image_size, float w_step_in_lambda,
                            int nr_channels, int nr_stations,
                            const float *uvw, const float *wavenumbers,
                            double *visibilities, const float *spheroidal,
                            const float *aterms,
                            const oracle_metadata *metadata,
                            const float *subgrids, int nthreads);

/*
 * check_error metric of tests/test_util.hpp:28-92: A = candidate, B =
 * reference, n complex values.  Returns the normalised RMS error; PASS iff
 * <= 1e-5.  *nnz receives the number of entries with |B| > 0.
 */
double oracle_check_error(int64_t n, const float *A, const float *B,
                          int64_t *nnz);

#ifdef __cplusplus
}
#endif

#endif
