/*
 * idg_mi355x.h -- C ABI of the MI355X IDG gridder/degridder
 *                 (libidg_mi355x.so, built from ska-sdp-idg-bench_amd/csrc).
 *
 * Plain C: pointers, sizes, int status codes; no C++ or torch types.  Each
 * entry point names the reference interface of ska-telescope/ska-sdp-idg-bench
 * it replaces.  The reference's own binding for this path is C++
 * (hip::c_run_gridder et al. with idg::ArrayND& arguments, mangled names);
 * libidg_mi355x.so exports those C++ symbols too (ska-sdp-idg-bench_amd/csrc/
 * lib-hip.hpp), and this header is the flat C twin an FFI (ctypes, cgo, JNI,
 * N-API) binds.  See INTEGRATION.md.
 *
 * Layouts (row-major, complex = interleaved {re, im} float32):
 *   uvw           [rows]                 idg_uvw_t     (rows = visibility rows)
 *   wavenumbers   [nr_channels]          float
 *   visibilities  [rows][nr_channels][4] idg_cfloat_t  (xx, xy, yx, yy)
 *   spheroidal    [S][S]                 float
 *   aterms        [slots][nr_stations][S][S][4] idg_cfloat_t
 *   metadata      [nr_subgrids]          idg_metadata_t
 *   subgrids      [nr_subgrids][4][S][S] idg_cfloat_t  (correlation-planar)
 * Row index of timestep t of subgrid s:
 *   (md[s].baseline_offset - md[0].baseline_offset) + md[s].time_offset + t
 *
 * Status: 0 = success, > 0 = hipError_t of the failing HIP call, < 0 = the
 * IDG_E_* codes below; idg_last_error() describes the last failure of the
 * calling thread.  (The reference's C++ entries abort the process on error,
 * app/HIP/util.cpp:5-15; the C++ symbols of this library keep that.)
 */
#ifndef IDG_MI355X_H_
#define IDG_MI355X_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define IDG_MI355X_ABI_VERSION 1

#define IDG_OK 0
#define IDG_E_INVALID_ARGUMENT (-1) /* bad sizes / null pointers          */
#define IDG_E_OUT_OF_BOUNDS (-2)    /* metadata indexes outside a buffer  */
#define IDG_E_NO_DEVICE (-3)        /* no HIP device visible              */

/* idg::Metadata (reference app/common/types.hpp:11-26), 36 bytes. */
typedef struct idg_metadata_t {
  int32_t baseline_offset;
  int32_t time_offset;
  int32_t nr_timesteps;
  int32_t aterm_index;
  uint32_t station1;
  uint32_t station2;
  int32_t coord_x;
  int32_t coord_y;
  int32_t coord_z;
} idg_metadata_t;

/* idg::UVWCoordinate<float> (types.hpp:49-54). */
typedef struct idg_uvw_t {
  float u, v, w;
} idg_uvw_t;

/* std::complex<float> */
typedef struct idg_cfloat_t {
  float re, im;
} idg_cfloat_t;

int idg_abi_version(void);

/* ---- host-buffer entries (synchronous, allocate + copy + launch + copy) ---
 * Replace hip::c_run_gridder / hip::c_run_degridder, the kernel-TU contract
 * of the reference (app/HIP/kernels/gridder_v1.hip.cpp:118-137 and
 * degridder_v1.hip.cpp; declared by the harness at
 * tests/gridder_common.cpp:21-30, tests/degridder_common.cpp:21-30), which
 * run app/HIP/util.cpp:255-311 / :392-448.  The ArrayND arguments become
 * (pointer, element count): uvw_rows UVW triplets (visibilities then hold
 * uvw_rows * nr_channels * 4 complex values) and aterm_slots timeslots.
 * Metadata is validated against these extents before anything is launched.
 * The gridder fully overwrites subgrids; the degridder writes every
 * visibility row referenced by the metadata. */
int idg_c_run_gridder(int nr_subgrids, int grid_size, int subgrid_size,
                      float image_size, float w_step_in_lambda,
                      int nr_channels, int nr_stations, const idg_uvw_t *uvw,
                      size_t uvw_rows, const float *wavenumbers,
                      const idg_cfloat_t *visibilities,
                      const float *spheroidal, const idg_cfloat_t *aterms,
                      size_t aterm_slots, const idg_metadata_t *metadata,
                      idg_cfloat_t *subgrids);

int idg_c_run_degridder(int nr_subgrids, int grid_size, int subgrid_size,
                        float image_size, float w_step_in_lambda,
                        int nr_channels, int nr_stations,
                        const idg_uvw_t *uvw, size_t uvw_rows,
                        const float *wavenumbers, idg_cfloat_t *visibilities,
                        const float *spheroidal, const idg_cfloat_t *aterms,
                        size_t aterm_slots, const idg_metadata_t *metadata,
                        const idg_cfloat_t *subgrids);

/* ---- device-buffer entries (asynchronous on `stream`) ---------------------
 * The launch half of the same pipeline: hipLaunchKernel with the 13-argument
 * kernel ABI, grid = nr_subgrids, block = 256 (reference
 * app/HIP/util.cpp:167-174 c_run_kernel and :237-244).  All pointers are
 * device pointers, resident in HBM; `stream` is a hipStream_t (NULL = the
 * legacy default stream).  The caller guarantees metadata validity (use
 * idg_validate_metadata on a host copy). */
int idg_gridder_launch(int nr_subgrids, int grid_size, int subgrid_size,
                       float image_size, float w_step_in_lambda,
                       int nr_channels, int nr_stations, const idg_uvw_t *uvw,
                       const float *wavenumbers,
                       const idg_cfloat_t *visibilities,
                       const float *spheroidal, const idg_cfloat_t *aterms,
                       const idg_metadata_t *metadata, idg_cfloat_t *subgrids,
                       void *stream);

int idg_degridder_launch(int nr_subgrids, int grid_size, int subgrid_size,
                         float image_size, float w_step_in_lambda,
                         int nr_channels, int nr_stations,
                         const idg_uvw_t *uvw, const float *wavenumbers,
                         idg_cfloat_t *visibilities, const float *spheroidal,
                         const idg_cfloat_t *aterms,
                         const idg_metadata_t *metadata,
                         const idg_cfloat_t *subgrids, void *stream);

/* Host-side bounds check of metadata against the buffer extents (what the
 * host-buffer entries run before launching).  Returns IDG_OK or
 * IDG_E_OUT_OF_BOUNDS / IDG_E_INVALID_ARGUMENT. */
int idg_validate_metadata(int nr_subgrids, int subgrid_size, int nr_channels,
                          int nr_stations, size_t uvw_rows, size_t aterm_slots,
                          const idg_metadata_t *metadata);

/* The chunk plan the host-buffer entries use for a batch whose copies move
 * bytes_moved bytes (visibilities + subgrids): consecutive subgrid ranges
 * [bounds[i], bounds[i+1]) whose visibility rows are disjoint and ascending,
 * so chunk i's copies overlap chunk i-1's kernel; one chunk when the rows are
 * not.  Writes at most max_bounds entries of bounds (nchunk + 1 in all) and
 * returns nchunk (< 0 on bad arguments).  No reference counterpart: the
 * reference's c_run_* copies everything, launches once, copies back
 * (app/HIP/util.cpp:255-311). */
int idg_host_chunk_plan(int nr_subgrids, const idg_metadata_t *metadata,
                        size_t bytes_moved, int *bounds, int max_bounds);

/* Name of the kernel the launch entries select for this geometry
 * (direction 0 = gridder, 1 = degridder); for profiles and reports. */
const char *idg_kernel_name(int direction, int subgrid_size, int nr_channels);

/* Precision options of the kernels the launch entries select for this
 * geometry (bit 0: the phase-reduction tail on every phasor, bit 1: blocked
 * summation, bit 2: the tail on one channel per quad); the
 * IDG_PREC environment variable overrides them.  No reference counterpart:
 * the reference's kernels have a single precision path. */
int idg_precision_options(int direction, int subgrid_size, int nr_channels);

/* ---- perf entries ---------------------------------------------------------
 * Replace hip::p_run_gridder / hip::p_run_degridder (kernel TUs, e.g.
 * gridder_v1.hip.cpp:114-116 -> app/HIP/util.cpp:176-253 / :313-390): the
 * problem comes from the environment (NR_STATIONS=50, NR_TIMESLOTS=20,
 * NR_TIMESTEPS_SUBGRID=128, NR_CHANNELS=16, SUBGRID_SIZE=32, GRID_SIZE=1024,
 * NR_WARM_UP_RUNS=2, NR_ITERATIONS=5), prints the reference report line and
 * CSV; returns milliseconds per launch (< 0 on error). */
double idg_p_run_gridder(void);
double idg_p_run_degridder(void);

/* ---- device info (app/lib-hip.hpp:5-9) ----------------------------------- */
void idg_print_device_info(void);
void idg_print_benchmark(void);
/* extern_get_device_name (declared, never defined, in the reference).
 * Writes at most len bytes incl. NUL; returns the full name length. */
int idg_get_device_name(char *buf, size_t len);

/* ---- work model (app/common/common.cpp:100-159) -------------------------- */
uint64_t idg_flops_gridder(uint64_t nr_channels, uint64_t nr_timesteps,
                           uint64_t nr_subgrids, uint64_t subgrid_size,
                           uint64_t nr_correlations);
uint64_t idg_bytes_gridder(uint64_t nr_channels, uint64_t nr_timesteps,
                           uint64_t nr_subgrids, uint64_t subgrid_size,
                           uint64_t nr_correlations);

/* ---- pipeline steps either side of the path ----
 * Not in the reference (its Grid type is unused, app/common/types.hpp:358-370):
 * these complete gridding into, and degridding from, a uv grid.  Conventions
 * (DESIGN.md §8f):
 *   gridding:   idg_gridder_launch -> idg_subgrid_fft_launch(+1, 1.0f)
 *               -> idg_adder_launch
 *   degridding: idg_splitter_launch -> idg_subgrid_fft_launch(-1, 1/S^2)
 *               -> idg_degridder_launch
 * grid: [nr_w_layers][4][grid_size][grid_size] complex64; a subgrid goes to
 * layer metadata.coordinate.z.  Device pointers, asynchronous on `stream`.
 */

/* In-place 2-D DFT of each [S][S] correlation plane of subgrids
 * [nr_subgrids][4][S][S]: out[k][l] = scale * sum in[y][x] *
 * exp(sign * 2 pi i (k y + l x) / S); sign = +1 or -1. */
int idg_subgrid_fft_launch(int nr_subgrids, int subgrid_size, int sign,
                           float scale, idg_cfloat_t *subgrids, void *stream);

/* grid[z][pol][y0 + y][x0 + x] += exp(i pi ((x + y)(S + 1)/S - 1)) *
 * subgrid[s][pol][(y + S/2) % S][(x + S/2) % S]; subgrids not wholly inside
 * the grid are skipped.  Deterministic: a per-tile gather in subgrid order,
 * no atomics. */
int idg_adder_launch(int nr_subgrids, int grid_size, int subgrid_size,
                     int nr_w_layers, const idg_metadata_t *metadata,
                     const idg_cfloat_t *subgrids, idg_cfloat_t *grid,
                     void *stream);

/* The adjoint placement: subgrid[s][pol][(y + S/2) % S][(x + S/2) % S] =
 * exp(-i pi ((x + y)(S + 1)/S - 1)) * grid[z][pol][y0 + y][x0 + x]; zero for
 * subgrids not wholly inside the grid. */
int idg_splitter_launch(int nr_subgrids, int grid_size, int subgrid_size,
                        int nr_w_layers, const idg_metadata_t *metadata,
                        const idg_cfloat_t *grid, idg_cfloat_t *subgrids,
                        void *stream);

/* idg_gridder_launch followed by idg_subgrid_fft_launch(+1, 1.0f): the
 * adder's input subgrids straight from the visibilities.  For S = 32 the FFT
 * runs in the gridder's epilogue (the image-domain subgrids never reach
 * HBM), bit for bit the two launches' result; other S <= 64 run the two
 * launches.  Arguments as idg_gridder_launch. */
int idg_gridder_fft_launch(int nr_subgrids, int grid_size, int subgrid_size,
                           float image_size, float w_step_in_lambda,
                           int nr_channels, int nr_stations,
                           const idg_uvw_t *uvw, const float *wavenumbers,
                           const idg_cfloat_t *visibilities,
                           const float *spheroidal, const idg_cfloat_t *aterms,
                           const idg_metadata_t *metadata,
                           idg_cfloat_t *subgrids, void *stream);

/* idg_splitter_launch followed by idg_subgrid_fft_launch(-1, 1/S^2): the
 * degridder's input subgrids straight from the grid.  For S = 32 and 64 one
 * fused kernel (the uv-domain subgrids never reach HBM), bit for bit the
 * two launches' result; other even S <= 64 run the two launches. */
int idg_splitter_fft_launch(int nr_subgrids, int grid_size, int subgrid_size,
                            int nr_w_layers, const idg_metadata_t *metadata,
                            const idg_cfloat_t *grid, idg_cfloat_t *subgrids,
                            void *stream);

/* ---- synthetic observation (app/common/init.cpp:4-180) -------------------
 * Exactly the reference harness' inputs: srand(0), then the initialize_*
 * generators in harness order.  nr_subgrids = nr_stations*(nr_stations-1)/2
 * * nr_timeslots is returned.  Any output pointer may be NULL to skip it
 * (the random stream is consumed identically either way).  Sizes:
 *   uvw [nr_subgrids*nr_timesteps], frequencies/wavenumbers [nr_channels],
 *   visibilities [nr_subgrids*nr_timesteps*nr_channels*4],
 *   spheroidal [S*S], aterms [nr_timeslots*nr_stations*S*S*4],
 *   metadata [nr_subgrids], subgrids [nr_subgrids*4*S*S].
 * nthreads > 1 parallelises the (random-free) visibility generator. */
int idg_generate(int nr_stations, int nr_timeslots, int nr_timesteps,
                 int nr_channels, int grid_size, int subgrid_size,
                 idg_uvw_t *uvw, float *frequencies, float *wavenumbers,
                 idg_cfloat_t *visibilities, float *spheroidal,
                 idg_cfloat_t *aterms, idg_metadata_t *metadata,
                 idg_cfloat_t *subgrids, int nthreads);

/* ---- workspaces -----------------------------------------------------------
 * The device entries keep their scratch (the two-kernel form's subgrid queue,
 * the adder's home sort and segment lists) cached per (device, stream), so a
 * launch makes no allocation.  idg_release_workspaces frees the cache of
 * `stream` on the current device (all != 0: of every stream of the current
 * device).  The stream(s) must be idle (their work complete): call it before
 * destroying a stream the entries used -- a new stream may be given the same
 * handle -- and before hipDeviceReset.  Returns IDG_OK or a HIP error code
 * (hipErrorNotReady: a slot was being enqueued on by another host thread and
 * was left).  No reference counterpart (the reference allocates per call,
 * app/HIP/util.cpp:220-232). */
int idg_release_workspaces(void *stream, int all);

const char *idg_last_error(void);

#ifdef __cplusplus
}
#endif

#endif /* IDG_MI355X_H_ */
