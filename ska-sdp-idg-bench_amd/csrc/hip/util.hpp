// util.hpp -- the HIP launch-and-buffer layer.
//
// Keeps the reference's app/HIP/util.hpp:13-63 API (p_run_kernel,
// c_run_kernel, p_run_gridder_ / c_run_gridder_, p_run_degridder_ /
// c_run_degridder_, device queries) so a kernel TU written against the
// reference drops in here and vice versa.  Differences, all deliberate:
//   * sizes are size_t end to end (the reference's int products overflow at
//     nr_channels = 256, util.cpp:220-231);
//   * every HIP call is checked; metadata is validated against the buffer
//     sizes on the host before any launch (a bad index would fault the GPU);
//   * the perf entry uploads real synthetic inputs (the reference times
//     kernels on uninitialised memory, util.cpp:234-235);
//   * launches go to an explicit stream (nullptr = legacy default stream).
#pragma once

#include <hip/hip_runtime.h>

#include <string>
#include <utility>
#include <vector>

#include "lib-common.hpp"

namespace hip {

// Aborts the process on error, as the reference's hipCheck does
// (util.cpp:5-15).
#define hipCheck(ans) ::hip::hip_assert((ans), __FILE__, __LINE__)
void hip_assert(hipError_t code, const char *file, int line, bool abort = true);

std::string get_device_name();
void print_device_info();
std::vector<int> get_launch_kernel_dimensions();
int get_cu_nr();
int get_max_threads();
size_t get_gmem_size();
int get_cu_freq();
void print_dimensions(dim3 gridDim, dim3 blockDim);

// Warm-up + event-timed loop of NR_ITERATIONS launches, then report() and
// report_csv() (reference util.cpp:81-165).  Returns seconds per launch.
double p_run_kernel(const void *func, dim3 gridDim, dim3 blockDim,
                    void **args, std::string func_name = "",
                    double gflops = 0, double gbytes = 0, double mvis = 0);

// One launch (reference util.cpp:167-174).
void c_run_kernel(const void *func, dim3 gridDim, dim3 blockDim, void **args);

void p_run_gridder_(const void *func, std::string func_name, int num_threads);

void c_run_gridder_(
    int nr_subgrids, int grid_size, int subgrid_size, float image_size,
    float w_step_in_lambda, int nr_channels, int nr_stations,
    idg::Array2D<idg::UVWCoordinate<float>> &uvw,
    idg::Array1D<float> &wavenumbers,
    idg::Array3D<idg::Visibility<std::complex<float>>> &visibilities,
    idg::Array2D<float> &spheroidal,
    idg::Array4D<idg::Matrix2x2<std::complex<float>>> &aterms,
    idg::Array1D<idg::Metadata> &metadata,
    idg::Array4D<std::complex<float>> &subgrids, const void *func,
    int num_threads);

void p_run_degridder_(const void *func, std::string func_name,
                      int num_threads);

void c_run_degridder_(
    int nr_subgrids, int grid_size, int subgrid_size, float image_size,
    float w_step_in_lambda, int nr_channels, int nr_stations,
    idg::Array2D<idg::UVWCoordinate<float>> &uvw,
    idg::Array1D<float> &wavenumbers,
    idg::Array3D<idg::Visibility<std::complex<float>>> &visibilities,
    idg::Array2D<float> &spheroidal,
    idg::Array4D<idg::Matrix2x2<std::complex<float>>> &aterms,
    idg::Array1D<idg::Metadata> &metadata,
    idg::Array4D<std::complex<float>> &subgrids, const void *func,
    int num_threads);

void print_benchmark();

}  // namespace hip

// ---------------------------------------------------------------------------
// MI355X runtime: kernel selection, validation and raw-pointer pipelines.
// Used by the kernel TUs, by util.cpp and by the C ABI (capi/idg_capi.cpp).
// ---------------------------------------------------------------------------
namespace idg_mi355x {

enum class Direction { kGridder = 0, kDegridder = 1 };

// Geometry of one gridder/degridder call; the 13-argument kernel ABI of the
// reference carries the same values.
struct Problem {
  int nr_subgrids = 0;
  int grid_size = 0;
  int subgrid_size = 0;
  float image_size = IMAGE_SIZE;
  float w_step_in_lambda = W_STEP;
  int nr_channels = 0;
  int nr_stations = 0;
  // gridder only: the output subgrids are their 2-D FFT (sign +1, scale 1),
  // as launch_subgrid_fft(+1, 1) after the plain gridder would make them
  // (in the kernel's epilogue where KernelChoice::fft_in_kernel, else a
  // launch_subgrid_fft after it)
  bool fft_out = false;
};

// Buffer extents used for host-side validation (element counts).
struct Extents {
  size_t uvw_rows = 0;      // UVW triplets (= visibility rows)
  size_t aterm_slots = 0;   // leading dimension of aterms (timeslots)
};

struct KernelChoice {
  // one kernel that handles every subgrid (__global__, 13-argument ABI,
  // grid = nr_subgrids): the reference's launch shape, used by the perf
  // entries and for caller-supplied kernels
  const void *func = nullptr;
  const char *name = "";
  int block = 256;
  int grid = 0;  // = nr_subgrids
  bool fft_in_kernel = false;  // Problem::fft_out done by these kernels
  int prec = 0;  // precision options of the MFMA kernels (device.hpp kPrec*)
  // The launch the device entries make instead, when parts[1] is set: one
  // kernel per subgrid class, each with the register allocation of its own
  // path.  parts[0] (kMirror; absent for odd S): grid =
  // nr_subgrids, the 13-argument ABI plus `int *queue`; it takes the
  // mirror-eligible subgrids and queues the others.  parts[1] (kGeneral): a
  // resident grid (occupancy x CUs, at most nr_subgrids), the 13 arguments
  // plus (int *queue, int nr_subgrids, int all); it takes the queued
  // subgrids (all of them with `all` set and no mirror launch).  queue:
  // device.hpp queue_ints(nr_subgrids) ints of stream-ordered workspace.
  // When no subgrid can be mirror-eligible (odd S, or w_step_in_lambda !=
  // 0), all_general is launched instead, once: grid = nr_subgrids, the
  // 13-argument ABI, one workgroup per subgrid on the general path.
  enum Kind { kPlain = 0, kMirror = 1, kGeneral = 2 };
  struct Part {
    const void *func = nullptr;
    int block = 0;
    int kind = kPlain;
    int per_subgrid = 1;  // workgroups per subgrid (mirror part: grid x;
                          // 0: a persistent mirror kernel, resident grid)
  } parts[2], all_general;
};

// The two-kernel launch of `k` (k.parts[1].func set) on `stream`; args13 is
// the 13-argument kernel ABI.  all_general: no subgrid can be
// mirror-eligible (w_step_in_lambda != 0), so the mirror launch is skipped.
hipError_t launch_parts(const KernelChoice &k, int nr_subgrids, void **args13,
                        bool all_general, hipStream_t stream);

// A device workspace cached per (device, stream, slot) (util.cpp), leased
// for the enqueueing of one launch sequence on `stream`: ptr holds at least
// the bytes asked for; `clean` = the last lease of this slot ended with
// leave_clean set (its contents are what that sequence left).  While another
// host thread holds the slot, ptr is a private stream-ordered allocation
// (never clean) freed after the sequence.
constexpr int kWorkspaceQueue = 0, kWorkspaceHomeSort = 1,
              kWorkspaceAdderSeg = 2;
// Not copyable: a copy would release the slot twice.
struct WorkspaceLease {
  void *ptr = nullptr;
  hipStream_t stream = nullptr;
  bool clean = false;
  bool leave_clean = false;
  WorkspaceLease() = default;
  WorkspaceLease(const WorkspaceLease &) = delete;
  WorkspaceLease &operator=(const WorkspaceLease &) = delete;
  hipError_t acquire(hipStream_t s, int slot, size_t bytes);
  ~WorkspaceLease();

 private:
  int dev_ = 0, slot_ = 0;
  bool private_ = false;
};

// Frees the cached workspaces of `stream` on the current device (all = true:
// of every stream of the current device).  The stream(s) must be idle: call
// it before destroying a stream the entries have used (a new stream may get
// the same handle) and before hipDeviceReset.  A slot leased at the moment
// (another host thread enqueueing on it) is left alone and reported as
// hipErrorNotReady.  idg_release_workspaces in the C ABI.
hipError_t release_workspaces(hipStream_t stream, bool all);

// Whether the device entries launch the two-kernel form (mirror kernel +
// queue-fed general kernel) or the one combined kernel: the two-kernel form
// from kTwoKernelMinLaunch subgrids up.  Below that (the N >= 4 shards of
// the batch) its fixed cost -- the queue's allocation and clear and a second
// launch, ~15 us per direction -- outweighs what the mirror kernel's own
// register allocation saves (one-GPU shard rehearsal at N = 8: 0.953 with
// it, 0.969 without).  IDG_KERNEL_FORM=combined / split forces either (A/B
// and tests; read per call).
constexpr int kTwoKernelMinLaunch = 8192;
bool two_kernel_form(int nr_subgrids);

// Precision options (device.hpp kPrecTail | kPrecFlush | kPrecTailAlt) of
// the MFMA kernels for a launch: the gridder takes
// the reduction tail on every phasor (kPrecTail; round 6, was kPrecTailAlt,
// one channel per quad, until channel-incoherent data showed it losing to the
// reference's own f32 sum) and, above
// kTailMinChannels channels, blocked summation (kPrecFlush: C = 256 gridder
// 8.4e-6 -> 2.0e-6 from exact accumulation); the degridder no tail.
// IDG_PREC=<0..7> forces the bits for both directions (A/B, tests).
constexpr int kTailMinChannels = 16;
int precision_for(Direction dir, const Problem &p);

// Defined in the kernel TUs.
KernelChoice select_gridder(const Problem &p);
KernelChoice select_degridder(const Problem &p);

// The order-preserving kernels (kernels/sequential_mi355x.hip.cpp): the
// reference CPU path's rounding sequence, bit for bit; 13-argument ABI, grid
// = nr_subgrids, block = sequential_block().  Selected per call by
// IDG_GRIDDER_IMPL=sequential / IDG_DEGRIDDER_IMPL=sequential.
const void *sequential_gridder(int subgrid_size);
const void *sequential_degridder(int subgrid_size);
int sequential_block();

// Returns an empty string if every subgrid's time range, stations and A-term
// slot lie inside the buffers, else a description of the first violation.
std::string validate(const Problem &p, const Extents &e,
                     const idg::Metadata *metadata);

// Asynchronous launch on device buffers (the C-ABI idg_*_launch path).
// `force` launches a caller-supplied 13-argument kernel instead of the
// selected one (the func/num_threads arguments of c_run_gridder_).
hipError_t launch(Direction dir, const Problem &p, const void *d_uvw,
                  const float *d_wavenumbers, void *d_visibilities,
                  const float *d_spheroidal, const void *d_aterms,
                  const void *d_metadata, void *d_subgrids,
                  hipStream_t stream, const KernelChoice *force = nullptr);

// Synchronous host-buffer pipeline: validate, allocate, H2D, launch, D2H,
// free.  Returns hipSuccess or the first error; *msg explains validation
// failures.
hipError_t run_host(Direction dir, const Problem &p, const Extents &e,
                    const void *uvw, const float *wavenumbers,
                    void *visibilities, const float *spheroidal,
                    const void *aterms, const idg::Metadata *metadata,
                    void *subgrids, std::string *msg,
                    const KernelChoice *force = nullptr);

// Chunk plan of run_host: subgrid bounds (nchunk + 1 entries) of
// consecutive chunks whose visibility rows are disjoint and ascending, and
// each chunk's merged row runs; one chunk when they are not.  `moved` =
// bytes of visibilities + subgrids.  Returns the chunk count.
int plan_host_chunks(const idg::Metadata *metadata, int nr_subgrids,
                     size_t moved, std::vector<int> *bounds,
                     std::vector<std::vector<std::pair<long long, long long>>>
                         *row_runs);

// Workgroups of `func` (block threads) resident on the current device at
// once: occupancy x CUs, cached per (device, kernel); 0 if the query fails.
int resident_workgroups(const void *func, int block);

// Pipeline steps (kernels/pipeline_mi355x.hip.cpp; include/idg_mi355x.h).
hipError_t launch_subgrid_fft(int nr_subgrids, int subgrid_size, int sign,
                              float scale, void *d_subgrids,
                              hipStream_t stream);
hipError_t launch_adder(int nr_subgrids, int grid_size, int subgrid_size,
                        int nr_w_layers, const void *d_metadata,
                        const void *d_subgrids, void *d_grid,
                        hipStream_t stream);
hipError_t launch_splitter(int nr_subgrids, int grid_size, int subgrid_size,
                           int nr_w_layers, const void *d_metadata,
                           const void *d_grid, void *d_subgrids,
                           hipStream_t stream);
// launch_splitter then launch_subgrid_fft(-1, 1/S^2), fused for S = 32/64
hipError_t launch_splitter_fft(int nr_subgrids, int grid_size,
                               int subgrid_size, int nr_w_layers,
                               const void *d_metadata, const void *d_grid,
                               void *d_subgrids, hipStream_t stream);

// Perf entry shared by p_run_gridder_/p_run_degridder_: env-configured
// problem, synthetic inputs, timed launches.  Returns seconds per launch.
double run_performance(Direction dir, const void *func, std::string name,
                       int num_threads);

}  // namespace idg_mi355x
