// idg_capi.cpp -- the extern "C" boundary (include/idg_mi355x.h).
#include "idg_mi355x.h"

#include <hip/hip_runtime.h>

#include <cstdio>
#include <algorithm>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "hip/util.hpp"
#include "lib-hip.hpp"

static_assert(sizeof(idg_metadata_t) == sizeof(idg::Metadata),
              "metadata layout");
static_assert(sizeof(idg_uvw_t) == sizeof(idg::UVWCoordinate<float>),
              "uvw layout");

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string &msg) {
  g_last_error = msg;
  return code;
}

int from_hip(hipError_t e, const char *what) {
  if (e == hipSuccess) return IDG_OK;
  return fail(static_cast<int>(e),
              std::string(what) + ": " + hipGetErrorString(e));
}

idg_mi355x::Problem make_problem(int nr_subgrids, int grid_size,
                                 int subgrid_size, float image_size,
                                 float w_step, int nr_channels,
                                 int nr_stations) {
  idg_mi355x::Problem p;
  p.nr_subgrids = nr_subgrids;
  p.grid_size = grid_size;
  p.subgrid_size = subgrid_size;
  p.image_size = image_size;
  p.w_step_in_lambda = w_step;
  p.nr_channels = nr_channels;
  p.nr_stations = nr_stations;
  return p;
}

int check_geometry(const idg_mi355x::Problem &p) {
  if (p.nr_subgrids < 0 || p.subgrid_size <= 0 || p.nr_channels <= 0 ||
      p.nr_stations <= 0)
    return fail(IDG_E_INVALID_ARGUMENT,
                "nr_subgrids >= 0, subgrid_size, nr_channels, nr_stations > 0 "
                "required");
  return IDG_OK;
}

int run_host(idg_mi355x::Direction dir, const idg_mi355x::Problem &p,
             size_t uvw_rows, size_t aterm_slots, const void *uvw,
             const float *wn, void *vis, const float *sph, const void *at,
             const idg_metadata_t *md, void *sg) {
  if (int rc = check_geometry(p)) return rc;
  if (p.nr_subgrids == 0) return IDG_OK;
  if (!uvw || !wn || !vis || !sph || !at || !md || !sg)
    return fail(IDG_E_INVALID_ARGUMENT, "null buffer");
  idg_mi355x::Extents e;
  e.uvw_rows = uvw_rows;
  e.aterm_slots = aterm_slots;
  std::string msg;
  const hipError_t err = idg_mi355x::run_host(
      dir, p, e, uvw, wn, vis, sph, at,
      reinterpret_cast<const idg::Metadata *>(md), sg, &msg);
  if (!msg.empty()) return fail(IDG_E_OUT_OF_BOUNDS, msg);
  return from_hip(err, dir == idg_mi355x::Direction::kGridder
                           ? "idg_c_run_gridder"
                           : "idg_c_run_degridder");
}

int launch(idg_mi355x::Direction dir, const idg_mi355x::Problem &p,
           const void *uvw, const float *wn, void *vis, const float *sph,
           const void *at, const void *md, void *sg, void *stream) {
  if (int rc = check_geometry(p)) return rc;
  if (p.nr_subgrids == 0) return IDG_OK;
  if (!uvw || !wn || !vis || !sph || !at || !md || !sg)
    return fail(IDG_E_INVALID_ARGUMENT, "null buffer");
  return from_hip(
      idg_mi355x::launch(dir, p, uvw, wn, vis, sph, at, md, sg,
                         static_cast<hipStream_t>(stream)),
      "hipLaunchKernel");
}

}  // namespace

extern "C" {

int idg_abi_version(void) { return IDG_MI355X_ABI_VERSION; }

const char *idg_last_error(void) { return g_last_error.c_str(); }

int idg_release_workspaces(void *stream, int all) {
  return from_hip(idg_mi355x::release_workspaces(
                      static_cast<hipStream_t>(stream), all != 0),
                  "idg_release_workspaces");
}

int idg_subgrid_fft_launch(int nr_subgrids, int subgrid_size, int sign,
                           float scale, idg_cfloat_t *subgrids, void *stream) {
  if (nr_subgrids < 0 || subgrid_size <= 0 || subgrid_size > 64 ||
      (sign != 1 && sign != -1))
    return fail(IDG_E_INVALID_ARGUMENT,
                "nr_subgrids >= 0, 0 < subgrid_size <= 64, sign = +1 or -1");
  return from_hip(idg_mi355x::launch_subgrid_fft(
                      nr_subgrids, subgrid_size, sign, scale, subgrids,
                      static_cast<hipStream_t>(stream)),
                  "idg_subgrid_fft_launch");
}

int idg_adder_launch(int nr_subgrids, int grid_size, int subgrid_size,
                     int nr_w_layers, const idg_metadata_t *metadata,
                     const idg_cfloat_t *subgrids, idg_cfloat_t *grid,
                     void *stream) {
  if (nr_subgrids < 0 || subgrid_size <= 0 || subgrid_size % 2 ||
      grid_size < subgrid_size || nr_w_layers <= 0)
    return fail(IDG_E_INVALID_ARGUMENT,
                "even subgrid_size <= grid_size, nr_w_layers > 0 required");
  return from_hip(idg_mi355x::launch_adder(
                      nr_subgrids, grid_size, subgrid_size, nr_w_layers,
                      metadata, subgrids, grid,
                      static_cast<hipStream_t>(stream)),
                  "idg_adder_launch");
}

int idg_splitter_launch(int nr_subgrids, int grid_size, int subgrid_size,
                        int nr_w_layers, const idg_metadata_t *metadata,
                        const idg_cfloat_t *grid, idg_cfloat_t *subgrids,
                        void *stream) {
  if (nr_subgrids < 0 || subgrid_size <= 0 || subgrid_size % 2 ||
      grid_size < subgrid_size || nr_w_layers <= 0)
    return fail(IDG_E_INVALID_ARGUMENT,
                "even subgrid_size <= grid_size, nr_w_layers > 0 required");
  return from_hip(idg_mi355x::launch_splitter(
                      nr_subgrids, grid_size, subgrid_size, nr_w_layers,
                      metadata, grid, subgrids,
                      static_cast<hipStream_t>(stream)),
                  "idg_splitter_launch");
}

int idg_splitter_fft_launch(int nr_subgrids, int grid_size, int subgrid_size,
                            int nr_w_layers, const idg_metadata_t *metadata,
                            const idg_cfloat_t *grid, idg_cfloat_t *subgrids,
                            void *stream) {
  if (nr_subgrids < 0 || subgrid_size <= 0 || subgrid_size % 2 ||
      subgrid_size > 64 || grid_size < subgrid_size || nr_w_layers <= 0)
    return fail(IDG_E_INVALID_ARGUMENT,
                "even subgrid_size <= min(64, grid_size), nr_w_layers > 0 "
                "required");
  return from_hip(idg_mi355x::launch_splitter_fft(
                      nr_subgrids, grid_size, subgrid_size, nr_w_layers,
                      metadata, grid, subgrids,
                      static_cast<hipStream_t>(stream)),
                  "idg_splitter_fft_launch");
}

int idg_c_run_gridder(int nr_subgrids, int grid_size, int subgrid_size,
                      float image_size, float w_step_in_lambda,
                      int nr_channels, int nr_stations, const idg_uvw_t *uvw,
                      size_t uvw_rows, const float *wavenumbers,
                      const idg_cfloat_t *visibilities,
                      const float *spheroidal, const idg_cfloat_t *aterms,
                      size_t aterm_slots, const idg_metadata_t *metadata,
                      idg_cfloat_t *subgrids) {
  const auto p = make_problem(nr_subgrids, grid_size, subgrid_size,
                              image_size, w_step_in_lambda, nr_channels,
                              nr_stations);
  return run_host(idg_mi355x::Direction::kGridder, p, uvw_rows, aterm_slots,
                  uvw, wavenumbers, const_cast<idg_cfloat_t *>(visibilities),
                  spheroidal, aterms, metadata, subgrids);
}

int idg_c_run_degridder(int nr_subgrids, int grid_size, int subgrid_size,
                        float image_size, float w_step_in_lambda,
                        int nr_channels, int nr_stations,
                        const idg_uvw_t *uvw, size_t uvw_rows,
                        const float *wavenumbers, idg_cfloat_t *visibilities,
                        const float *spheroidal, const idg_cfloat_t *aterms,
                        size_t aterm_slots, const idg_metadata_t *metadata,
                        const idg_cfloat_t *subgrids) {
  const auto p = make_problem(nr_subgrids, grid_size, subgrid_size,
                              image_size, w_step_in_lambda, nr_channels,
                              nr_stations);
  return run_host(idg_mi355x::Direction::kDegridder, p, uvw_rows,
                  aterm_slots, uvw, wavenumbers, visibilities, spheroidal,
                  aterms, metadata, const_cast<idg_cfloat_t *>(subgrids));
}

int idg_gridder_launch(int nr_subgrids, int grid_size, int subgrid_size,
                       float image_size, float w_step_in_lambda,
                       int nr_channels, int nr_stations, const idg_uvw_t *uvw,
                       const float *wavenumbers,
                       const idg_cfloat_t *visibilities,
                       const float *spheroidal, const idg_cfloat_t *aterms,
                       const idg_metadata_t *metadata, idg_cfloat_t *subgrids,
                       void *stream) {
  const auto p = make_problem(nr_subgrids, grid_size, subgrid_size,
                              image_size, w_step_in_lambda, nr_channels,
                              nr_stations);
  return launch(idg_mi355x::Direction::kGridder, p, uvw, wavenumbers,
                const_cast<idg_cfloat_t *>(visibilities), spheroidal, aterms,
                metadata, subgrids, stream);
}

int idg_gridder_fft_launch(int nr_subgrids, int grid_size, int subgrid_size,
                           float image_size, float w_step_in_lambda,
                           int nr_channels, int nr_stations,
                           const idg_uvw_t *uvw, const float *wavenumbers,
                           const idg_cfloat_t *visibilities,
                           const float *spheroidal, const idg_cfloat_t *aterms,
                           const idg_metadata_t *metadata,
                           idg_cfloat_t *subgrids, void *stream) {
  if (subgrid_size > 64)
    return fail(IDG_E_INVALID_ARGUMENT,
                "idg_gridder_fft_launch: subgrid_size <= 64 (the FFT's)");
  auto p = make_problem(nr_subgrids, grid_size, subgrid_size, image_size,
                        w_step_in_lambda, nr_channels, nr_stations);
  p.fft_out = true;
  return launch(idg_mi355x::Direction::kGridder, p, uvw, wavenumbers,
                const_cast<idg_cfloat_t *>(visibilities), spheroidal, aterms,
                metadata, subgrids, stream);
}

int idg_degridder_launch(int nr_subgrids, int grid_size, int subgrid_size,
                         float image_size, float w_step_in_lambda,
                         int nr_channels, int nr_stations,
                         const idg_uvw_t *uvw, const float *wavenumbers,
                         idg_cfloat_t *visibilities, const float *spheroidal,
                         const idg_cfloat_t *aterms,
                         const idg_metadata_t *metadata,
                         const idg_cfloat_t *subgrids, void *stream) {
  const auto p = make_problem(nr_subgrids, grid_size, subgrid_size,
                              image_size, w_step_in_lambda, nr_channels,
                              nr_stations);
  return launch(idg_mi355x::Direction::kDegridder, p, uvw, wavenumbers,
                visibilities, spheroidal, aterms, metadata,
                const_cast<idg_cfloat_t *>(subgrids), stream);
}

int idg_validate_metadata(int nr_subgrids, int subgrid_size, int nr_channels,
                          int nr_stations, size_t uvw_rows, size_t aterm_slots,
                          const idg_metadata_t *metadata) {
  idg_mi355x::Problem p;
  p.nr_subgrids = nr_subgrids;
  p.subgrid_size = subgrid_size;
  p.nr_channels = nr_channels;
  p.nr_stations = nr_stations;
  if (int rc = check_geometry(p)) return rc;
  idg_mi355x::Extents e;
  e.uvw_rows = uvw_rows;
  e.aterm_slots = aterm_slots;
  const std::string msg = idg_mi355x::validate(
      p, e, reinterpret_cast<const idg::Metadata *>(metadata));
  if (!msg.empty()) return fail(IDG_E_OUT_OF_BOUNDS, msg);
  return IDG_OK;
}

int idg_host_chunk_plan(int nr_subgrids, const idg_metadata_t *metadata,
                        size_t bytes_moved, int *bounds, int max_bounds) {
  if (nr_subgrids <= 0 || metadata == nullptr)
    return fail(IDG_E_INVALID_ARGUMENT, "nr_subgrids <= 0 or null metadata");
  std::vector<int> sb;
  const int n = idg_mi355x::plan_host_chunks(
      reinterpret_cast<const idg::Metadata *>(metadata), nr_subgrids,
      bytes_moved, &sb, nullptr);
  if (bounds)
    for (int i = 0; i < static_cast<int>(sb.size()) && i < max_bounds; ++i)
      bounds[i] = sb[i];
  return n;
}

const char *idg_kernel_name(int direction, int subgrid_size, int nr_channels) {
  idg_mi355x::Problem p;
  p.subgrid_size = subgrid_size;
  p.nr_channels = nr_channels;
  return direction == 0 ? idg_mi355x::select_gridder(p).name
                        : idg_mi355x::select_degridder(p).name;
}

int idg_precision_options(int direction, int subgrid_size, int nr_channels) {
  idg_mi355x::Problem p;
  p.subgrid_size = subgrid_size;
  p.nr_channels = nr_channels;
  return direction == 0 ? idg_mi355x::select_gridder(p).prec
                        : idg_mi355x::select_degridder(p).prec;
}

double idg_p_run_gridder(void) {
  idg_mi355x::Problem p;
  p.subgrid_size = static_cast<int>(get_env_var("SUBGRID_SIZE", 32));
  p.nr_channels = static_cast<int>(get_env_var("NR_CHANNELS", 16));
  const auto k = idg_mi355x::select_gridder(p);
  return 1e3 * idg_mi355x::run_performance(idg_mi355x::Direction::kGridder,
                                           k.func, "gridder_mi355x", k.block);
}

double idg_p_run_degridder(void) {
  idg_mi355x::Problem p;
  p.subgrid_size = static_cast<int>(get_env_var("SUBGRID_SIZE", 32));
  p.nr_channels = static_cast<int>(get_env_var("NR_CHANNELS", 16));
  // the batch run_performance builds (the kernel choice depends on its size)
  const int nr_stations = static_cast<int>(get_env_var("NR_STATIONS", 50));
  p.nr_subgrids = nr_stations * (nr_stations - 1) / 2 *
                  static_cast<int>(get_env_var("NR_TIMESLOTS", 20));
  const auto k = idg_mi355x::select_degridder(p);
  return 1e3 * idg_mi355x::run_performance(idg_mi355x::Direction::kDegridder,
                                           k.func, "degridder_mi355x",
                                           k.block);
}

void idg_print_device_info(void) { hip::print_device_info(); }
void idg_print_benchmark(void) { hip::print_benchmark(); }

int idg_get_device_name(char *buf, size_t len) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
    return fail(IDG_E_NO_DEVICE, "no HIP device");
  const std::string name = hip::extern_get_device_name();
  if (buf && len) {
    std::strncpy(buf, name.c_str(), len - 1);
    buf[len - 1] = '\0';
  }
  return static_cast<int>(name.size());
}

uint64_t idg_flops_gridder(uint64_t nr_channels, uint64_t nr_timesteps,
                           uint64_t nr_subgrids, uint64_t subgrid_size,
                           uint64_t nr_correlations) {
  return flops_gridder(nr_channels, nr_timesteps, nr_subgrids, subgrid_size,
                       nr_correlations);
}

uint64_t idg_bytes_gridder(uint64_t nr_channels, uint64_t nr_timesteps,
                           uint64_t nr_subgrids, uint64_t subgrid_size,
                           uint64_t nr_correlations) {
  return bytes_gridder(nr_channels, nr_timesteps, nr_subgrids, subgrid_size,
                       nr_correlations);
}

int idg_generate(int nr_stations, int nr_timeslots, int nr_timesteps,
                 int nr_channels, int grid_size, int subgrid_size,
                 idg_uvw_t *uvw, float *frequencies, float *wavenumbers,
                 idg_cfloat_t *visibilities, float *spheroidal,
                 idg_cfloat_t *aterms, idg_metadata_t *metadata,
                 idg_cfloat_t *subgrids, int nthreads) {
  if (nr_stations < 2 || nr_timeslots < 1 || nr_timesteps < 1 ||
      nr_channels < 1 || grid_size < 1 || subgrid_size < 1)
    return fail(IDG_E_INVALID_ARGUMENT, "idg_generate: bad parameters");
  using UVW = idg::UVWCoordinate<float>;
  using Vis = idg::Visibility<std::complex<float>>;
  using Jones = idg::Matrix2x2<std::complex<float>>;
  const int nbl = nr_stations * (nr_stations - 1) / 2;
  const int ns = nbl * nr_timeslots;
  const size_t S = static_cast<size_t>(subgrid_size);
  // Caller buffers where given, owned temporaries otherwise (every generator
  // still runs, so the rand() stream is consumed exactly as the harness does).
  std::vector<UVW> t_uvw(uvw ? 0 : static_cast<size_t>(ns) * nr_timesteps);
  std::vector<float> t_f(frequencies ? 0 : nr_channels),
      t_wn(wavenumbers ? 0 : nr_channels), t_sph(spheroidal ? 0 : S * S);
  std::vector<Jones> t_at(aterms ? 0 : nr_timeslots * nr_stations * S * S);
  std::vector<idg::Metadata> t_md(metadata ? 0 : ns);
  UVW *p_uvw = uvw ? reinterpret_cast<UVW *>(uvw) : t_uvw.data();
  float *p_f = frequencies ? frequencies : t_f.data();
  float *p_wn = wavenumbers ? wavenumbers : t_wn.data();
  float *p_sph = spheroidal ? spheroidal : t_sph.data();
  Jones *p_at = aterms ? reinterpret_cast<Jones *>(aterms) : t_at.data();
  idg::Metadata *p_md =
      metadata ? reinterpret_cast<idg::Metadata *>(metadata) : t_md.data();

  idg::Array2D<UVW> a_uvw(p_uvw, ns, nr_timesteps);
  idg::Array1D<float> a_f(p_f, nr_channels), a_wn(p_wn, nr_channels);
  idg::Array1D<idg::Baseline> a_bl(nbl);
  idg::Array2D<float> a_sph(p_sph, subgrid_size, subgrid_size);
  idg::Array4D<Jones> a_at(p_at, nr_timeslots, nr_stations, subgrid_size,
                           subgrid_size);
  idg::Array1D<idg::Metadata> a_md(p_md, ns);

  srand(0);
  initialize_uvw(grid_size, a_uvw);
  initialize_frequencies(a_f);
  initialize_wavenumbers(a_f, a_wn);
  if (visibilities) {
    // Row-parallel: this generator draws no random numbers.
    const int nt = std::max(1, std::min(nthreads, ns));
    std::vector<std::thread> pool;
    for (int w = 0; w < nt; ++w) {
      const int r0 = static_cast<int>(static_cast<long long>(ns) * w / nt);
      const int r1 = static_cast<int>(static_cast<long long>(ns) * (w + 1) / nt);
      if (r1 <= r0) continue;
      pool.emplace_back([&a_f, p_uvw, visibilities, grid_size, nr_timesteps,
                         nr_channels, r0, r1]() {
        idg::Array2D<UVW> u(p_uvw + static_cast<size_t>(r0) * nr_timesteps,
                            r1 - r0, nr_timesteps);
        idg::Array3D<Vis> v(
            reinterpret_cast<Vis *>(visibilities) +
                static_cast<size_t>(r0) * nr_timesteps * nr_channels,
            r1 - r0, nr_timesteps, nr_channels);
        initialize_visibilities(grid_size, IMAGE_SIZE, a_f, u, v);
      });
    }
    for (auto &th : pool) th.join();
  }
  initialize_baselines(nr_stations, a_bl);
  initialize_spheroidal(a_sph);
  initialize_aterms(a_sph, a_at);
  if (subgrids) {
    idg::Array4D<std::complex<float>> a_sg(
        reinterpret_cast<std::complex<float> *>(subgrids), ns, 4,
        subgrid_size, subgrid_size);
    initialize_subgrids(a_sg);
  }
  initialize_metadata(grid_size, nr_timeslots, nr_timesteps, a_bl, a_md);
  return ns;
}

}  // extern "C"
