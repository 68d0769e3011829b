// idg_harness.cpp -- the hip-<kernel> executables (TEST INFRASTRUCTURE).
//
// Restates the reference's tests/gridder_common.cpp and
// tests/degridder_common.cpp (compiled twice: -DIDG_DEGRIDDER=0 builds
// hip-gridder_mi355x, -DIDG_DEGRIDDER=1 builds hip-degridder_mi355x):
//   no argument         -> run_performance(): hip::p_run_{de,}gridder()
//   argument "-c..."    -> run_correctness(): -c defaults (NR_STATIONS=2,
//                          NR_TIMESLOTS=2, ...), srand(0) + generators,
//                          CPU reference, device kernel, check_error
//   anything else       -> usage, exit 1
// Deviation (documented): -c exits 1 when the result is FAILED.
#include <cstring>
#include <iostream>

#include "lib-cpu.hpp"
#include "lib-hip.hpp"
#include "test_util.hpp"

#ifndef IDG_DEGRIDDER
#define IDG_DEGRIDDER 0
#endif

namespace {

void run_performance() {
  hip::print_device_info();
#if IDG_DEGRIDDER
  hip::p_run_degridder();
#else
  hip::p_run_gridder();
#endif
}

bool run_correctness() {
  std::cout << (IDG_DEGRIDDER ? ">>> Correctness IDG-Degridder test"
                              : ">>> Correctness IDG-Gridder test")
            << std::endl;
  hip::print_device_info();
  hip::print_benchmark();

  const int nr_correlations = static_cast<int>(get_env_var("NR_CORRELATIONS", 4));
  const int grid_size = static_cast<int>(get_env_var("GRID_SIZE", 1024));
  const int subgrid_size = static_cast<int>(get_env_var("SUBGRID_SIZE", 32));
  const int nr_stations = static_cast<int>(get_env_var("NR_STATIONS", 2));
  const int nr_timeslots = static_cast<int>(get_env_var("NR_TIMESLOTS", 2));
  const int nr_timesteps =
      static_cast<int>(get_env_var("NR_TIMESTEPS_SUBGRID", 128));
  const int nr_channels = static_cast<int>(get_env_var("NR_CHANNELS", 16));
  const int nr_baselines = nr_stations * (nr_stations - 1) / 2;
  const int nr_subgrids = nr_baselines * nr_timeslots;
  const int total_nr_timesteps = nr_subgrids * nr_timesteps;
  print_parameters(nr_stations, nr_channels, nr_timesteps, nr_correlations,
                   nr_timeslots, IMAGE_SIZE, grid_size, subgrid_size, W_STEP,
                   nr_baselines, nr_subgrids, total_nr_timesteps);

  std::cout << ">>> Allocate data structures on host" << std::endl;
  idg::Array2D<idg::UVWCoordinate<float>> uvw(nr_subgrids, nr_timesteps);
  idg::Array3D<idg::Visibility<std::complex<float>>> cpu_vis(
      nr_subgrids, nr_timesteps, nr_channels);
  idg::Array3D<idg::Visibility<std::complex<float>>> gpu_vis(
      nr_subgrids, nr_timesteps, nr_channels);
  idg::Array1D<idg::Baseline> baselines(nr_baselines);
  idg::Array4D<idg::Matrix2x2<std::complex<float>>> aterms(
      nr_timeslots, nr_stations, subgrid_size, subgrid_size);
  idg::Array1D<float> frequencies(nr_channels), wavenumbers(nr_channels);
  idg::Array2D<float> spheroidal(subgrid_size, subgrid_size);
  idg::Array4D<std::complex<float>> cpu_sg(nr_subgrids, nr_correlations,
                                           subgrid_size, subgrid_size);
  idg::Array4D<std::complex<float>> gpu_sg(nr_subgrids, nr_correlations,
                                           subgrid_size, subgrid_size);
  idg::Array1D<idg::Metadata> metadata(nr_subgrids);

  std::cout << ">>> Initialize data structures on host" << std::endl;
  srand(0);
  initialize_uvw(grid_size, uvw);
  initialize_frequencies(frequencies);
  initialize_wavenumbers(frequencies, wavenumbers);
#if !IDG_DEGRIDDER
  initialize_visibilities(grid_size, IMAGE_SIZE, frequencies, uvw, cpu_vis);
#endif
  initialize_baselines(nr_stations, baselines);
  initialize_spheroidal(spheroidal);
  initialize_aterms(spheroidal, aterms);
#if IDG_DEGRIDDER
  initialize_subgrids(cpu_sg);
#endif
  initialize_metadata(grid_size, nr_timeslots, nr_timesteps, baselines,
                      metadata);

  std::cout << ">>> Run on cpu" << std::endl;
#if IDG_DEGRIDDER
  cpu::c_run_degridder_reference(nr_subgrids, grid_size, subgrid_size,
                                 IMAGE_SIZE, W_STEP, nr_channels, nr_stations,
                                 uvw, wavenumbers, cpu_vis, spheroidal, aterms,
                                 metadata, cpu_sg);
  std::cout << ">>> Run on gpu" << std::endl;
  hip::c_run_degridder(nr_subgrids, grid_size, subgrid_size, IMAGE_SIZE,
                       W_STEP, nr_channels, nr_stations, uvw, wavenumbers,
                       gpu_vis, spheroidal, aterms, metadata, cpu_sg);
  std::cout << ">>> Checking" << std::endl;
  return compare_visibilities(cpu_vis, gpu_vis);
#else
  cpu::c_run_gridder_reference(nr_subgrids, grid_size, subgrid_size,
                               IMAGE_SIZE, W_STEP, nr_channels, nr_stations,
                               uvw, wavenumbers, cpu_vis, spheroidal, aterms,
                               metadata, cpu_sg);
  std::cout << ">>> Run on gpu" << std::endl;
  hip::c_run_gridder(nr_subgrids, grid_size, subgrid_size, IMAGE_SIZE, W_STEP,
                     nr_channels, nr_stations, uvw, wavenumbers, cpu_vis,
                     spheroidal, aterms, metadata, gpu_sg);
  std::cout << ">>> Checking" << std::endl;
  return compare_subgrids(cpu_sg, gpu_sg);
#endif
}

}  // namespace

int main(int argc, char *argv[]) {
  if (argc == 1) {
    run_performance();
    return EXIT_SUCCESS;
  }
  if (argc == 2 && std::strncmp(argv[1], "-c", 2) == 0)
    return run_correctness() ? EXIT_SUCCESS : EXIT_FAILURE;
  std::cerr << "Usage: " << argv[0] << " [-c]" << std::endl;
  return EXIT_FAILURE;
}
