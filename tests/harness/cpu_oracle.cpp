// cpu_oracle.cpp -- cpu::c_run_*_reference over the C oracle.
// TEST INFRASTRUCTURE (see lib-cpu.hpp).
#include <cstdlib>

#include "idg_oracle.h"
#include "lib-cpu.hpp"

namespace {
int oracle_threads() {
  const char *v = std::getenv("IDG_ORACLE_THREADS");
  return v ? std::atoi(v) : 1;
}
}  // namespace

namespace cpu {

void c_run_gridder_reference(
    int nr_subgrids, int grid_size, int subgrid_size, float image_size,
    float w_step_in_lambda, int nr_channels, int nr_stations,
    idg::Array2D<idg::UVWCoordinate<float>> &uvw,
    idg::Array1D<float> &wavenumbers,
    idg::Array3D<idg::Visibility<std::complex<float>>> &visibilities,
    idg::Array2D<float> &spheroidal,
    idg::Array4D<idg::Matrix2x2<std::complex<float>>> &aterms,
    idg::Array1D<idg::Metadata> &metadata,
    idg::Array4D<std::complex<float>> &subgrids) {
  oracle_gridder(nr_subgrids, grid_size, subgrid_size, image_size,
                 w_step_in_lambda, nr_channels, nr_stations,
                 reinterpret_cast<const float *>(uvw.data()),
                 wavenumbers.data(),
                 reinterpret_cast<const float *>(visibilities.data()),
                 spheroidal.data(),
                 reinterpret_cast<const float *>(aterms.data()),
                 reinterpret_cast<const oracle_metadata *>(metadata.data()),
                 reinterpret_cast<float *>(subgrids.data()), oracle_threads());
}

void c_run_degridder_reference(
    int nr_subgrids, int grid_size, int subgrid_size, float image_size,
    float w_step_in_lambda, int nr_channels, int nr_stations,
    idg::Array2D<idg::UVWCoordinate<float>> &uvw,
    idg::Array1D<float> &wavenumbers,
    idg::Array3D<idg::Visibility<std::complex<float>>> &visibilities,
    idg::Array2D<float> &spheroidal,
    idg::Array4D<idg::Matrix2x2<std::complex<float>>> &aterms,
    idg::Array1D<idg::Metadata> &metadata,
    idg::Array4D<std::complex<float>> &subgrids) {
  oracle_degridder(nr_subgrids, grid_size, subgrid_size, image_size,
                   w_step_in_lambda, nr_channels, nr_stations,
                   reinterpret_cast<const float *>(uvw.data()),
                   wavenumbers.data(),
                   reinterpret_cast<float *>(visibilities.data()),
                   spheroidal.data(),
                   reinterpret_cast<const float *>(aterms.data()),
                   reinterpret_cast<const oracle_metadata *>(metadata.data()),
                   reinterpret_cast<const float *>(subgrids.data()),
                   oracle_threads());
}

}  // namespace cpu
