// lib-cpu.hpp -- the CPU reference entry points the harness compares against.
//
// TEST INFRASTRUCTURE.  Same declarations as the reference's app/lib-cpu.hpp:
// 9-29; implemented (cpu_oracle.cpp) on top of the plain-C oracle in
// oracle/idg_oracle.c.  (cpu::c_run_vadd is declared but never defined in the
// reference and is not carried over.)
#pragma once

#include "lib-common.hpp"

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
    idg::Array4D<std::complex<float>> &subgrids);

void c_run_degridder_reference(
    int nr_subgrids, int grid_size, int subgrid_size, float image_size,
    float w_step_in_lambda, int nr_channels, int nr_stations,
    idg::Array2D<idg::UVWCoordinate<float>> &uvw,
    idg::Array1D<float> &wavenumbers,
    idg::Array3D<idg::Visibility<std::complex<float>>> &visibilities,
    idg::Array2D<float> &spheroidal,
    idg::Array4D<idg::Matrix2x2<std::complex<float>>> &aterms,
    idg::Array1D<idg::Metadata> &metadata,
    idg::Array4D<std::complex<float>> &subgrids);

}  // namespace cpu
