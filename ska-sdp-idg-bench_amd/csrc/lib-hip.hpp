// lib-hip.hpp -- public C++ API of the MI355X HIP backend.
//
// Same namespace and entry points as the reference's app/lib-hip.hpp:5-9, so
// the reference harness (tests/gridder_common.cpp, tests/degridder_common.cpp)
// compiles against it unchanged.  extern_get_device_name() is declared but
// never defined in the reference; it is defined here.
//
// The kernel translation units additionally provide (the TU contract the
// harness forward-declares, tests/gridder_common.cpp:13-31):
//   hip::p_run_gridder() / hip::c_run_gridder(...)
//   hip::p_run_degridder() / hip::c_run_degridder(...)
#pragma once

#include <string>

#include "lib-common.hpp"

namespace hip {
void print_device_info();
std::string extern_get_device_name();
void print_benchmark();

void p_run_gridder();
void c_run_gridder(
    int nr_subgrids, int grid_size, int subgrid_size, float image_size,
    float w_step_in_lambda, int nr_channels, int nr_stations,
    idg::Array2D<idg::UVWCoordinate<float>> &uvw,
    idg::Array1D<float> &wavenumbers,
    idg::Array3D<idg::Visibility<std::complex<float>>> &visibilities,
    idg::Array2D<float> &spheroidal,
    idg::Array4D<idg::Matrix2x2<std::complex<float>>> &aterms,
    idg::Array1D<idg::Metadata> &metadata,
    idg::Array4D<std::complex<float>> &subgrids);

void p_run_degridder();
void c_run_degridder(
    int nr_subgrids, int grid_size, int subgrid_size, float image_size,
    float w_step_in_lambda, int nr_channels, int nr_stations,
    idg::Array2D<idg::UVWCoordinate<float>> &uvw,
    idg::Array1D<float> &wavenumbers,
    idg::Array3D<idg::Visibility<std::complex<float>>> &visibilities,
    idg::Array2D<float> &spheroidal,
    idg::Array4D<idg::Matrix2x2<std::complex<float>>> &aterms,
    idg::Array1D<idg::Metadata> &metadata,
    idg::Array4D<std::complex<float>> &subgrids);
}  // namespace hip
