// ref_shim.cpp -- extern "C" shim over the REFERENCE's own CPU path.
//
// TEST INFRASTRUCTURE ONLY.  Compiled (oracle/Makefile) together with the
// reference sources where they lie under /root/reference -- nothing of the
// reference is copied into this repository -- into oracle/_ref/libidgref*.so.
// Used to (1) generate the golden vectors in tests/golden/ and (2) time the
// reference CPU path as bench.py's cpu_baseline ("kind": "reference").
//
// It reproduces exactly what the reference harness does in run_correctness
// (tests/gridder_common.cpp:43-124, tests/degridder_common.cpp:43-124):
// srand(0), the initialize_* calls in the harness order, then
// cpu::c_run_{gridder,degridder}_reference.
#include <cstdlib>

#include "lib-cpu.hpp"

namespace {
using UVW = idg::UVWCoordinate<float>;
using Vis = idg::Visibility<std::complex<float>>;
using Jones = idg::Matrix2x2<std::complex<float>>;
using Cplx = std::complex<float>;
}  // namespace

extern "C" {

// Buffers are caller-allocated with the sizes implied by the parameters
// (nr_subgrids = nr_stations*(nr_stations-1)/2 * nr_timeslots).
int ref_generate(int nr_stations, int nr_timeslots, int nr_timesteps,
                 int nr_channels, int grid_size, int subgrid_size, float *uvw,
                 float *frequencies, float *wavenumbers, float *visibilities,
                 float *spheroidal, float *aterms, void *metadata,
                 float *subgrids) {
  const int nr_baselines = (nr_stations * (nr_stations - 1)) / 2;
  const int nr_subgrids = nr_baselines * nr_timeslots;
  idg::Array2D<UVW> a_uvw(reinterpret_cast<UVW *>(uvw), nr_subgrids,
                          nr_timesteps);
  idg::Array1D<float> a_freq(frequencies, nr_channels);
  idg::Array1D<float> a_wn(wavenumbers, nr_channels);
  idg::Array3D<Vis> a_vis(reinterpret_cast<Vis *>(visibilities), nr_subgrids,
                          nr_timesteps, nr_channels);
  idg::Array1D<idg::Baseline> a_bl(nr_baselines);
  idg::Array2D<float> a_sph(spheroidal, subgrid_size, subgrid_size);
  idg::Array4D<Jones> a_at(reinterpret_cast<Jones *>(aterms), nr_timeslots,
                           nr_stations, subgrid_size, subgrid_size);
  idg::Array4D<Cplx> a_sg(reinterpret_cast<Cplx *>(subgrids), nr_subgrids, 4,
                          subgrid_size, subgrid_size);
  idg::Array1D<idg::Metadata> a_md(static_cast<idg::Metadata *>(metadata),
                                   nr_subgrids);
  srand(0);
  initialize_uvw(grid_size, a_uvw);
  initialize_frequencies(a_freq);
  initialize_wavenumbers(a_freq, a_wn);
  initialize_visibilities(grid_size, IMAGE_SIZE, a_freq, a_uvw, a_vis);
  initialize_baselines(nr_stations, a_bl);
  initialize_spheroidal(a_sph);
  initialize_aterms(a_sph, a_at);
  initialize_subgrids(a_sg);
  initialize_metadata(grid_size, nr_timeslots, nr_timesteps, a_bl, a_md);
  return nr_subgrids;
}

// The reference kernels only ever call .data() on the arrays, so the
// non-owning views below only need the right base pointers.
void ref_gridder(int nr_subgrids, int grid_size, int subgrid_size,
                 float image_size, float w_step_in_lambda, int nr_channels,
                 int nr_stations, const float *uvw, const float *wavenumbers,
                 const float *visibilities, const float *spheroidal,
                 const float *aterms, const void *metadata, float *subgrids) {
  idg::Array2D<UVW> a_uvw((UVW *)uvw, 1, 1);
  idg::Array1D<float> a_wn((float *)wavenumbers, nr_channels);
  idg::Array3D<Vis> a_vis((Vis *)visibilities, 1, 1, 1);
  idg::Array2D<float> a_sph((float *)spheroidal, subgrid_size, subgrid_size);
  idg::Array4D<Jones> a_at((Jones *)aterms, 1, 1, 1, 1);
  idg::Array1D<idg::Metadata> a_md((idg::Metadata *)metadata, nr_subgrids);
  idg::Array4D<Cplx> a_sg((Cplx *)subgrids, nr_subgrids, 4, subgrid_size,
                          subgrid_size);
  cpu::c_run_gridder_reference(nr_subgrids, grid_size, subgrid_size,
                               image_size, w_step_in_lambda, nr_channels,
                               nr_stations, a_uvw, a_wn, a_vis, a_sph, a_at,
                               a_md, a_sg);
}

void ref_degridder(int nr_subgrids, int grid_size, int subgrid_size,
                   float image_size, float w_step_in_lambda, int nr_channels,
                   int nr_stations, const float *uvw, const float *wavenumbers,
                   float *visibilities, const float *spheroidal,
                   const float *aterms, const void *metadata,
                   const float *subgrids) {
  idg::Array2D<UVW> a_uvw((UVW *)uvw, 1, 1);
  idg::Array1D<float> a_wn((float *)wavenumbers, nr_channels);
  idg::Array3D<Vis> a_vis((Vis *)visibilities, 1, 1, 1);
  idg::Array2D<float> a_sph((float *)spheroidal, subgrid_size, subgrid_size);
  idg::Array4D<Jones> a_at((Jones *)aterms, 1, 1, 1, 1);
  idg::Array1D<idg::Metadata> a_md((idg::Metadata *)metadata, nr_subgrids);
  idg::Array4D<Cplx> a_sg((Cplx *)subgrids, nr_subgrids, 4, subgrid_size,
                          subgrid_size);
  cpu::c_run_degridder_reference(nr_subgrids, grid_size, subgrid_size,
                                 image_size, w_step_in_lambda, nr_channels,
                                 nr_stations, a_uvw, a_wn, a_vis, a_sph, a_at,
                                 a_md, a_sg);
}

float ref_image_size(void) { return IMAGE_SIZE; }
float ref_w_step(void) { return W_STEP; }

}  // extern "C"
