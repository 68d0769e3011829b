// print.cpp -- see print.hpp.
#include "print.hpp"

#include <algorithm>
#include <iomanip>
#include <string>
#include <utility>
#include <vector>

void print_parameters(int nr_stations, int nr_channels, int nr_timesteps,
                      int nr_correlations, int nr_timeslots, float image_size,
                      int grid_size, int subgrid_size, float w_step,
                      int nr_baselines, int nr_subgrids,
                      int total_nr_timesteps) {
  format_saver keep(&std::cout);
  const std::vector<std::pair<const char *, double>> rows = {
      {"Number of stations", nr_stations},
      {"Number of channels", nr_channels},
      {"Number of timesteps", nr_timesteps},
      {"Number of correlations", nr_correlations},
      {"Number of timeslots", nr_timeslots},
      {"Imagesize", image_size},
      {"Grid size", grid_size},
      {"Subgrid size", subgrid_size},
      {"W step size", w_step},
      {"Number of baselines", nr_baselines},
      {"Number of subgrids", nr_subgrids},
      {"Total number of timesteps", total_nr_timesteps}};
  std::cout << "-----------\nPARAMETERS:\n";
  for (const auto &r : rows)
    std::cout << std::setw(30) << std::left << r.first << "== "
              << std::setw(10) << std::right << r.second << "\n";
  std::cout << "-----------" << std::endl;
}

namespace {

constexpr unsigned kMaxCorr = 4, kMaxRows = 3, kMaxCols = 3, kMaxTime = 3,
                   kMaxChan = 4;

void put(std::complex<float> v) {
  std::cout << std::setw(12) << std::setprecision(4) << std::fixed << v.real()
            << (v.imag() < 0 ? " - " : " + ") << std::setw(10)
            << std::abs(v.imag()) << "i  ";
}

}  // namespace

void print_subgrid(idg::Array4D<std::complex<float>> &sg, unsigned i) {
  format_saver keep(&std::cout);
  const unsigned nc = std::min<unsigned>(sg.get_z_dim(), kMaxCorr);
  const unsigned ny = std::min<unsigned>(sg.get_y_dim(), kMaxRows);
  const unsigned nx = std::min<unsigned>(sg.get_x_dim(), kMaxCols);
  for (unsigned c = 0; c < nc; ++c) {
    std::cout << "subgrid " << i << " correlation " << c << "\n";
    for (unsigned y = 0; y < ny; ++y) {
      for (unsigned x = 0; x < nx; ++x) put(sg(i, c, y, x));
      std::cout << "\n";
    }
  }
  std::cout << std::endl;
}

void print_subgrid_diff(idg::Array4D<std::complex<float>> &a,
                        idg::Array4D<std::complex<float>> &b, unsigned i) {
  format_saver keep(&std::cout);
  const unsigned nc = std::min<unsigned>(a.get_z_dim(), kMaxCorr);
  const unsigned ny = std::min<unsigned>(a.get_y_dim(), kMaxRows);
  const unsigned nx = std::min<unsigned>(a.get_x_dim(), kMaxCols);
  for (unsigned c = 0; c < nc; ++c) {
    std::cout << "subgrid diff " << i << " correlation " << c << "\n";
    for (unsigned y = 0; y < ny; ++y) {
      for (unsigned x = 0; x < nx; ++x) put(a(i, c, y, x) - b(i, c, y, x));
      std::cout << "\n";
    }
  }
  std::cout << std::endl;
}

void print_visibilities(
    idg::Array3D<idg::Visibility<std::complex<float>>> &vis, unsigned i) {
  format_saver keep(&std::cout);
  const unsigned nt = std::min<unsigned>(vis.get_y_dim(), kMaxTime);
  const unsigned nch = std::min<unsigned>(vis.get_x_dim(), kMaxChan);
  for (unsigned t = 0; t < nt; ++t) {
    for (unsigned c = 0; c < nch; ++c) {
      const auto &v = vis(i, t, c);
      std::cout << "row " << i << " t " << t << " c " << c << ": ";
      put(v.xx);
      put(v.xy);
      put(v.yx);
      put(v.yy);
      std::cout << "\n";
    }
  }
  std::cout << std::endl;
}

void print_visibilities_diff(
    idg::Array3D<idg::Visibility<std::complex<float>>> &a,
    idg::Array3D<idg::Visibility<std::complex<float>>> &b, unsigned i) {
  format_saver keep(&std::cout);
  const unsigned nt = std::min<unsigned>(a.get_y_dim(), kMaxTime);
  const unsigned nch = std::min<unsigned>(a.get_x_dim(), kMaxChan);
  for (unsigned t = 0; t < nt; ++t) {
    for (unsigned c = 0; c < nch; ++c) {
      const auto d = a(i, t, c) - b(i, t, c);
      std::cout << "row " << i << " t " << t << " c " << c << " diff: ";
      put(d.xx);
      put(d.xy);
      put(d.yx);
      put(d.yy);
      std::cout << "\n";
    }
  }
  std::cout << std::endl;
}
