// print.hpp -- parameter banner and debug dumps.
// Entry points of the reference's app/common/print.{hpp,cpp}.
#pragma once

#include <complex>
#include <iostream>

#include "types.hpp"

// Restores an ostream's flags and precision on scope exit.
class format_saver {
 public:
  explicit format_saver(std::ostream *s)
      : s_(s), flags_(s->flags()), precision_(s->precision()) {}
  ~format_saver() {
    s_->flags(flags_);
    s_->precision(precision_);
  }

 private:
  std::ostream *s_;
  std::ios_base::fmtflags flags_;
  std::streamsize precision_;
};

void print_parameters(int nr_stations, int nr_channels, int nr_timesteps,
                      int nr_correlations, int nr_timeslots, float image_size,
                      int grid_size, int subgrid_size, float w_step,
                      int nr_baselines, int nr_subgrids,
                      int total_nr_timesteps);

void print_subgrid(idg::Array4D<std::complex<float>> &subgrids, unsigned i);

void print_subgrid_diff(idg::Array4D<std::complex<float>> &subgrids1,
                        idg::Array4D<std::complex<float>> &subgrids2,
                        unsigned i);

void print_visibilities(
    idg::Array3D<idg::Visibility<std::complex<float>>> &visibilities,
    unsigned i);

void print_visibilities_diff(
    idg::Array3D<idg::Visibility<std::complex<float>>> &visibilities1,
    idg::Array3D<idg::Visibility<std::complex<float>>> &visibilities2,
    unsigned i);
