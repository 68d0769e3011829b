// print.hpp -- the parameter banner of the reference's app/common/print.cpp
// (print_parameters, the one printer on the path; the reference's
// print_subgrid* / print_visibilities* debug dumps have no caller and are
// out of scope).
#pragma once

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
