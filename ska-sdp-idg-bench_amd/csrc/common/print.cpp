// print.cpp -- see print.hpp.
#include "print.hpp"

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
