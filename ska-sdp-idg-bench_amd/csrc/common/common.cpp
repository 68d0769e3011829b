// common.cpp -- see common.hpp.
#include "common.hpp"

#include <cmath>
#include <cstdlib>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <sstream>

unsigned roundToPowOf2(unsigned number) {
  if (number == 0) return 0;
  unsigned p = 1;
  while (p <= number / 2) p <<= 1;
  return p;
}

// Integer env var (atoi semantics, like reference common.cpp:10-16).
unsigned long get_env_var(const char *env_var, unsigned long default_value) {
  const char *v = std::getenv(env_var);
  return v ? static_cast<unsigned long>(atoi(v)) : default_value;
}

std::string get_env_var(const char *env_var, std::string default_value) {
  const char *v = std::getenv(env_var);
  return v ? std::string(v) : default_value;
}

namespace {

// The derived rates shared by the stdout and CSV reports, in the reference's
// order and units (common.cpp:27-98).
struct Rates {
  double ms, gflops_s, gb_s, flop_per_byte, mvis_s, watt, gflops_w, mvis_j;
  bool has_flops, has_bytes, has_mvis, has_energy;
};

Rates derive(double seconds, double gflops, double gbytes, double mvis,
             double joules) {
  Rates r{};
  r.ms = seconds * 1e3;
  r.has_flops = gflops != 0;
  r.has_bytes = gbytes != 0;
  r.has_mvis = mvis != 0;
  r.has_energy = joules != 0;
  if (r.has_flops) r.gflops_s = gflops / seconds;
  if (r.has_bytes) r.gb_s = gbytes / seconds;
  if (r.has_flops && r.has_bytes)
    r.flop_per_byte = static_cast<float>(gflops / gbytes);
  if (r.has_mvis) r.mvis_s = mvis / seconds;
  if (r.has_energy) {
    r.watt = joules / seconds;
    r.gflops_w = gflops / joules;
    r.mvis_j = mvis / joules;
  }
  return r;
}

}  // namespace

void report(std::string name, double seconds, double gflops, double gbytes,
            double mvis, double joules) {
  const Rates r = derive(seconds, gflops, gbytes, mvis, joules);
  std::ostringstream o;
  o << std::setw(20) << name << ": " << std::setprecision(2) << std::fixed
    << std::setw(7) << r.ms << " ms";
  if (r.has_flops) o << ", " << std::setw(7) << r.gflops_s << " GFLOP/s";
  if (r.has_bytes) o << ", " << std::setw(7) << r.gb_s << " GB/s";
  if (r.has_flops && r.has_bytes)
    o << ", " << std::setw(7) << r.flop_per_byte << " FLOP/byte";
  if (r.has_mvis) o << ", " << std::setw(7) << r.mvis_s << " MVis/s";
  if (r.has_energy)
    o << ", " << std::setw(7) << r.watt << " W, " << std::setw(7)
      << r.gflops_w << " GFLOP/s/W, " << std::setw(7) << r.mvis_j
      << " MVis/J";
  std::cout << o.str() << std::endl;
}

void report_csv(std::string name, std::string device_name,
                std::string file_extension, double seconds, double gflops,
                double gbytes, double mvis, double joules) {
  if (device_name.empty() || file_extension.empty()) {
    std::cout << ">>> Device name or file extension not provided" << std::endl;
    return;
  }
  for (char &ch : device_name)
    if (ch == '/') ch = '-';
  const std::string dir = get_env_var("OUTPUT_PATH", std::string("."));
  const std::string path = dir + "/" + device_name + "-" + name + file_extension;
  std::cout << "Saving output in " << dir << std::endl << path << std::endl;
  const Rates r = derive(seconds, gflops, gbytes, mvis, joules);
  std::ofstream out(path);
  out << std::fixed << std::setprecision(2);
  out << "ms," << r.ms << "\n";
  if (r.has_flops) out << "GFLOP/s," << r.gflops_s << "\n";
  if (r.has_bytes) out << "GB/s," << r.gb_s << "\n";
  if (r.has_flops && r.has_bytes) out << "FLOP/Byte," << r.flop_per_byte << "\n";
  if (r.has_mvis) out << "MVis/s," << r.mvis_s << "\n";
  if (r.has_energy)
    out << "W," << r.watt << "\nGFLOP/s/W," << r.gflops_w << "\nMVis/J,"
        << r.mvis_j << "\n";
}

// Work model of reference common.cpp:100-129.  Per visibility-timestep and
// pixel: 5 (phase index) + 5 (phase offset) + 2C (phase) + 8*C*ncorr (update);
// per subgrid pixel: 6 (shift).
uint64_t flops_gridder(uint64_t nr_channels, uint64_t nr_timesteps,
                       uint64_t nr_subgrids, uint64_t subgrid_size,
                       uint64_t nr_correlations) {
  const uint64_t pixels = subgrid_size * subgrid_size;
  const uint64_t per_vis = 5 + 5 + 2 * nr_channels +
                           8 * nr_channels * nr_correlations;
  return nr_timesteps * pixels * per_vis + nr_subgrids * pixels * 6;
}

// Byte model of reference common.cpp:131-159: uvw and visibilities read once
// per timestep; per subgrid pixel: pixel read+write, two A-terms, spheroidal.
uint64_t bytes_gridder(uint64_t nr_channels, uint64_t nr_timesteps,
                       uint64_t nr_subgrids, uint64_t subgrid_size,
                       uint64_t nr_correlations) {
  const uint64_t f = sizeof(float);
  const uint64_t pixels = nr_subgrids * subgrid_size * subgrid_size;
  const uint64_t per_timestep = 3 * f + nr_channels * nr_correlations * 2 * f;
  const uint64_t per_pixel = 2 * (nr_correlations * 2 * f) +  // pixel r+w
                             2 * nr_correlations * 2 * f +    // two A-terms
                             f;                               // spheroidal
  return nr_timesteps * per_timestep + pixels * per_pixel;
}
