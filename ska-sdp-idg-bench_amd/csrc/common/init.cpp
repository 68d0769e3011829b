// init.cpp -- synthetic observation generators (see init.hpp).
//
// Every expression below states its evaluation precision explicitly so the
// numbers match the reference generators (app/common/init.cpp) regardless of
// the host compiler: float/double conversions are spelled out and the
// multiply-adds the reference build fuses (the ellipse radii and A-term scale
// in double, the point-source phase u*l + v*m in float) are written as
// fma/fmaf.  Built with -ffp-contract=off.
#include "init.hpp"

#include <cmath>
#include <cstdlib>

#include "math.hpp"

namespace {

constexpr double kSpeedOfLight = 299792458.0;
constexpr double kPi = 3.14159265358979323846;

// One glibc rand() draw mapped to [0, 1], as the reference does everywhere.
inline double draw_unit() {
  return static_cast<double>(rand()) / static_cast<double>(RAND_MAX);
}

}  // namespace

// One random ellipse per row; rows are baselines (or subgrids, as the
// harness allocates uvw per subgrid).  reference init.cpp:4-25
void initialize_uvw(unsigned int grid_size,
                    idg::Array2D<idg::UVWCoordinate<float>> &uvw) {
  const size_t rows = uvw.get_y_dim();
  const size_t steps = uvw.get_x_dim();
  const double half = static_cast<double>(grid_size / 2);
  const float deg_per_step = 360.0f / static_cast<float>(steps);
  for (size_t r = 0; r < rows; ++r) {
    // The reference build (GCC 11, -O3 -march=native) fuses the double
    // `half + u * half` (init.cpp:11-14) and -- as its disassembly shows --
    // keeps the radii in double: the `float radius_u` rounding is elided
    // and u = (float)(radius * cos(angle * pi)) is formed from the double.
    const double ru = std::fma(draw_unit(), half, half);
    const double rv = std::fma(draw_unit(), half, half);
    idg::UVWCoordinate<float> *row = uvw.data(r);
    for (size_t t = 0; t < steps; ++t) {
      const float angle = static_cast<float>(
          (static_cast<double>(t) + 0.5) / static_cast<double>(deg_per_step));
      const double a = static_cast<double>(angle) * kPi;
      row[t].u = static_cast<float>(ru * std::cos(a));
      row[t].v = static_cast<float>(rv * std::sin(a));
      row[t].w = 0.0f;
    }
  }
}

// 150 MHz + 0.7 MHz * channel, in float.  reference init.cpp:27-36
void initialize_frequencies(idg::Array1D<float> &frequencies) {
  for (size_t c = 0; c < frequencies.get_x_dim(); ++c)
    frequencies(c) = static_cast<float>(150000000u) +
                     700000.0f * static_cast<float>(c);
}

// k = 2*pi*f/c in double, rounded to float.  reference init.cpp:38-46
void initialize_wavenumbers(const idg::Array1D<float> &frequencies,
                            idg::Array1D<float> &wavenumbers) {
  for (size_t c = 0; c < frequencies.get_x_dim(); ++c)
    wavenumbers(c) = static_cast<float>(
        2.0 * kPi * static_cast<double>(frequencies(c)) / kSpeedOfLight);
}

// A unit point source at (0.6, 0.7) * grid_size pixels, with per-correlation
// gains 1.01 .. 1.04.  reference init.cpp:48-79
void initialize_visibilities(
    unsigned int grid_size, float image_size,
    const idg::Array1D<float> &frequencies,
    const idg::Array2D<idg::UVWCoordinate<float>> &uvw,
    idg::Array3D<idg::Visibility<std::complex<float>>> &visibilities) {
  const size_t rows = visibilities.get_z_dim();
  const size_t steps = visibilities.get_y_dim();
  const size_t chans = visibilities.get_x_dim();
  const float gsize = static_cast<float>(grid_size);
  const float src_l =
      static_cast<float>(0.6 * grid_size) * image_size / gsize;
  const float src_m =
      static_cast<float>(0.7 * grid_size) * image_size / gsize;
  static const float gains[4] = {1.01f, 1.02f, 1.03f, 1.04f};
  for (size_t r = 0; r < rows; ++r) {
    for (size_t t = 0; t < steps; ++t) {
      const idg::UVWCoordinate<float> c = uvw(r, t);
      for (size_t ch = 0; ch < chans; ++ch) {
        const double lambda_inv =
            static_cast<double>(frequencies(ch)) / kSpeedOfLight;
        const float u = static_cast<float>(lambda_inv * c.u);
        const float v = static_cast<float>(lambda_inv * c.v);
        const float arg = static_cast<float>(
            -2.0 * kPi * static_cast<double>(fmaf(u, src_l, v * src_m)));
        const std::complex<float> value =
            std::exp(std::complex<float>(0.0f, arg));
        std::complex<float> *dst =
            reinterpret_cast<std::complex<float> *>(visibilities.data(r, t, ch));
        for (int p = 0; p < 4; ++p)
          dst[p] = std::complex<float>(value.real() * gains[p],
                                       value.imag() * gains[p]);
      }
    }
  }
}

// All station pairs (s1 < s2) in lexicographic order.  reference init.cpp:81-95
void initialize_baselines(unsigned int nr_stations,
                          idg::Array1D<idg::Baseline> &baselines) {
  const size_t n = baselines.get_x_dim();
  size_t bl = 0;
  for (unsigned s1 = 0; s1 < nr_stations && bl < n; ++s1)
    for (unsigned s2 = s1 + 1; s2 < nr_stations && bl < n; ++s2)
      baselines(bl++) = {s1, s2};
}

// Separable "tent" taper |2y/S - 1| * |2x/S - 1|.  reference init.cpp:97-107
void initialize_spheroidal(idg::Array2D<float> &spheroidal) {
  const size_t S = spheroidal.get_x_dim();
  const float fs = static_cast<float>(S);
  for (size_t y = 0; y < S; ++y) {
    const float ty = std::fabs(-1.0f + static_cast<float>(y) * 2.0f / fs);
    for (size_t x = 0; x < S; ++x) {
      const float tx = std::fabs(-1.0f + static_cast<float>(x) * 2.0f / fs);
      spheroidal(y, x) = ty * tx;
    }
  }
}

// Per (timeslot, station, pixel): taper * U(0.8, 1.2) plus fixed offsets.
// reference init.cpp:109-132
void initialize_aterms(
    const idg::Array2D<float> &spheroidal,
    idg::Array4D<idg::Matrix2x2<std::complex<float>>> &aterms) {
  const size_t slots = aterms.get_w_dim();
  const size_t stations = aterms.get_z_dim();
  const size_t S = aterms.get_y_dim();
  for (size_t a = 0; a < slots; ++a)
    for (size_t st = 0; st < stations; ++st)
      for (size_t y = 0; y < S; ++y)
        for (size_t x = 0; x < S; ++x) {
          // fused in the reference build: fma(u, 0.4, 0.8) (init.cpp:120)
          const float scale = static_cast<float>(std::fma(draw_unit(), 0.4, 0.8));
          const double value = static_cast<double>(spheroidal(y, x) * scale);
          const float hi = static_cast<float>(value + 0.1);
          const float lo = static_cast<float>(value - 0.2);
          aterms(a, st, y, x) = {{hi, -0.1f}, {lo, 0.1f}, {lo, 0.1f},
                                 {hi, -0.1f}};
        }
}

// One subgrid per (baseline, timeslot), placed uniformly at random on the
// grid.  reference init.cpp:134-159
void initialize_metadata(unsigned int grid_size, unsigned int nr_timeslots,
                         unsigned int nr_timesteps_subgrid,
                         const idg::Array1D<idg::Baseline> &baselines,
                         idg::Array1D<idg::Metadata> &metadata) {
  const size_t nbl = baselines.get_x_dim();
  for (size_t bl = 0; bl < nbl; ++bl)
    for (unsigned ts = 0; ts < nr_timeslots; ++ts) {
      idg::Metadata m{};
      m.baseline_offset = 0;
      m.time_offset = static_cast<int>((bl * nr_timeslots + ts) *
                                       nr_timesteps_subgrid);
      m.nr_timesteps = static_cast<int>(nr_timesteps_subgrid);
      m.aterm_index = 0;
      m.baseline = baselines(bl);
      m.coordinate.x = static_cast<int>(draw_unit() * grid_size);
      m.coordinate.y = static_cast<int>(draw_unit() * grid_size);
      m.coordinate.z = 0;
      metadata(bl * nr_timeslots + ts) = m;
    }
}

// Deterministic ramp used as degridder input.  reference init.cpp:161-180
void initialize_subgrids(idg::Array4D<std::complex<float>> &subgrids) {
  const size_t ns = subgrids.get_w_dim();
  const size_t nc = subgrids.get_z_dim();
  const size_t S = subgrids.get_y_dim();
  const float denom =
      100.0f * static_cast<float>(S) * static_cast<float>(S);
  for (size_t s = 0; s < ns; ++s)
    for (size_t c = 0; c < nc; ++c)
      for (size_t y = 0; y < S; ++y)
        for (size_t x = 0; x < S; ++x)
          subgrids(s, c, y, x) = std::complex<float>(
              static_cast<float>(static_cast<unsigned>(y * S + x + 1)) / denom,
              static_cast<float>(c) / 10.0f);
}

// (u, v, w) offsets of each subgrid in wavelengths.  reference init.cpp:182-199
void initialize_uvw_offsets(unsigned int subgrid_size, unsigned int grid_size,
                            float image_size, float w_step,
                            const idg::Array1D<idg::Metadata> &metadata,
                            idg::Array2D<float> &uvw_offsets) {
  const double scale = 2.0 * kPi / static_cast<double>(image_size);
  for (size_t i = 0; i < metadata.get_x_dim(); ++i) {
    const idg::Coordinate c = metadata(i).coordinate;
    const float w_lambda =
        static_cast<float>(w_step * (static_cast<double>(c.z) + 0.5));
    const float s2 = static_cast<float>(subgrid_size / 2);
    const float g2 = static_cast<float>(grid_size / 2);
    uvw_offsets(i, 0) =
        static_cast<float>((static_cast<float>(c.x) + s2 - g2) * scale);
    uvw_offsets(i, 1) =
        static_cast<float>((static_cast<float>(c.y) + s2 - g2) * scale);
    uvw_offsets(i, 2) = static_cast<float>(2.0 * kPi * w_lambda);
  }
}

// Direction cosines (l, m, n) of every subgrid pixel.  reference init.cpp:201-222
void initialize_lmn(float image_size, idg::Array3D<float> &lmn) {
  const int S = static_cast<int>(lmn.get_z_dim());
  for (int y = 0; y < S; ++y)
    for (int x = 0; x < S; ++x) {
      const float l = idg::compute_l(x, S, image_size);
      const float m = idg::compute_m(y, S, image_size);
      lmn(y, x, 0) = l;
      lmn(y, x, 1) = m;
      lmn(y, x, 2) = idg::compute_n(l, m);
    }
}
