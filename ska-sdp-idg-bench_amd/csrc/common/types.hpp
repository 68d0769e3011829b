// types.hpp -- IDG data types for the MI355X build.
//
// API-compatible with the reference's app/common/types.hpp:11-370
// (idg::Metadata, idg::UVWCoordinate, idg::Matrix2x2 / Visibility,
// idg::Array1D..Array4D with the same constructors, accessors and move-only
// semantics), re-designed as a single rank-generic ArrayND so it compiles
// cleanly under hipcc/clang (the reference's Array4D move constructor,
// types.hpp:286-290, names members that do not exist and is a clang error).
//
// Host arrays are 64-byte aligned, row-major, outermost dimension first.
#pragma once

#include <array>
#include <complex>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <new>
#include <type_traits>
#include <utility>

namespace idg {

struct Coordinate {
  int x, y, z;
};

struct Baseline {
  unsigned int station1, station2;
};

// 36 bytes; binary layout shared with the C-ABI (include/idg_mi355x.h).
struct Metadata {
  int baseline_offset;
  int time_offset;
  int nr_timesteps;
  int aterm_index;
  Baseline baseline;
  Coordinate coordinate;
};
static_assert(sizeof(Metadata) == 36, "Metadata must stay 36 bytes");

template <class T>
struct Matrix2x2 {
  T xx, xy, yx, yy;
};

template <class T>
Matrix2x2<T> operator-(const Matrix2x2<T> &a, const Matrix2x2<T> &b) {
  return {a.xx - b.xx, a.xy - b.xy, a.yx - b.yx, a.yy - b.yy};
}

template <class T>
using Visibility = Matrix2x2<T>;

template <class T>
struct UVWCoordinate {
  T u, v, w;
};

template <class T>
T *allocate_memory(size_t n) {
  void *ptr = nullptr;
  if (n == 0) return nullptr;
  if (posix_memalign(&ptr, 64, n * sizeof(T)) != 0) throw std::bad_alloc();
  return static_cast<T *>(ptr);
}

// Rank-R array.  dims_[0] is the outermost dimension, dims_[R-1] the
// innermost ("x").  Owning arrays free their buffer; views do not.
template <class T, int R>
class ArrayND {
  static_assert(R >= 1 && R <= 4, "rank 1..4");

 public:
  ArrayND() { dims_.fill(0); }

  template <class... D, typename = std::enable_if_t<
                            sizeof...(D) == R &&
                            (std::is_integral<D>::value && ...)>>
  explicit ArrayND(D... dims) : dims_{static_cast<size_t>(dims)...} {
    owned_ = count() > 0;
    buf_ = allocate_memory<T>(count());
  }

  template <class... D, typename = std::enable_if_t<
                            sizeof...(D) == R &&
                            (std::is_integral<D>::value && ...)>>
  ArrayND(T *data, D... dims)
      : dims_{static_cast<size_t>(dims)...}, owned_(false), buf_(data) {}

  ArrayND(const ArrayND &) = delete;
  ArrayND &operator=(const ArrayND &) = delete;

  ArrayND(ArrayND &&o) noexcept
      : dims_(o.dims_), owned_(o.owned_), buf_(o.buf_) {
    o.buf_ = nullptr;
    o.owned_ = false;
  }

  ArrayND &operator=(ArrayND &&o) noexcept {
    if (this != &o) {
      release();
      dims_ = o.dims_;
      owned_ = o.owned_;
      buf_ = o.buf_;
      o.buf_ = nullptr;
      o.owned_ = false;
    }
    return *this;
  }

  virtual ~ArrayND() { release(); }

  // Element pointer at the given (outermost-first) index prefix.
  template <class... I>
  T *data(I... idx) const {
    static_assert(sizeof...(I) <= R, "too many indices");
    return buf_ + offset_of(std::array<size_t, sizeof...(I)>{
                      static_cast<size_t>(idx)...});
  }

  template <class... I>
  T &operator()(I... idx) {
    static_assert(sizeof...(I) == R, "need one index per dimension");
    return *data(idx...);
  }
  template <class... I>
  const T &operator()(I... idx) const {
    static_assert(sizeof...(I) == R, "need one index per dimension");
    return *data(idx...);
  }

  // Reference accessor names: x = innermost ... w = outermost of a 4-D array.
  size_t get_x_dim() const { return dims_[R - 1]; }
  size_t get_y_dim() const { return inner(1); }
  size_t get_z_dim() const { return inner(2); }
  size_t get_w_dim() const { return inner(3); }

  size_t size() const { return count(); }
  size_t bytes() const { return count() * sizeof(T); }

  void init(const T &a) {
    for (size_t i = 0, n = count(); i < n; ++i) buf_[i] = a;
  }
  void zero() {
    if (buf_) std::memset(static_cast<void *>(buf_), 0, bytes());
  }

 protected:
  size_t count() const {
    size_t n = 1;
    for (size_t d : dims_) n *= d;
    return n;
  }
  size_t inner(int k) const { return R - 1 - k >= 0 ? dims_[R - 1 - k] : 1; }
  template <size_t K>
  size_t offset_of(const std::array<size_t, K> &idx) const {
    size_t off = 0;
    for (int d = 0; d < R; ++d)
      off = off * dims_[d] + (static_cast<size_t>(d) < K ? idx[d] : 0);
    return off;
  }
  void release() {
    if (owned_) free(buf_);
    buf_ = nullptr;
    owned_ = false;
  }

  std::array<size_t, R> dims_{};
  bool owned_ = false;
  T *buf_ = nullptr;
};

template <class T>
using Array1D = ArrayND<T, 1>;
template <class T>
using Array2D = ArrayND<T, 2>;
template <class T>
using Array3D = ArrayND<T, 3>;
template <class T>
using Array4D = ArrayND<T, 4>;

// The reference declares (but never uses) a Grid type; kept for API parity.
class Grid : public Array4D<std::complex<float>> {
 public:
  using Array4D<std::complex<float>>::Array4D;
};

}  // namespace idg
