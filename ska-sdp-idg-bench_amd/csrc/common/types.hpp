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

// Rank-R array, row-major, outermost index first in every accessor.
//
// Binary layout and symbol names are those of the reference's classes
// (types.hpp:59-356): a vtable, then the extents in the reference's member
// order (Array1D: x; Array2D: x, y; Array3D: x, y, z; Array4D: w, z, y, x),
// then the ownership flag and the buffer pointer; Array1D..Array4D are
// distinct class templates (not aliases), so a C++ entry point compiled
// against either header mangles identically and objects can be passed across.
template <class T, int R>
class ArrayND {
  static_assert(R >= 1 && R <= 4, "rank 1..4");

 public:
  ArrayND() { ext_.fill(0); }

  template <class... D, typename = std::enable_if_t<
                            sizeof...(D) == R &&
                            (std::is_integral<D>::value && ...)>>
  explicit ArrayND(D... dims) {
    set_dims({static_cast<size_t>(dims)...});
    owned_ = count() > 0;
    buf_ = allocate_memory<T>(count());
  }

  template <class... D, typename = std::enable_if_t<
                            sizeof...(D) == R &&
                            (std::is_integral<D>::value && ...)>>
  ArrayND(T *data, D... dims) : owned_(false), buf_(data) {
    set_dims({static_cast<size_t>(dims)...});
  }

  ArrayND(const ArrayND &) = delete;
  ArrayND &operator=(const ArrayND &) = delete;

  ArrayND(ArrayND &&o) noexcept
      : ext_(o.ext_), owned_(o.owned_), buf_(o.buf_) {
    o.buf_ = nullptr;
    o.owned_ = false;
  }

  ArrayND &operator=(ArrayND &&o) noexcept {
    if (this != &o) {
      release();
      ext_ = o.ext_;
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
    const size_t ix[R + 1] = {static_cast<size_t>(idx)..., 0};
    size_t off = 0;
    for (int d = 0; d < R; ++d)
      off = off * dim(d) + (d < static_cast<int>(sizeof...(I)) ? ix[d] : 0);
    return buf_ + off;
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
  size_t get_x_dim() const { return dim(R - 1); }
  size_t get_y_dim() const { return R >= 2 ? dim(R - 2) : 1; }
  size_t get_z_dim() const { return R >= 3 ? dim(R - 3) : 1; }
  size_t get_w_dim() const { return R >= 4 ? dim(R - 4) : 1; }

  size_t size() const { return count(); }
  size_t bytes() const { return count() * sizeof(T); }

  void init(const T &a) {
    for (size_t i = 0, n = count(); i < n; ++i) buf_[i] = a;
  }
  void zero() {
    if (buf_) std::memset(static_cast<void *>(buf_), 0, bytes());
  }

 protected:
  // Storage slot of outermost-first dimension d (reference member order).
  static constexpr int slot(int d) { return R == 4 ? d : R - 1 - d; }
  size_t dim(int d) const { return ext_[slot(d)]; }
  void set_dims(std::array<size_t, R> outer_first) {
    for (int d = 0; d < R; ++d) ext_[slot(d)] = outer_first[d];
  }
  size_t count() const {
    size_t n = 1;
    for (size_t e : ext_) n *= e;
    return n;
  }
  void release() {
    if (owned_) free(buf_);
    buf_ = nullptr;
    owned_ = false;
  }

  std::array<size_t, R> ext_{};
  bool owned_ = false;
  T *buf_ = nullptr;
};

#define IDG_ARRAY_CLASS(NAME, RANK)                                  \
  template <class T>                                                 \
  class NAME : public ArrayND<T, RANK> {                             \
   public:                                                           \
    using ArrayND<T, RANK>::ArrayND;                                 \
    NAME() = default;                                                \
    NAME(NAME &&) noexcept = default;                                \
    NAME &operator=(NAME &&) noexcept = default;                     \
  };

IDG_ARRAY_CLASS(Array1D, 1)
IDG_ARRAY_CLASS(Array2D, 2)
IDG_ARRAY_CLASS(Array3D, 3)
IDG_ARRAY_CLASS(Array4D, 4)
#undef IDG_ARRAY_CLASS

// Layout checks against the reference classes' member order.
static_assert(sizeof(Array1D<float>) == 32, "Array1D layout");
static_assert(sizeof(Array2D<float>) == 40, "Array2D layout");
static_assert(sizeof(Array3D<float>) == 48, "Array3D layout");
static_assert(sizeof(Array4D<float>) == 56, "Array4D layout");

// The reference declares (but never uses) a Grid type; kept for API parity.
class Grid : public Array4D<std::complex<float>> {
 public:
  using Array4D<std::complex<float>>::Array4D;
  explicit Grid(Array4D<std::complex<float>> &array)
      : Array4D<std::complex<float>>(array.data(), 1, array.get_z_dim(),
                                     array.get_y_dim(), array.get_x_dim()) {}
};

}  // namespace idg
