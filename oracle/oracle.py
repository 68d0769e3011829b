"""ctypes wrapper of the CPU checkers -- TEST INFRASTRUCTURE ONLY.

Imported only by tests/, by __graft_entry__.smoke() and by bench.py's
cpu_baseline leg, always as the checker / the timed CPU baseline, never as the
product path (the product library, ska-sdp-idg-bench_amd/, has no CPU
fallback and never loads this module).

  liboracle.so        oracle/idg_oracle.c, plain-C restatement of the
                      reference app/CPU path (explicit-fmaf fusion pattern)
  _ref/libidgref*.so  the reference's own app/CPU + app/common sources,
                      compiled where they lie under /root/reference
                      (oracle/Makefile) -- present only where built
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

METADATA_DTYPE = np.dtype([("baseline_offset", "<i4"), ("time_offset", "<i4"),
                           ("nr_timesteps", "<i4"), ("aterm_index", "<i4"),
                           ("station1", "<u4"), ("station2", "<u4"),
                           ("x", "<i4"), ("y", "<i4"), ("z", "<i4")])

_P = ctypes.c_void_p
_I = ctypes.c_int
_F = ctypes.c_float


def _ptr(a):
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "arrays must be C-contiguous"
    return a.ctypes.data_as(_P)


def _md(a):
    a = np.ascontiguousarray(a)
    if a.dtype != METADATA_DTYPE:
        a = np.ascontiguousarray(a.astype(np.int32).reshape(-1, 9)).view(
            METADATA_DTYPE).reshape(-1)
    return a


_KERNEL_ARGS = [_I, _I, _I, _F, _F, _I, _I, _P, _P, _P, _P, _P, _P, _P]


class Oracle:
    """The plain-C restatement (liboracle.so)."""

    def __init__(self, path=None):
        path = path or os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: run make -C oracle")
        self.lib = ctypes.CDLL(path)
        for fn in (self.lib.oracle_gridder, self.lib.oracle_degridder,
                   self.lib.oracle_gridder_exact,
                   self.lib.oracle_degridder_exact):
            fn.argtypes = _KERNEL_ARGS + [_I]
            fn.restype = None
        self.lib.oracle_check_error.argtypes = [ctypes.c_int64, _P, _P, _P]
        self.lib.oracle_check_error.restype = ctypes.c_double

    def gridder(self, nr_subgrids, grid_size, subgrid_size, image_size,
                w_step, nr_channels, nr_stations, uvw, wavenumbers,
                visibilities, spheroidal, aterms, metadata, subgrids,
                nthreads=1):
        md = _md(metadata)
        self.lib.oracle_gridder(nr_subgrids, grid_size, subgrid_size,
                                image_size, w_step, nr_channels, nr_stations,
                                _ptr(uvw), _ptr(wavenumbers),
                                _ptr(visibilities), _ptr(spheroidal),
                                _ptr(aterms), _ptr(md), _ptr(subgrids),
                                nthreads)
        return subgrids

    def degridder(self, nr_subgrids, grid_size, subgrid_size, image_size,
                  w_step, nr_channels, nr_stations, uvw, wavenumbers,
                  visibilities, spheroidal, aterms, metadata, subgrids,
                  nthreads=1):
        md = _md(metadata)
        self.lib.oracle_degridder(nr_subgrids, grid_size, subgrid_size,
                                  image_size, w_step, nr_channels,
                                  nr_stations, _ptr(uvw), _ptr(wavenumbers),
                                  _ptr(visibilities), _ptr(spheroidal),
                                  _ptr(aterms), _ptr(md), _ptr(subgrids),
                                  nthreads)
        return visibilities

    def gridder_exact(self, nr_subgrids, grid_size, subgrid_size, image_size,
                      w_step, nr_channels, nr_stations, uvw, wavenumbers,
                      visibilities, spheroidal, aterms, metadata, subgrids,
                      nthreads=1):
        """The reference's f32 phases, everything after them in double
        (oracle_gridder_exact); subgrids: float64 [..., 2]."""
        assert subgrids.dtype == np.float64
        md = _md(metadata)
        self.lib.oracle_gridder_exact(
            nr_subgrids, grid_size, subgrid_size, image_size, w_step,
            nr_channels, nr_stations, _ptr(uvw), _ptr(wavenumbers),
            _ptr(visibilities), _ptr(spheroidal), _ptr(aterms), _ptr(md),
            _ptr(subgrids), nthreads)
        return subgrids

    def degridder_exact(self, nr_subgrids, grid_size, subgrid_size,
                        image_size, w_step, nr_channels, nr_stations, uvw,
                        wavenumbers, visibilities, spheroidal, aterms,
                        metadata, subgrids, nthreads=1):
        """As degridder, accumulated in double; visibilities: float64."""
        assert visibilities.dtype == np.float64
        md = _md(metadata)
        self.lib.oracle_degridder_exact(
            nr_subgrids, grid_size, subgrid_size, image_size, w_step,
            nr_channels, nr_stations, _ptr(uvw), _ptr(wavenumbers),
            _ptr(visibilities), _ptr(spheroidal), _ptr(aterms), _ptr(md),
            _ptr(subgrids), nthreads)
        return visibilities

    def check_error(self, candidate, reference):
        """tests/test_util.hpp:28-92 metric; returns (error, nnz)."""
        a = np.ascontiguousarray(candidate, np.float32)
        b = np.ascontiguousarray(reference, np.float32)
        assert a.size == b.size and a.size % 2 == 0
        nnz = ctypes.c_int64(0)
        err = self.lib.oracle_check_error(a.size // 2, _ptr(a), _ptr(b),
                                          ctypes.byref(nnz))
        return err, nnz.value


def check_error(candidate, reference):
    """Pure-numpy twin of the parity metric (A = candidate, B = reference)."""
    a = np.asarray(candidate, np.float32).reshape(-1, 2)
    b = np.asarray(reference, np.float32).reshape(-1, 2)
    r_max = max(1.0, float(np.abs(a[:, 0]).max(initial=0.0)))
    i_max = max(1.0, float(np.abs(a[:, 1]).max(initial=0.0)))
    mask = np.hypot(b[:, 0], b[:, 1]) > 0
    dr = (b[mask, 0] - a[mask, 0]).astype(np.float64)
    di = (b[mask, 1] - a[mask, 1]).astype(np.float64)
    nnz = max(1, int(mask.sum()))
    return float(np.sqrt((dr * dr).sum() / r_max / nnz +
                         (di * di).sum() / i_max / nnz))


class Reference:
    """The reference's own CPU path (oracle/_ref/libidgref*.so), if built."""

    def __init__(self, portable=True):
        name = "libidgref_v3.so" if portable else "libidgref.so"
        path = os.path.join(HERE, "_ref", name)
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        self.path = path
        self.lib = ctypes.CDLL(path)
        for fn in (self.lib.ref_gridder, self.lib.ref_degridder):
            fn.argtypes = list(_KERNEL_ARGS)
            fn.restype = None

    @staticmethod
    def available(portable=True):
        name = "libidgref_v3.so" if portable else "libidgref.so"
        return os.path.exists(os.path.join(HERE, "_ref", name))

    def gridder(self, nr_subgrids, grid_size, subgrid_size, image_size,
                w_step, nr_channels, nr_stations, uvw, wavenumbers,
                visibilities, spheroidal, aterms, metadata, subgrids):
        md = _md(metadata)
        self.lib.ref_gridder(nr_subgrids, grid_size, subgrid_size, image_size,
                             w_step, nr_channels, nr_stations, _ptr(uvw),
                             _ptr(wavenumbers), _ptr(visibilities),
                             _ptr(spheroidal), _ptr(aterms), _ptr(md),
                             _ptr(subgrids))
        return subgrids

    def degridder(self, nr_subgrids, grid_size, subgrid_size, image_size,
                  w_step, nr_channels, nr_stations, uvw, wavenumbers,
                  visibilities, spheroidal, aterms, metadata, subgrids):
        md = _md(metadata)
        self.lib.ref_degridder(nr_subgrids, grid_size, subgrid_size,
                               image_size, w_step, nr_channels, nr_stations,
                               _ptr(uvw), _ptr(wavenumbers),
                               _ptr(visibilities), _ptr(spheroidal),
                               _ptr(aterms), _ptr(md), _ptr(subgrids))
        return visibilities
