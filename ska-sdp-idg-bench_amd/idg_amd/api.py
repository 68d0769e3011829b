"""Python mirror of the reference's gridder/degridder operator interface.

Same names, argument order and meaning as the reference's kernel-TU contract
(hip::c_run_gridder / hip::c_run_degridder, declared by the harness at
tests/gridder_common.cpp:13-31 and tests/degridder_common.cpp:13-31) and its
perf entries (hip::p_run_gridder / hip::p_run_degridder), over the C ABI of
libidg_mi355x.so.  numpy arrays stand in for the idg::ArrayND objects;
device-resident variants take torch CUDA tensors (PyTorch is only used as the
device allocator / stream provider).

Errors: where the reference's C++ entries abort the process (hipCheck ->
exit, app/HIP/util.cpp:5-15), these raise IdgError carrying the status code
and message.
"""
import ctypes

import numpy as np

from ._lib import lib

IMAGE_SIZE = 0.01   # app/common/parameters.hpp:4
W_STEP = 0.0        # app/common/parameters.hpp:5
NR_CORRELATIONS = 4

METADATA_DTYPE = np.dtype([("baseline_offset", "<i4"), ("time_offset", "<i4"),
                           ("nr_timesteps", "<i4"), ("aterm_index", "<i4"),
                           ("station1", "<u4"), ("station2", "<u4"),
                           ("x", "<i4"), ("y", "<i4"), ("z", "<i4")])
assert METADATA_DTYPE.itemsize == 36


class IdgError(RuntimeError):
    def __init__(self, code, what):
        msg = lib.idg_last_error().decode(errors="replace")
        super().__init__(f"{what} failed (status {code}): {msg}")
        self.code = code


def _check(code, what):
    if code != 0:
        raise IdgError(code, what)


def _np_ptr(a, dtype, name, writable=False):
    if not isinstance(a, np.ndarray):
        raise TypeError(f"{name} must be a numpy array")
    if a.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {a.dtype}")
    if not a.flags["C_CONTIGUOUS"]:
        raise ValueError(f"{name} must be C-contiguous")
    if writable and not a.flags["WRITEABLE"]:
        raise ValueError(f"{name} must be writable")
    return a.ctypes.data_as(ctypes.c_void_p)


def as_metadata(md):
    """Accept a METADATA_DTYPE array or an int32 [n, 9] array."""
    md = np.asarray(md)
    if md.dtype == METADATA_DTYPE:
        return np.ascontiguousarray(md)
    md = np.ascontiguousarray(md, dtype=np.int32).reshape(-1, 9)
    return md.view(METADATA_DTYPE).reshape(-1)


def nr_subgrids_for(nr_stations, nr_timeslots):
    return nr_stations * (nr_stations - 1) // 2 * nr_timeslots


# ---------------------------------------------------------------------------
# Synthetic observation (app/common/init.cpp, harness order, srand(0))
# ---------------------------------------------------------------------------
def generate(nr_stations, nr_timeslots, nr_timesteps, nr_channels, grid_size,
             subgrid_size, want=("uvw", "frequencies", "wavenumbers",
                                 "visibilities", "spheroidal", "aterms",
                                 "metadata", "subgrids"), nthreads=8):
    """Return a dict of numpy arrays holding exactly the inputs the reference
    harness builds (tests/gridder_common.cpp:87-101).  Shapes:
      uvw [NS, T, 3] f32; frequencies, wavenumbers [C] f32;
      visibilities [NS, T, C, 4, 2] f32; spheroidal [S, S] f32;
      aterms [TS, ST, S, S, 4, 2] f32; metadata [NS] METADATA_DTYPE;
      subgrids [NS, 4, S, S, 2] f32 (the degridder input ramp)."""
    ns = nr_subgrids_for(nr_stations, nr_timeslots)
    S = subgrid_size
    shapes = {
        "uvw": ((ns, nr_timesteps, 3), np.float32),
        "frequencies": ((nr_channels,), np.float32),
        "wavenumbers": ((nr_channels,), np.float32),
        "visibilities": ((ns, nr_timesteps, nr_channels, 4, 2), np.float32),
        "spheroidal": ((S, S), np.float32),
        "aterms": ((nr_timeslots, nr_stations, S, S, 4, 2), np.float32),
        "metadata": ((ns,), METADATA_DTYPE),
        "subgrids": ((ns, 4, S, S, 2), np.float32),
    }
    out = {k: np.empty(*shapes[k]) for k in want}
    ptr = {k: (out[k].ctypes.data_as(ctypes.c_void_p) if k in out else None)
           for k in shapes}
    got = lib.idg_generate(nr_stations, nr_timeslots, nr_timesteps,
                           nr_channels, grid_size, subgrid_size, ptr["uvw"],
                           ptr["frequencies"], ptr["wavenumbers"],
                           ptr["visibilities"], ptr["spheroidal"],
                           ptr["aterms"], ptr["metadata"], ptr["subgrids"],
                           nthreads)
    if got < 0:
        raise IdgError(got, "idg_generate")
    assert got == ns
    return out


# ---------------------------------------------------------------------------
# Host-buffer entries: hip::c_run_gridder / hip::c_run_degridder
# ---------------------------------------------------------------------------
def _extents(nr_channels, uvw, visibilities, aterms, subgrids, subgrid_size,
             nr_subgrids, nr_stations):
    rows = uvw.size // 3
    if uvw.size % 3:
        raise ValueError("uvw must hold whole (u, v, w) triplets")
    if visibilities.size != rows * nr_channels * 8:
        raise ValueError(
            f"visibilities must hold rows*nr_channels*4 complex values "
            f"({rows}*{nr_channels}*4), got {visibilities.size // 2}")
    per_slot = nr_stations * subgrid_size * subgrid_size * 8
    if aterms.size % per_slot:
        raise ValueError("aterms must be [slots][nr_stations][S][S][4] complex")
    if subgrids.size != nr_subgrids * 4 * subgrid_size * subgrid_size * 2:
        raise ValueError("subgrids must be [nr_subgrids][4][S][S] complex")
    return rows, aterms.size // per_slot


def c_run_gridder(nr_subgrids, grid_size, subgrid_size, image_size,
                  w_step_in_lambda, nr_channels, nr_stations, uvw,
                  wavenumbers, visibilities, spheroidal, aterms, metadata,
                  subgrids):
    """Grid visibilities onto subgrids (fills `subgrids` in place)."""
    md = as_metadata(metadata)
    rows, slots = _extents(nr_channels, uvw, visibilities, aterms, subgrids,
                           subgrid_size, nr_subgrids, nr_stations)
    _check(lib.idg_c_run_gridder(
        nr_subgrids, grid_size, subgrid_size, image_size, w_step_in_lambda,
        nr_channels, nr_stations, _np_ptr(uvw, np.float32, "uvw"), rows,
        _np_ptr(wavenumbers, np.float32, "wavenumbers"),
        _np_ptr(visibilities, np.float32, "visibilities"),
        _np_ptr(spheroidal, np.float32, "spheroidal"),
        _np_ptr(aterms, np.float32, "aterms"), slots,
        _np_ptr(md, METADATA_DTYPE, "metadata"),
        _np_ptr(subgrids, np.float32, "subgrids", True)), "c_run_gridder")
    return subgrids


def c_run_degridder(nr_subgrids, grid_size, subgrid_size, image_size,
                    w_step_in_lambda, nr_channels, nr_stations, uvw,
                    wavenumbers, visibilities, spheroidal, aterms, metadata,
                    subgrids):
    """Degrid subgrids into visibilities (fills `visibilities` in place)."""
    md = as_metadata(metadata)
    rows, slots = _extents(nr_channels, uvw, visibilities, aterms, subgrids,
                           subgrid_size, nr_subgrids, nr_stations)
    _check(lib.idg_c_run_degridder(
        nr_subgrids, grid_size, subgrid_size, image_size, w_step_in_lambda,
        nr_channels, nr_stations, _np_ptr(uvw, np.float32, "uvw"), rows,
        _np_ptr(wavenumbers, np.float32, "wavenumbers"),
        _np_ptr(visibilities, np.float32, "visibilities", True),
        _np_ptr(spheroidal, np.float32, "spheroidal"),
        _np_ptr(aterms, np.float32, "aterms"), slots,
        _np_ptr(md, METADATA_DTYPE, "metadata"),
        _np_ptr(subgrids, np.float32, "subgrids")), "c_run_degridder")
    return visibilities


def validate_metadata(nr_subgrids, subgrid_size, nr_channels, nr_stations,
                      uvw_rows, aterm_slots, metadata):
    md = as_metadata(metadata)
    _check(lib.idg_validate_metadata(
        nr_subgrids, subgrid_size, nr_channels, nr_stations, uvw_rows,
        aterm_slots, _np_ptr(md, METADATA_DTYPE, "metadata")),
        "validate_metadata")


def host_chunk_plan(metadata, bytes_moved):
    """Subgrid bounds of the chunks the host-buffer entries split a batch
    into (idg_host_chunk_plan; util.cpp plan_host_chunks): a list of
    nchunk + 1 subgrid indices."""
    import numpy as np
    md = as_metadata(metadata)
    bounds = np.zeros(18, np.int32)
    n = lib.idg_host_chunk_plan(md.size, _np_ptr(md, METADATA_DTYPE,
                                                  "metadata"),
                                int(bytes_moved), bounds.ctypes.data_as(
                                    ctypes.c_void_p), bounds.size)
    if n < 0:
        _check(n, "host_chunk_plan")
    return [int(b) for b in bounds[:n + 1]]


# ---------------------------------------------------------------------------
# Device-buffer entries (torch CUDA tensors, asynchronous on a stream)
# ---------------------------------------------------------------------------
def _dev_ptr(t, name, dtype=None):
    import torch
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise TypeError(f"{name} must be a CUDA (HIP) torch tensor")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if dtype is not None and t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {t.dtype}")
    return ctypes.c_void_p(t.data_ptr())


def _stream_handle(stream):
    import torch
    if stream is None:
        stream = torch.cuda.current_stream()
    return ctypes.c_void_p(stream.cuda_stream)


def _dev_extents(nr_subgrids, subgrid_size, nr_channels, nr_stations, uvw,
                 wavenumbers, visibilities, spheroidal, aterms, metadata,
                 subgrids, validate):
    """Host-side shape checks of a device launch (no device access): every
    tensor must hold exactly the extents the kernel's grid will index.
    With validate=True the metadata is also copied to the host once and
    checked against those extents (idg_validate_metadata: row ranges,
    A-term slots, stations); launches stay asynchronous otherwise, so
    callers that build their own metadata validate it once up front."""
    S, C = subgrid_size, nr_channels
    if uvw.numel() % 3:
        raise ValueError("uvw must hold whole (u, v, w) triplets")
    rows = uvw.numel() // 3
    if visibilities.numel() != rows * C * 8:
        raise ValueError(
            f"visibilities must hold uvw rows x nr_channels x 4 complex "
            f"({rows} x {C} x 4), got {visibilities.numel() // 2}")
    if wavenumbers.numel() < C:
        raise ValueError(f"wavenumbers must hold nr_channels ({C}) values")
    if spheroidal.numel() != S * S:
        raise ValueError(f"spheroidal must be [{S}][{S}]")
    per_slot = nr_stations * S * S * 8
    if aterms.numel() == 0 or aterms.numel() % per_slot:
        raise ValueError("aterms must be [slots][nr_stations][S][S][4] "
                         "complex")
    if metadata.numel() * metadata.element_size() != nr_subgrids * 36:
        raise ValueError(f"metadata must hold nr_subgrids ({nr_subgrids}) "
                         "x 36-byte records")
    if subgrids.numel() != nr_subgrids * 4 * S * S * 2:
        raise ValueError(f"subgrids must be [{nr_subgrids}][4][{S}][{S}] "
                         "complex")
    if validate:
        md = metadata.detach().cpu().contiguous().view(-1).numpy()
        validate_metadata(nr_subgrids, S, C, nr_stations, rows,
                          aterms.numel() // per_slot,
                          np.frombuffer(md.tobytes(), METADATA_DTYPE))


def gridder_launch(nr_subgrids, grid_size, subgrid_size, image_size,
                   w_step_in_lambda, nr_channels, nr_stations, uvw,
                   wavenumbers, visibilities, spheroidal, aterms, metadata,
                   subgrids, stream=None, validate=False):
    """Enqueue the gridder on device-resident tensors (metadata as int32
    [NS, 9] tensor or uint8 view of METADATA_DTYPE); returns immediately.
    Tensor extents are checked on the host; validate=True also checks the
    metadata (one device-to-host copy)."""
    import torch
    f32 = torch.float32
    _dev_extents(nr_subgrids, subgrid_size, nr_channels, nr_stations, uvw,
                 wavenumbers, visibilities, spheroidal, aterms, metadata,
                 subgrids, validate)
    _check(lib.idg_gridder_launch(
        nr_subgrids, grid_size, subgrid_size, image_size, w_step_in_lambda,
        nr_channels, nr_stations, _dev_ptr(uvw, "uvw", f32),
        _dev_ptr(wavenumbers, "wavenumbers", f32),
        _dev_ptr(visibilities, "visibilities", f32),
        _dev_ptr(spheroidal, "spheroidal", f32),
        _dev_ptr(aterms, "aterms", f32), _dev_ptr(metadata, "metadata"),
        _dev_ptr(subgrids, "subgrids", f32), _stream_handle(stream)),
        "gridder_launch")


def gridder_fft_launch(nr_subgrids, grid_size, subgrid_size, image_size,
                       w_step_in_lambda, nr_channels, nr_stations, uvw,
                       wavenumbers, visibilities, spheroidal, aterms, metadata,
                       subgrids, stream=None, validate=False):
    """gridder_launch followed by subgrid_fft_launch(+1, 1.0): the adder's
    input (uv-domain) subgrids; the FFT runs in the gridder's epilogue for
    S = 32, bit for bit the two launches' result."""
    import torch
    f32 = torch.float32
    _dev_extents(nr_subgrids, subgrid_size, nr_channels, nr_stations, uvw,
                 wavenumbers, visibilities, spheroidal, aterms, metadata,
                 subgrids, validate)
    _check(lib.idg_gridder_fft_launch(
        nr_subgrids, grid_size, subgrid_size, image_size, w_step_in_lambda,
        nr_channels, nr_stations, _dev_ptr(uvw, "uvw", f32),
        _dev_ptr(wavenumbers, "wavenumbers", f32),
        _dev_ptr(visibilities, "visibilities", f32),
        _dev_ptr(spheroidal, "spheroidal", f32),
        _dev_ptr(aterms, "aterms", f32), _dev_ptr(metadata, "metadata"),
        _dev_ptr(subgrids, "subgrids", f32), _stream_handle(stream)),
        "gridder_fft_launch")


def degridder_launch(nr_subgrids, grid_size, subgrid_size, image_size,
                     w_step_in_lambda, nr_channels, nr_stations, uvw,
                     wavenumbers, visibilities, spheroidal, aterms, metadata,
                     subgrids, stream=None, validate=False):
    """Enqueue the degridder on device-resident tensors; returns immediately.
    Extent checks and `validate` as for gridder_launch."""
    import torch
    f32 = torch.float32
    _dev_extents(nr_subgrids, subgrid_size, nr_channels, nr_stations, uvw,
                 wavenumbers, visibilities, spheroidal, aterms, metadata,
                 subgrids, validate)
    _check(lib.idg_degridder_launch(
        nr_subgrids, grid_size, subgrid_size, image_size, w_step_in_lambda,
        nr_channels, nr_stations, _dev_ptr(uvw, "uvw", f32),
        _dev_ptr(wavenumbers, "wavenumbers", f32),
        _dev_ptr(visibilities, "visibilities", f32),
        _dev_ptr(spheroidal, "spheroidal", f32),
        _dev_ptr(aterms, "aterms", f32), _dev_ptr(metadata, "metadata"),
        _dev_ptr(subgrids, "subgrids", f32), _stream_handle(stream)),
        "degridder_launch")


# ---------------------------------------------------------------------------
# Pipeline steps either side of the path (not in the
# reference).  gridding:   gridder -> subgrid_fft(+1) -> adder
#              degridding: splitter -> subgrid_fft(-1, 1/S^2) -> degridder
# ---------------------------------------------------------------------------
def _pipe_extents(ns, grid_size, S, nr_w_layers, metadata, subgrids, grid):
    if subgrids.dim() != 5 or tuple(subgrids.shape[1:]) != (4, S, S, 2):
        raise ValueError("subgrids must be [NS][4][S][S][2] float32")
    if metadata.numel() * metadata.element_size() != ns * 36:
        raise ValueError(f"metadata must hold {ns} x 36-byte records")
    if grid.numel() != nr_w_layers * 4 * grid_size * grid_size * 2:
        raise ValueError(f"grid must be [{nr_w_layers}][4][{grid_size}]"
                         f"[{grid_size}][2] float32")


def subgrid_fft_launch(subgrids, sign, scale=1.0, stream=None):
    """In-place 2-D DFT of every [S][S] correlation plane of a float32
    [NS, 4, S, S, 2] tensor: out = scale * sum in * exp(sign 2 pi i ...)."""
    import torch
    ns, _, S = subgrids.shape[0], subgrids.shape[1], subgrids.shape[2]
    _check(lib.idg_subgrid_fft_launch(
        ns, S, int(sign), float(scale),
        _dev_ptr(subgrids, "subgrids", torch.float32), _stream_handle(stream)),
        "subgrid_fft_launch")


def adder_launch(grid_size, metadata, subgrids, grid, nr_w_layers=1,
                 stream=None):
    """grid [W, 4, G, G, 2] float32 += the FFT'd subgrids placed at their
    metadata coordinates.  A deterministic gather: each 16x16 grid tile adds
    the subgrids overlapping it in ascending subgrid order (no atomics on
    the grid)."""
    import torch
    ns, S = subgrids.shape[0], subgrids.shape[2]
    _pipe_extents(ns, grid_size, S, nr_w_layers, metadata, subgrids, grid)
    _check(lib.idg_adder_launch(
        ns, grid_size, S, nr_w_layers, _dev_ptr(metadata, "metadata"),
        _dev_ptr(subgrids, "subgrids", torch.float32),
        _dev_ptr(grid, "grid", torch.float32), _stream_handle(stream)),
        "adder_launch")


def splitter_launch(grid_size, metadata, grid, subgrids, nr_w_layers=1,
                    stream=None):
    """subgrids [NS, 4, S, S, 2] = the uv cells under each subgrid (adjoint
    of adder_launch's placement)."""
    import torch
    ns, S = subgrids.shape[0], subgrids.shape[2]
    _pipe_extents(ns, grid_size, S, nr_w_layers, metadata, subgrids, grid)
    _check(lib.idg_splitter_launch(
        ns, grid_size, S, nr_w_layers, _dev_ptr(metadata, "metadata"),
        _dev_ptr(grid, "grid", torch.float32),
        _dev_ptr(subgrids, "subgrids", torch.float32), _stream_handle(stream)),
        "splitter_launch")


def splitter_fft_launch(grid_size, metadata, grid, subgrids, nr_w_layers=1,
                        stream=None):
    """splitter_launch followed by subgrid_fft_launch(-1, 1/S^2): the
    degridder's input subgrids from the grid (one fused kernel for S = 32 and
    64, bit for bit the two launches' result)."""
    import torch
    ns, S = subgrids.shape[0], subgrids.shape[2]
    _pipe_extents(ns, grid_size, S, nr_w_layers, metadata, subgrids, grid)
    _check(lib.idg_splitter_fft_launch(
        ns, grid_size, S, nr_w_layers, _dev_ptr(metadata, "metadata"),
        _dev_ptr(grid, "grid", torch.float32),
        _dev_ptr(subgrids, "subgrids", torch.float32), _stream_handle(stream)),
        "splitter_fft_launch")


def grid_onto(nr_subgrids, grid_size, subgrid_size, image_size,
              w_step_in_lambda, nr_channels, nr_stations, uvw, wavenumbers,
              visibilities, spheroidal, aterms, metadata, grid,
              nr_w_layers=1, subgrids=None, stream=None):
    """Visibilities -> uv grid: gridder and subgrid FFT (+1), fused for
    S = 32 (gridder_fft_launch), then the adder into `grid` (accumulates).
    Returns the (uv-domain) subgrid scratch."""
    import torch
    if subgrids is None:
        subgrids = torch.empty((nr_subgrids, 4, subgrid_size, subgrid_size, 2),
                               dtype=torch.float32, device=grid.device)
    gridder_fft_launch(nr_subgrids, grid_size, subgrid_size, image_size,
                       w_step_in_lambda, nr_channels, nr_stations, uvw,
                       wavenumbers, visibilities, spheroidal, aterms,
                       metadata, subgrids, stream)
    adder_launch(grid_size, metadata, subgrids, grid, nr_w_layers, stream)
    return subgrids


def degrid_from(nr_subgrids, grid_size, subgrid_size, image_size,
                w_step_in_lambda, nr_channels, nr_stations, uvw, wavenumbers,
                visibilities, spheroidal, aterms, metadata, grid,
                nr_w_layers=1, subgrids=None, stream=None):
    """uv grid -> visibilities: splitter and subgrid FFT (-1, 1/S^2), fused
    for S = 32 / 64 (splitter_fft_launch), then the degridder (overwrites
    the visibility rows of every subgrid)."""
    import torch
    if subgrids is None:
        subgrids = torch.empty((nr_subgrids, 4, subgrid_size, subgrid_size, 2),
                               dtype=torch.float32, device=grid.device)
    splitter_fft_launch(grid_size, metadata, grid, subgrids, nr_w_layers,
                        stream)
    degridder_launch(nr_subgrids, grid_size, subgrid_size, image_size,
                     w_step_in_lambda, nr_channels, nr_stations, uvw,
                     wavenumbers, visibilities, spheroidal, aterms, metadata,
                     subgrids, stream)
    return subgrids


# ---------------------------------------------------------------------------
# Perf entries, device info, work model
# ---------------------------------------------------------------------------
def p_run_gridder():
    """hip::p_run_gridder: env-configured perf run; returns ms per launch."""
    ms = lib.idg_p_run_gridder()
    if ms < 0:
        raise IdgError(-1, "p_run_gridder")
    return ms


def p_run_degridder():
    ms = lib.idg_p_run_degridder()
    if ms < 0:
        raise IdgError(-1, "p_run_degridder")
    return ms


def device_name():
    buf = ctypes.create_string_buffer(256)
    n = lib.idg_get_device_name(buf, 256)
    if n < 0:
        raise IdgError(n, "get_device_name")
    return buf.value.decode()


def kernel_name(direction, subgrid_size, nr_channels):
    d = {"gridder": 0, "degridder": 1}.get(direction, direction)
    return lib.idg_kernel_name(d, subgrid_size, nr_channels).decode()


PRECISION_BITS = {1: "reduction tail on every phasor",
                  2: "blocked summation (f32 master every 16 fills)",
                  4: "reduction tail on one channel per quad"}


def precision_options(direction, subgrid_size, nr_channels):
    """The selected kernels' precision options (include/idg_mi355x.h
    idg_precision_options): (bits, description)."""
    d = {"gridder": 0, "degridder": 1}.get(direction, direction)
    bits = int(lib.idg_precision_options(d, subgrid_size, nr_channels))
    desc = [v for k, v in PRECISION_BITS.items() if bits & k]
    return bits, "; ".join(desc) if desc else "none"


def flops_gridder(nr_channels, nr_timesteps, nr_subgrids, subgrid_size,
                  nr_correlations=NR_CORRELATIONS):
    """Reference work model (app/common/common.cpp:100-129); nr_timesteps is
    the TOTAL number of timesteps, as the reference passes it."""
    return lib.idg_flops_gridder(nr_channels, nr_timesteps, nr_subgrids,
                                 subgrid_size, nr_correlations)


def bytes_gridder(nr_channels, nr_timesteps, nr_subgrids, subgrid_size,
                  nr_correlations=NR_CORRELATIONS):
    return lib.idg_bytes_gridder(nr_channels, nr_timesteps, nr_subgrids,
                                 subgrid_size, nr_correlations)


def abi_version():
    return lib.idg_abi_version()


def release_workspaces(stream=None, all_streams=False):
    """Free the device workspaces the launch entries cache for `stream` (a
    torch stream; None = the current stream) on the current device, or for
    every stream with all_streams=True (include/idg_mi355x.h
    idg_release_workspaces).  The stream must be idle: call it before
    dropping a stream the entries have used."""
    import torch
    if all_streams:
        handle = ctypes.c_void_p(None)
        # every stream's queued launches finished before their slots go
        torch.cuda.synchronize()
    else:
        handle = _stream_handle(stream)
        (stream or torch.cuda.current_stream()).synchronize()
    _check(lib.idg_release_workspaces(handle, 1 if all_streams else 0),
           "idg_release_workspaces")
