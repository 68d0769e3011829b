"""ctypes binding of libidg_mi355x.so (the C ABI in include/idg_mi355x.h).

The library is built in-tree (`make -C ska-sdp-idg-bench_amd`, or
__graft_entry__.build()).  There is no fallback: if the library is missing
or fails to load, importing this module raises.
"""
import ctypes
import os

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# IDG_MI355X_LIB selects another build of the same library (A/B-testing a
# kernel variant); it is read once, at import.
LIB_PATH = os.environ.get("IDG_MI355X_LIB") or os.path.join(
    PKG_DIR, "libidg_mi355x.so")

_P = ctypes.c_void_p
_I = ctypes.c_int
_F = ctypes.c_float
_Z = ctypes.c_size_t
_U64 = ctypes.c_uint64
_D = ctypes.c_double
_S = ctypes.c_char_p

# name -> (restype, argtypes); mirrors include/idg_mi355x.h one to one.
SIGNATURES = {
    "idg_abi_version": (_I, []),
    "idg_last_error": (_S, []),
    "idg_c_run_gridder": (_I, [_I, _I, _I, _F, _F, _I, _I, _P, _Z, _P, _P,
                               _P, _P, _Z, _P, _P]),
    "idg_c_run_degridder": (_I, [_I, _I, _I, _F, _F, _I, _I, _P, _Z, _P, _P,
                                 _P, _P, _Z, _P, _P]),
    "idg_gridder_launch": (_I, [_I, _I, _I, _F, _F, _I, _I, _P, _P, _P, _P,
                                _P, _P, _P, _P]),
    "idg_gridder_fft_launch": (_I, [_I, _I, _I, _F, _F, _I, _I, _P, _P, _P,
                                    _P, _P, _P, _P, _P]),
    "idg_degridder_launch": (_I, [_I, _I, _I, _F, _F, _I, _I, _P, _P, _P, _P,
                                  _P, _P, _P, _P]),
    "idg_validate_metadata": (_I, [_I, _I, _I, _I, _Z, _Z, _P]),
    "idg_host_chunk_plan": (_I, [_I, _P, _Z, _P, _I]),
    "idg_kernel_name": (_S, [_I, _I, _I]),
    "idg_precision_options": (_I, [_I, _I, _I]),
    "idg_p_run_gridder": (_D, []),
    "idg_p_run_degridder": (_D, []),
    "idg_print_device_info": (None, []),
    "idg_print_benchmark": (None, []),
    "idg_get_device_name": (_I, [ctypes.c_char_p, _Z]),
    "idg_flops_gridder": (_U64, [_U64, _U64, _U64, _U64, _U64]),
    "idg_bytes_gridder": (_U64, [_U64, _U64, _U64, _U64, _U64]),
    "idg_generate": (_I, [_I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P,
                          _P, _I]),
    "idg_subgrid_fft_launch": (_I, [_I, _I, _I, _F, _P, _P]),
    "idg_adder_launch": (_I, [_I, _I, _I, _I, _P, _P, _P, _P]),
    "idg_splitter_launch": (_I, [_I, _I, _I, _I, _P, _P, _P, _P]),
    "idg_splitter_fft_launch": (_I, [_I, _I, _I, _I, _P, _P, _P, _P]),
    "idg_release_workspaces": (_I, [_P, _I]),
}


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with "
            "`make -C ska-sdp-idg-bench_amd` (or __graft_entry__.build()); "
            "the MI355X path has no CPU fallback")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()
