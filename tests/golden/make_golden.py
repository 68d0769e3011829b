#!/usr/bin/env python3
"""Generate the golden vectors in tests/golden/ from the REFERENCE's own CPU path.

Runs only in the build container (needs /root/reference): `make -C oracle`
compiles the reference sources where they lie into oracle/_ref/libidgref.so
(with the reference's flags, -O3 -fno-math-errno -march=native), together with
oracle/ref_shim.cpp, which replays exactly what the reference harness does in
run_correctness (tests/gridder_common.cpp:43-124 and
tests/degridder_common.cpp:43-124): srand(0), the initialize_* generators, then
cpu::c_run_gridder_reference / cpu::c_run_degridder_reference.

Each case is written as tests/golden/<case>.npz holding the inputs (as the
reference generated them) and the two reference outputs; manifest.json lists
the parameters.  These files are data (inputs + expected outputs), not source.

    python3 tests/golden/make_golden.py
"""
import ctypes
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))

# name: (nr_stations, nr_timeslots, nr_timesteps, nr_channels, grid_size,
#        subgrid_size)
CASES = {
    # the reference -c defaults (tests/gridder_common.cpp:54-60) = BASELINE
    # configs[0]
    "c_default": (2, 2, 128, 16, 1024, 32),
    # large subgrid (BASELINE configs[4] shape at small NS)
    "s64": (2, 1, 32, 8, 1024, 64),
    # large channel count (BASELINE configs[2] shape at small NS)
    "c256": (2, 1, 16, 256, 1024, 32),
    # several stations/baselines/timeslots: station + time-offset indexing
    "multi": (4, 2, 16, 4, 512, 16),
    # odd subgrid size, odd timestep/channel counts, S^2 not a multiple of 64
    "odd": (3, 2, 7, 3, 256, 33),
}

META = np.dtype([("baseline_offset", "<i4"), ("time_offset", "<i4"),
                 ("nr_timesteps", "<i4"), ("aterm_index", "<i4"),
                 ("station1", "<u4"), ("station2", "<u4"),
                 ("x", "<i4"), ("y", "<i4"), ("z", "<i4")])


def ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def generate(lib, case):
    st, ts, T, C, G, S = CASES[case]
    nbl = st * (st - 1) // 2
    ns = nbl * ts
    uvw = np.zeros((ns, T, 3), np.float32)
    freq = np.zeros(C, np.float32)
    wn = np.zeros(C, np.float32)
    vis_in = np.zeros((ns, T, C, 4, 2), np.float32)
    sph = np.zeros((S, S), np.float32)
    aterms = np.zeros((ts, st, S, S, 4, 2), np.float32)
    md = np.zeros(ns, META)
    sg_in = np.zeros((ns, 4, S, S, 2), np.float32)
    got = lib.ref_generate(st, ts, T, C, G, S, ptr(uvw), ptr(freq), ptr(wn),
                           ptr(vis_in), ptr(sph), ptr(aterms), ptr(md),
                           ptr(sg_in))
    assert got == ns
    img = lib.ref_image_size()
    wstep = lib.ref_w_step()
    grid_out = np.zeros((ns, 4, S, S, 2), np.float32)
    lib.ref_gridder(ns, G, S, ctypes.c_float(img), ctypes.c_float(wstep), C,
                    st, ptr(uvw), ptr(wn), ptr(vis_in), ptr(sph), ptr(aterms),
                    ptr(md), ptr(grid_out))
    degrid_out = np.zeros((ns, T, C, 4, 2), np.float32)
    lib.ref_degridder(ns, G, S, ctypes.c_float(img), ctypes.c_float(wstep), C,
                      st, ptr(uvw), ptr(wn), ptr(degrid_out), ptr(sph),
                      ptr(aterms), ptr(md), ptr(sg_in))
    params = dict(nr_stations=st, nr_timeslots=ts, nr_timesteps=T,
                  nr_channels=C, grid_size=G, subgrid_size=S,
                  nr_subgrids=ns, image_size=float(img),
                  w_step_in_lambda=float(wstep))
    arrays = dict(uvw=uvw, frequencies=freq, wavenumbers=wn,
                  visibilities=vis_in, spheroidal=sph, aterms=aterms,
                  metadata=md.view(np.int32).reshape(ns, 9),
                  subgrids=sg_in, gridder_out=grid_out,
                  degridder_out=degrid_out)
    return params, arrays


def main():
    libpath = os.path.join(REPO, "oracle", "_ref", "libidgref.so")
    if not os.path.exists(libpath):
        sys.exit("build the reference first: make -C oracle")
    lib = ctypes.CDLL(libpath)
    lib.ref_image_size.restype = ctypes.c_float
    lib.ref_w_step.restype = ctypes.c_float
    manifest = {"generator": "oracle/_ref/libidgref.so (reference app/common "
                             "+ app/CPU, g++ -O3 -fno-math-errno "
                             "-march=native) via oracle/ref_shim.cpp",
                "cases": {}}
    for case in CASES:
        params, arrays = generate(lib, case)
        path = os.path.join(HERE, case + ".npz")
        np.savez_compressed(path, **arrays)
        digests = {k: hashlib.sha256(np.ascontiguousarray(v).tobytes())
                   .hexdigest()[:16] for k, v in arrays.items()}
        manifest["cases"][case] = dict(params=params, sha256_16=digests)
        print(f"{case}: NS={params['nr_subgrids']} -> {path} "
              f"({os.path.getsize(path) // 1024} KiB)")
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
