"""PCIe-inclusive rate of the host-buffer boundary (idg_c_run_gridder /
idg_c_run_degridder: allocate, copy in, launch, copy out, free -- the
reference's c_run_* contract, app/HIP/util.cpp:255-311) at BASELINE
configs[1], beside the resident-data kernel time.  Prints one JSON line.
  python tools/debug/host_rate.py [--reps 3]"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "ska-sdp-idg-bench_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import numpy as np
    import idg_amd
    import bench
    w = bench.workload("default")
    a = bench.make_batch(w, nthreads=16)
    ns = a["metadata"].size
    T, C, S = w["nr_timesteps"], w["nr_channels"], w["subgrid_size"]
    p = (ns, w["grid_size"], S, idg_amd.IMAGE_SIZE, idg_amd.W_STEP, C,
         w["nr_stations"])
    nvis = ns * T * C
    sub = np.zeros_like(a["subgrids"])
    vis = np.zeros_like(a["visibilities"])
    out = {"workload": "configs[1]", "nvis": nvis,
           "bytes_in_gridder": int(a["visibilities"].nbytes + a["uvw"].nbytes),
           "bytes_out_gridder": int(sub.nbytes),
           "bytes_in_degridder": int(a["subgrids"].nbytes + vis.nbytes),
           "bytes_out_degridder": int(vis.nbytes)}
    for name, fn, args_ in (
            ("gridder", idg_amd.c_run_gridder,
             (a["uvw"], a["wavenumbers"], a["visibilities"], a["spheroidal"],
              a["aterms"], a["metadata"], sub)),
            ("degridder", idg_amd.c_run_degridder,
             (a["uvw"], a["wavenumbers"], vis, a["spheroidal"], a["aterms"],
              a["metadata"], a["subgrids"]))):
        ts = []
        for _ in range(args.reps + 1):  # the first call pays HIP init
            t0 = time.perf_counter()
            fn(*p, *args_)
            ts.append(time.perf_counter() - t0)
        t = min(ts[1:])
        out[name] = {"ms": round(t * 1e3, 2), "mvis_s": round(nvis / t / 1e6, 1),
                     "all_ms": [round(x * 1e3, 2) for x in ts]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
