"""Accuracy of the blocked summation's flush interval (IDG_FLUSH_FILLS, a
build option): the C = 256 gridder at the harness' -c shape (T = 128, 2
subgrids) and at 4 sampled subgrids of configs[2]-like data, against the
exact (double) sum of the reference's own f32 phases, in the reference
metric.  Run once per library: IDG_MI355X_LIB=ab/x.so python
tools/debug/flush_ab.py TAG -> one JSON line."""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "ska-sdp-idg-bench_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))


def main():
    import idg_amd
    import oracle
    o = oracle.Oracle()
    out = {"tag": sys.argv[1] if len(sys.argv) > 1 else "",
           "lib": os.environ.get("IDG_MI355X_LIB", "default")}
    for name, (st, ts) in (("c_shape", (2, 2)), ("four_baselines", (3, 2))):
        T, C, G, S = 128, 256, 1024, 32
        a = idg_amd.generate(st, ts, T, C, G, S, nthreads=8)
        ns = a["metadata"].size
        args = (ns, G, S, idg_amd.IMAGE_SIZE, idg_amd.W_STEP, C, st)
        ours = np.zeros((ns, 4, S, S, 2), np.float32)
        idg_amd.c_run_gridder(*args, a["uvw"], a["wavenumbers"],
                              a["visibilities"], a["spheroidal"], a["aterms"],
                              a["metadata"], ours)
        exact = np.zeros(ours.shape, np.float64)
        o.gridder_exact(*args, a["uvw"], a["wavenumbers"], a["visibilities"],
                        a["spheroidal"], a["aterms"], a["metadata"], exact,
                        nthreads=16)
        out[name] = float(o.check_error(ours, exact.astype(np.float32))[0])
    out["precision"] = idg_amd.precision_options("gridder", 32, 256)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
