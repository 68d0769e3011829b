"""Debug aid (GPU box): the gridder's distance to exact accumulation for one
library build (IDG_MI355X_LIB selects it), at the -c defaults and at
-c NR_CHANNELS=256 (T = 128).  Prints one JSON line per configuration and direction
(IDG_PREC=<0..3> forces the kernels' precision options, util.hpp):
ours_vs_exact / ref_vs_exact in the reference metric, plus the error of the
largest pixels split into a coherent amplitude part (mean Re((o-e) e*)/|e|^2),
a coherent phase part (the Im of the same) and the rest.  DESIGN.md §3.1.

    python tools/debug/accuracy_ab.py [tag]
"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for _p in ("ska-sdp-idg-bench_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(REPO, _p))
import idg_amd  # noqa: E402
import oracle as orc  # noqa: E402

CONFIGS = {"c_default": (2, 2, 128, 16), "c256": (2, 2, 128, 256)}


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else os.path.basename(
        os.environ.get("IDG_MI355X_LIB", "head"))
    tag += f" IDG_PREC={os.environ.get('IDG_PREC', 'default')}"
    o = orc.Oracle()
    ref_lib = orc.Reference(portable=True) if orc.Reference.available(
        portable=True) else o
    for name, (st, ts, T, C) in CONFIGS.items():
        G, S = 1024, 32
        a = idg_amd.generate(st, ts, T, C, G, S, nthreads=8)
        ns = a["metadata"].size
        args = (ns, G, S, idg_amd.IMAGE_SIZE, idg_amd.W_STEP, C, st)
        ins = (a["uvw"], a["wavenumbers"], a["visibilities"], a["spheroidal"],
               a["aterms"], a["metadata"])
        ours = np.zeros((ns, 4, S, S, 2), np.float32)
        idg_amd.c_run_gridder(*args, *ins, ours)
        ref = np.zeros_like(ours)
        ref_lib.gridder(*args, *ins, ref)
        exact = np.zeros(ours.shape, np.float64)
        o.gridder_exact(*args, *ins, exact, nthreads=8)
        e32 = exact.astype(np.float32)
        oc = ours[..., 0].astype(np.float64) + 1j * ours[..., 1]
        ec = exact[..., 0] + 1j * exact[..., 1]
        big = np.abs(ec) > 0.25 * np.abs(ec).max()
        rel = ((oc - ec) * np.conj(ec))[big] / (np.abs(ec[big]) ** 2)
        rec = {
            "tag": tag, "config": name, "direction": "gridder",
            "ours_vs_exact": float(o.check_error(ours, e32)[0]),
            "ref_vs_exact": float(o.check_error(ref, e32)[0]),
            "ours_vs_ref": float(o.check_error(ours, ref)[0]),
            "big_pixels": int(big.sum()),
            "big_amp_bias": float(rel.real.mean()),
            "big_phase_bias": float(rel.imag.mean()),
            "big_rel_rms": float(np.sqrt(np.mean(np.abs(rel) ** 2))),
        }
        print(json.dumps(rec), flush=True)
        # the degridder, on the reference's own degridder input subgrids
        vo = np.zeros_like(a["visibilities"])
        idg_amd.c_run_degridder(*args, a["uvw"], a["wavenumbers"], vo,
                                a["spheroidal"], a["aterms"], a["metadata"],
                                a["subgrids"])
        vr = np.zeros_like(vo)
        ref_lib.degridder(*args, a["uvw"], a["wavenumbers"], vr,
                          a["spheroidal"], a["aterms"], a["metadata"],
                          a["subgrids"])
        vx = np.zeros(vo.shape, np.float64)
        o.degridder_exact(*args, a["uvw"], a["wavenumbers"], vx,
                          a["spheroidal"], a["aterms"], a["metadata"],
                          a["subgrids"], nthreads=8)
        vx32 = vx.astype(np.float32)
        print(json.dumps({
            "tag": tag, "config": name, "direction": "degridder",
            "ours_vs_exact": float(o.check_error(vo, vx32)[0]),
            "ref_vs_exact": float(o.check_error(vr, vx32)[0]),
            "ours_vs_ref": float(o.check_error(vo, vr)[0])}), flush=True)


if __name__ == "__main__":
    main()
