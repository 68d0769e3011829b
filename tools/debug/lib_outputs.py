"""Gridder and degridder outputs of the library IDG_MI355X_LIB selects, on a
few fixed batches (C = 16 and 256, a w-term mix, ragged subgrids), saved
to one .npz: run once per A/B library, then compare the files bit for bit.
    IDG_MI355X_LIB=ab/x.so python tools/debug/lib_outputs.py OUT.npz
    python tools/debug/lib_outputs.py --compare A.npz B.npz"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "ska-sdp-idg-bench_amd"))


def compare(a, b):
    x, y = np.load(a), np.load(b)
    bad = 0
    for k in sorted(x.files):
        same = np.array_equal(x[k].view(np.uint32), y[k].view(np.uint32))
        print(f"{k:24s} {'bitwise equal' if same else 'DIFFERENT'}")
        bad += not same
    return bad


def main():
    if sys.argv[1] == "--compare":
        raise SystemExit(1 if compare(sys.argv[2], sys.argv[3]) else 0)
    import torch
    import idg_amd
    out = {}
    cases = {"c16": (20, 8, 128, 16, 1024, 32), "c256": (6, 4, 128, 256, 1024, 32),
             "s64": (8, 4, 64, 16, 1024, 64)}
    for name, (st, ts, T, C, G, S) in cases.items():
        a = idg_amd.generate(st, ts, T, C, G, S, nthreads=8)
        md = a["metadata"].copy()
        ns = md.size
        rng = np.random.default_rng(5)
        # a w-term on every third subgrid (general path), ragged counts
        a["uvw"][::3, :, 2] = rng.uniform(-50, 50, a["uvw"][::3, :, 2].shape)
        md["nr_timesteps"][1::7] = T // 2 + 3
        dev = {k: torch.from_numpy(np.ascontiguousarray(a[k])).cuda()
               for k in ("uvw", "wavenumbers", "visibilities", "spheroidal",
                         "aterms", "subgrids")}
        dmd = torch.from_numpy(md.view(np.int32).reshape(-1, 9).copy()).cuda()
        p = (ns, G, S, idg_amd.IMAGE_SIZE, 0.0, C, st)
        g = torch.zeros_like(dev["subgrids"])
        idg_amd.gridder_launch(*p, dev["uvw"], dev["wavenumbers"],
                               dev["visibilities"], dev["spheroidal"],
                               dev["aterms"], dmd, g)
        d = torch.zeros_like(dev["visibilities"])
        idg_amd.degridder_launch(*p, dev["uvw"], dev["wavenumbers"], d,
                                 dev["spheroidal"], dev["aterms"], dmd,
                                 dev["subgrids"])
        torch.cuda.synchronize()
        out[f"{name}_gridder"] = g.cpu().numpy()
        out[f"{name}_degridder"] = d.cpu().numpy()
    np.savez(sys.argv[1], **out)
    print("saved", sys.argv[1], os.environ.get("IDG_MI355X_LIB", "default"))


if __name__ == "__main__":
    main()
