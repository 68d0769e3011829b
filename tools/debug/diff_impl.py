"""Debug aid: per-subgrid difference between the MFMA and VALU gridder /
degridder implementations at the full BASELINE config (GPU)."""
import os, sys
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "ska-sdp-idg-bench_amd"))
import idg_amd
print("library:", idg_amd.LIB_PATH)

st, ts, T, C, G, S = 50, 20, 128, int(os.environ.get("DIFF_C", 16)), 1024, int(os.environ.get("DIFF_S", 32))
a = idg_amd.generate(st, ts, T, C, G, S, nthreads=16)
WSTEP = 0.0
if os.environ.get("DIFF_W"):  # w-terms as bench.py's 'wterm' workload
    rng = np.random.default_rng(7)
    a["uvw"][..., 2] = rng.uniform(-200.0, 200.0, a["uvw"].shape[:2])
    a["metadata"]["z"] = rng.integers(0, 7, a["metadata"].size)
    WSTEP = 2.5
ns = a["metadata"].size
dev = {k: torch.from_numpy(a[k]).cuda() for k in ("uvw", "wavenumbers", "visibilities", "spheroidal", "aterms", "subgrids")}
md = torch.from_numpy(a["metadata"].view(np.int32).reshape(-1, 9).copy()).cuda()
p = (ns, G, S, idg_amd.IMAGE_SIZE, WSTEP, C, st)
out = {}
for impl in ("valu", "mfma"):
    os.environ["IDG_GRIDDER_IMPL"] = impl
    os.environ["IDG_DEGRIDDER_IMPL"] = impl
    g = torch.zeros_like(dev["subgrids"]); v = torch.zeros_like(dev["visibilities"])
    idg_amd.gridder_launch(*p, dev["uvw"], dev["wavenumbers"], dev["visibilities"], dev["spheroidal"], dev["aterms"], md, g)
    idg_amd.degridder_launch(*p, dev["uvw"], dev["wavenumbers"], v, dev["spheroidal"], dev["aterms"], md, dev["subgrids"])
    torch.cuda.synchronize()
    out[impl] = (g.double(), v.double())
for k, name in ((0, "gridder"), (1, "degridder")):
    a_, b_ = out["valu"][k], out["mfma"][k]
    diff = (a_ - b_).reshape(ns, -1).abs().max(dim=1).values
    mag = a_.reshape(ns, -1).abs().max(dim=1).values
    rel = (diff / mag).cpu().numpy()
    worst = np.argsort(rel)[::-1][:8]
    print(name, "median rel", np.median(rel), "n>1e-4:", int((rel > 1e-4).sum()))
    for s in worst:
        m = a["metadata"][s]
        print("  s", s, "rel %.3e" % rel[s], "x", m["x"], "y", m["y"], "st", m["station1"], m["station2"])
