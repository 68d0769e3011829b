"""Debug aid: MFMA gridder with identity A-terms and unit taper (raw pixel
sums) vs VALU and the oracle; proportionality across correlations."""
import os, sys
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "ska-sdp-idg-bench_amd"))
sys.path.insert(0, REPO)
import idg_amd
print("library:", idg_amd.LIB_PATH)
from oracle.oracle import Oracle
np.set_printoptions(linewidth=150, precision=5)
st, ts, T, C, G, S = 50, 20, 128, 16, 1024, 32
a = idg_amd.generate(st, ts, T, C, G, S, nthreads=16)
a["aterms"][:] = 0
at = a["aterms"].reshape(-1, 4, 2)
at[:, 0, 0] = 1.0
at[:, 3, 0] = 1.0
a["spheroidal"][:] = 1.0
ns = a["metadata"].size
dev = {k: torch.from_numpy(a[k]).cuda() for k in ("uvw", "wavenumbers", "visibilities", "spheroidal", "aterms", "subgrids")}
md = torch.from_numpy(a["metadata"].view(np.int32).reshape(-1, 9).copy()).cuda()
p = (ns, G, S, idg_amd.IMAGE_SIZE, 0.0, C, st)
res = {}
for name, impl in (("valu", "valu"), ("m1", "mfma"), ("m2", "mfma")):
    os.environ["IDG_GRIDDER_IMPL"] = impl
    g = torch.zeros_like(dev["subgrids"])
    idg_amd.gridder_launch(*p, dev["uvw"], dev["wavenumbers"], dev["visibilities"], dev["spheroidal"], dev["aterms"], md, g)
    torch.cuda.synchronize()
    res[name] = g.cpu().numpy().reshape(ns, 4, S * S, 2).astype(np.float64)
gains = np.array([1.01, 1.02, 1.03, 1.04])
mag = np.abs(res["valu"]).reshape(ns, -1).max(axis=1)
for name, r in res.items():
    pred = r[:, 0:1] * (gains / gains[0])[None, :, None, None]
    dv = (np.abs(r - pred).max(axis=2) / mag[:, None, None])
    e = np.abs(r - res["valu"]).reshape(ns, -1).max(axis=1) / mag
    print(name, "non-proportional subgrids", int((dv.max(axis=(1, 2)) > 1e-4).sum()),
          "| vs valu >1e-4:", int((e > 1e-4).sum()), "max", e.max())
orc = Oracle()
sel = list(range(64)) + list(np.where(np.abs(res["m1"] - res["valu"]).reshape(ns, -1).max(axis=1) / mag > 1e-4)[0][:16])
for s in sel[60:]:
    go = np.zeros((1, 4, S, S, 2), np.float32)
    orc.gridder(1, G, S, idg_amd.IMAGE_SIZE, 0.0, C, st, a["uvw"], a["wavenumbers"], a["visibilities"],
                a["spheroidal"], a["aterms"], a["metadata"][s:s + 1], go)
    go = go.reshape(4, S * S, 2).astype(np.float64)
    ev = np.abs(res["valu"][s] - go).max() / mag[s]
    em = np.abs(res["m1"][s] - go).max() / mag[s]
    print(f"s {s}: valu-vs-oracle {ev:.2e}  mfma-vs-oracle {em:.2e}")
