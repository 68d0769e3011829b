"""Debug aid: IDG_DBG_PROBE build stores (A2[yx].im, tmp[3].im) in corr 3."""
import os, sys
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "ska-sdp-idg-bench_amd"))
import idg_amd
print("library:", idg_amd.LIB_PATH)
np.set_printoptions(linewidth=160, precision=6)
st, ts, T, C, G, S = 50, 20, 128, 16, 1024, 32
a = idg_amd.generate(st, ts, T, C, G, S, nthreads=16)
ns = a["metadata"].size
md = torch.from_numpy(a["metadata"].view(np.int32).reshape(-1, 9).copy()).cuda()
p = (ns, G, S, idg_amd.IMAGE_SIZE, 0.0, C, st)
dev = {k: torch.from_numpy(a[k]).cuda() for k in ("uvw", "wavenumbers", "visibilities", "spheroidal", "aterms", "subgrids")}
def run(impl):
    os.environ["IDG_GRIDDER_IMPL"] = impl
    g = torch.zeros_like(dev["subgrids"])
    idg_amd.gridder_launch(*p, dev["uvw"], dev["wavenumbers"], dev["visibilities"], dev["spheroidal"], dev["aterms"], md, g)
    torch.cuda.synchronize()
    r = g.cpu().numpy().reshape(ns, 4, S * S, 2).astype(np.float64)
    return r
V = run("valu"); M = run("mfma")
mag = np.abs(V[:, :3]).reshape(ns, -1).max(axis=1)
e2 = np.abs(M[:, 2, :, 0] - V[:, 2, :, 0]) / mag[:, None]
bad = np.argwhere(e2 > 1e-4)
print("bad corr2-re entries", len(bad))
d3 = np.abs(M[:, 3] - V[:, 3]).max(axis=-1)
print("probe (a22im, t3im) mfma vs valu: max abs diff", d3.max(), " at bad entries:", d3[bad[:, 0], bad[:, 1]].max() if len(bad) else None)
for s, pix in bad[:5]:
    print(s, pix, "valu probe", V[s, 3, pix], "mfma probe", M[s, 3, pix], "corr2 re valu", V[s, 2, pix, 0], "mfma", M[s, 2, pix, 0])
