"""Debug aid: raw D accumulators (IDG_DBG_DUMPD build) run-to-run."""
import os, sys
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "ska-sdp-idg-bench_amd"))
import idg_amd
print("library:", idg_amd.LIB_PATH)
np.set_printoptions(linewidth=160, precision=5)
st, ts, T, C, G, S = 50, 20, 128, 16, 1024, 32
a = idg_amd.generate(st, ts, T, C, G, S, nthreads=16)
ns = a["metadata"].size
md = torch.from_numpy(a["metadata"].view(np.int32).reshape(-1, 9).copy()).cuda()
p = (ns, G, S, idg_amd.IMAGE_SIZE, 0.0, C, st)
dev = {k: torch.from_numpy(a[k]).cuda() for k in ("uvw", "wavenumbers", "visibilities", "spheroidal", "aterms", "subgrids")}
res = []
for r in range(3):
    g = torch.zeros_like(dev["subgrids"])
    idg_amd.gridder_launch(*p, dev["uvw"], dev["wavenumbers"], dev["visibilities"], dev["spheroidal"], dev["aterms"], md, g)
    torch.cuda.synchronize()
    res.append(g.cpu().numpy().reshape(ns, 1, 512, 16))   # [s][gbase0][row][col]
for i, j in ((0, 1), (0, 2), (1, 2)):
    d = res[i] != res[j]
    print(f"runs {i},{j}: differing subgrids", int(d.any(axis=(1, 2, 3)).sum()),
          "cols", np.where(d.any(axis=(0, 1, 2)))[0], "rows mod 64", np.unique(np.where(d.any(axis=(0, 1, 3)))[0] % 64))
hi, lo = res[0][..., :8], res[0][..., 8:]
print("median |lo|/|hi|", np.median(np.abs(lo) / (np.abs(hi) + 1e-30)))
r0 = res[0][0, 0]
print("subgrid0 row0", r0[0], "\nrow1", r0[1])
