"""Debug aid: C = 256 parity of MFMA and VALU kernels vs the oracle on a
few subgrids (GPU)."""
import os, sys
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "ska-sdp-idg-bench_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import idg_amd
import oracle as orc

st, ts, T, G, S = 50, 1, 128, 1024, 32
C = int(os.environ.get("C", 256))
a = idg_amd.generate(st, ts, T, C, G, S, nthreads=16)
ns = a["metadata"].size
dev = {k: torch.from_numpy(a[k]).cuda() for k in ("uvw", "wavenumbers", "visibilities", "spheroidal", "aterms", "subgrids")}
md = torch.from_numpy(a["metadata"].view(np.int32).reshape(-1, 9).copy()).cuda()
p = (ns, G, S, idg_amd.IMAGE_SIZE, 0.0, C, st)
o = orc.Oracle()
samples = (0, 1, 2, 600)
ref_g, ref_d = {}, {}
for s in samples:
    m = a["metadata"][s:s + 1]
    go = np.zeros((1, 4, S, S, 2), np.float32)
    o.gridder(1, G, S, idg_amd.IMAGE_SIZE, 0.0, C, st, a["uvw"], a["wavenumbers"], a["visibilities"], a["spheroidal"], a["aterms"], m, go)
    ref_g[s] = go
    m0 = m.copy(); m0["time_offset"] = 0
    do = np.zeros((1, T, C, 4, 2), np.float32)
    o.degridder(1, G, S, idg_amd.IMAGE_SIZE, 0.0, C, st, np.ascontiguousarray(a["uvw"][s]), a["wavenumbers"], do, a["spheroidal"], a["aterms"], m0, np.ascontiguousarray(a["subgrids"][s:s + 1]))
    ref_d[s] = do
saved = {}
for impl in ("valu", "mfma"):
    os.environ["IDG_GRIDDER_IMPL"] = impl
    os.environ["IDG_DEGRIDDER_IMPL"] = impl
    g = torch.zeros_like(dev["subgrids"]); v = torch.zeros_like(dev["visibilities"])
    idg_amd.gridder_launch(*p, dev["uvw"], dev["wavenumbers"], dev["visibilities"], dev["spheroidal"], dev["aterms"], md, g)
    idg_amd.degridder_launch(*p, dev["uvw"], dev["wavenumbers"], v, dev["spheroidal"], dev["aterms"], md, dev["subgrids"])
    torch.cuda.synchronize()
    for s in samples:
        eg = o.check_error(g[s:s + 1].cpu().numpy(), ref_g[s])[0]
        ed = o.check_error(v[s:s + 1].cpu().numpy(), ref_d[s])[0]
        print(impl, "C", C, "subgrid", s, "gridder %.3e degridder %.3e" % (eg, ed))
        saved[f"{impl}_{s}"] = g[s:s + 1].cpu().numpy()
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(REPO, "gpurun_out", f"c{C}_grid.npz"), **saved)
