"""Debug aid: raw-P dump build vs identity-A-term normal build (both = P).
usage: IDG_DEBUG_LIB=... python dump_vs_ident.py MODE OUT.npy   (MODE ident|real)"""
import os, sys
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "ska-sdp-idg-bench_amd"))
import idg_amd
print("library:", idg_amd.LIB_PATH)
mode, outp = sys.argv[1], sys.argv[2]
st, ts, T, C, G, S = 50, 20, 128, 16, 1024, 32
a = idg_amd.generate(st, ts, T, C, G, S, nthreads=16)
ns = a["metadata"].size
md = torch.from_numpy(a["metadata"].view(np.int32).reshape(-1, 9).copy()).cuda()
p = (ns, G, S, idg_amd.IMAGE_SIZE, 0.0, C, st)
dev = {k: torch.from_numpy(a[k]).cuda() for k in ("uvw", "wavenumbers", "visibilities", "spheroidal", "aterms", "subgrids")}
at, sph = dev["aterms"], dev["spheroidal"]
if mode == "ident":
    ident = np.zeros_like(a["aterms"]); iv = ident.reshape(-1, 4, 2); iv[:, 0, 0] = 1; iv[:, 3, 0] = 1
    at = torch.from_numpy(ident).cuda(); sph = torch.ones_like(sph)
g = torch.zeros_like(dev["subgrids"])
idg_amd.gridder_launch(*p, dev["uvw"], dev["wavenumbers"], dev["visibilities"], sph, at, md, g)
torch.cuda.synchronize()
np.save(outp, g[:200].cpu().numpy())
