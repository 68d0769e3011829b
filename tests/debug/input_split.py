"""Debug aid: which input (A-terms / taper) exposes the MFMA-path mismatch."""
import os, sys
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "ska-sdp-idg-bench_amd"))
import idg_amd
print("library:", idg_amd.LIB_PATH)
st, ts, T, C, G, S = 50, 20, 128, 16, 1024, 32
a = idg_amd.generate(st, ts, T, C, G, S, nthreads=16)
ns = a["metadata"].size
md = torch.from_numpy(a["metadata"].view(np.int32).reshape(-1, 9).copy()).cuda()
p = (ns, G, S, idg_amd.IMAGE_SIZE, 0.0, C, st)
base = {k: torch.from_numpy(a[k]).cuda() for k in ("uvw", "wavenumbers", "visibilities", "spheroidal", "aterms", "subgrids")}
ident = np.zeros_like(a["aterms"]); iv = ident.reshape(-1, 4, 2); iv[:, 0, 0] = 1; iv[:, 3, 0] = 1
flat = a["aterms"].reshape(-1, st, S, S, 4, 2)
flat = np.broadcast_to(flat[:, :, :1, :1], flat.shape).copy().reshape(a["aterms"].shape)
variants = {
    "real": (a["aterms"], a["spheroidal"]),
    "ident_aterm": (ident, a["spheroidal"]),
    "unit_sph": (a["aterms"], np.ones_like(a["spheroidal"])),
    "pixel_const_aterm": (flat, np.ones_like(a["spheroidal"])),
    "pixel_const_aterm_real_sph": (flat, a["spheroidal"]),
}
for name, (at, sph) in variants.items():
    atd = torch.from_numpy(np.ascontiguousarray(at)).cuda()
    spd = torch.from_numpy(np.ascontiguousarray(sph)).cuda()
    out = {}
    for impl in ("valu", "mfma"):
        os.environ["IDG_GRIDDER_IMPL"] = impl
        g = torch.zeros_like(base["subgrids"])
        idg_amd.gridder_launch(*p, base["uvw"], base["wavenumbers"], base["visibilities"], spd, atd, md, g)
        torch.cuda.synchronize()
        out[impl] = g.cpu().numpy().reshape(ns, -1).astype(np.float64)
    mag = np.abs(out["valu"]).max(axis=1)
    e = np.abs(out["valu"] - out["mfma"]).max(axis=1) / mag
    print(f"{name:28s} bad(>1e-4) {int((e > 1e-4).sum()):5d}  max {e.max():.2e}")
