"""Debug aid: where (pixel / correlation) the MFMA gridder differs from VALU."""
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
dev = {k: torch.from_numpy(a[k]).cuda() for k in ("uvw", "wavenumbers", "visibilities", "spheroidal", "aterms", "subgrids")}
md = torch.from_numpy(a["metadata"].view(np.int32).reshape(-1, 9).copy()).cuda()
p = (ns, G, S, idg_amd.IMAGE_SIZE, 0.0, C, st)
res = []
for impl in ("valu", "valu", "mfma", "mfma"):
    os.environ["IDG_GRIDDER_IMPL"] = impl
    g = torch.zeros_like(dev["subgrids"])
    idg_amd.gridder_launch(*p, dev["uvw"], dev["wavenumbers"], dev["visibilities"], dev["spheroidal"], dev["aterms"], md, g)
    torch.cuda.synchronize()
    res.append(g.cpu().numpy().astype(np.float64))
v, v2, m1, m2 = res
os.environ["IDG_GRIDDER_IMPL"] = "mfma"
g = torch.zeros_like(dev["subgrids"])
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(5):
    idg_amd.gridder_launch(*p, dev["uvw"], dev["wavenumbers"], dev["visibilities"], dev["spheroidal"], dev["aterms"], md, g)
e1.record(); torch.cuda.synchronize()
print("mfma gridder ms/launch: %.3f" % (e0.elapsed_time(e1) / 5))
print("valu run-to-run identical:", np.array_equal(v, v2))
print("mfma run-to-run identical:", np.array_equal(m1, m2), "max diff", np.abs(m1 - m2).max())
d = np.abs(v - m1).reshape(ns, 4, S, S, 2).max(axis=-1)   # [s, corr, y, x]
mag = np.abs(v).reshape(ns, -1).max(axis=1)
bad = np.where(d.reshape(ns, -1).max(axis=1) / mag > 1e-4)[0]
print("bad subgrids", len(bad), bad[:10])
for s in bad[:3]:
    ds = d[s] / mag[s]
    yy, xx = np.where(ds.max(axis=0) > 1e-4)
    pix = yy * S + xx
    print("s", s, "bad pixels", len(pix), "corr", np.where(ds.reshape(4, -1).max(axis=1) > 1e-4)[0],
          "pix sample", pix[:12], "base(<512)", int((pix < 512).sum()), "mirror", int((pix >= 512).sum()))

# detail: per bad subgrid, error of the bad tile in base and mirror position
for s in bad[:6]:
    dv = (m1 - v).reshape(ns, 4, S * S, 2)[s] / mag[s]
    worst = np.unravel_index(np.argmax(np.abs(dv)), dv.shape)
    q, p = worst[0], worst[1]
    b = p if p < 512 else S * S - 1 - p
    t0 = (b // 16) * 16
    print(f"s {s} corr {q} tile {t0}: mag {mag[s]:.3g}")
    for name, pix in (("base", np.arange(t0, t0 + 16)), ("mirr", S * S - 1 - np.arange(t0, t0 + 16))):
        for c in range(4):
            e = dv[c, pix]
            print(f"  {name} corr{c} re {np.abs(e[:,0]).max():.2e} im {np.abs(e[:,1]).max():.2e}")
    print("  base err re (x1e4):", np.round(dv[q, t0:t0+16, 0] * 1e4, 2))
    print("  base err im (x1e4):", np.round(dv[q, t0:t0+16, 1] * 1e4, 2))
    print("  run2 same?", np.array_equal(m1[s], m2[s]))
