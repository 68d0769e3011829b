"""Debug aid: un-A-termed MFMA pixel sums (IDG_DBG_DUMP build)."""
import os, sys
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "ska-sdp-idg-bench_amd"))
import idg_amd
print("library:", idg_amd.LIB_PATH)
np.set_printoptions(linewidth=150, precision=5)
st, ts, T, C, G, S = 50, 20, 128, 16, 1024, 32
a = idg_amd.generate(st, ts, T, C, G, S, nthreads=16)
ns = a["metadata"].size
dev = {k: torch.from_numpy(a[k]).cuda() for k in ("uvw", "wavenumbers", "visibilities", "spheroidal", "aterms", "subgrids")}
md = torch.from_numpy(a["metadata"].view(np.int32).reshape(-1, 9).copy()).cuda()
p = (ns, G, S, idg_amd.IMAGE_SIZE, 0.0, C, st)
res = []
for r in range(2):
    g = torch.zeros_like(dev["subgrids"])
    idg_amd.gridder_launch(*p, dev["uvw"], dev["wavenumbers"], dev["visibilities"], dev["spheroidal"], dev["aterms"], md, g)
    torch.cuda.synchronize()
    res.append(g.cpu().numpy().reshape(ns, 4, S * S, 2).astype(np.float64))
r0, r1 = res
# pols are proportional (gains 1.01..1.04): pol q / pol 0 = g_q / g_0
gains = np.array([1.01, 1.02, 1.03, 1.04])
pred = r0[:, 0:1] * (gains / gains[0])[None, :, None, None]
mag = np.abs(r0).reshape(ns, -1).max(axis=1)
dev_ = np.abs(r0 - pred).max(axis=(2,)) / mag[:, None, None]   # [s, q, re/im]
print("max deviation from proportionality per pol/re-im (over subgrids):\n", dev_.max(axis=0))
badq = np.where(dev_.max(axis=(1, 2)) > 1e-4)[0]
print("subgrids non-proportional:", len(badq), badq[:10])
d = (r0 != r1)
print("run-to-run differing subgrids:", int(d.any(axis=(1, 2, 3)).sum()))
s = badq[0] if len(badq) else 0
e = np.abs(r0[s] - pred[s]) / mag[s]
pix = np.where(e.max(axis=(0, 2)) > 1e-4)[0]
print("subgrid", s, "bad pixels", pix, "pols", np.where(e.max(axis=(1, 2)) > 1e-4)[0], "re/im", np.where(e.max(axis=(0, 1)) > 1e-4)[0])
for pp in pix[:4]:
    print(" pix", pp, "pols re:", r0[s, :, pp, 0] / gains, " im:", r0[s, :, pp, 1] / gains)

# exact (float64) pre-A-term pixel sums for a few subgrids
IS = idg_amd.IMAGE_SIZE
md_np = a["metadata"]
uvw = a["uvw"].reshape(-1, 3).astype(np.float64)
vis = a["visibilities"].reshape(-1, C, 4, 2).astype(np.float64)
vis = vis[..., 0] + 1j * vis[..., 1]
k = a["wavenumbers"].astype(np.float64)
x = np.arange(S)
lx = (x + 0.5 - S // 2) * IS / S
L = np.tile(lx, S)            # pixel p = y*S + x
M = np.repeat(lx, S)
bo0 = int(md_np["baseline_offset"][0])
for s in [0] + list(badq[1:3]):
    m = md_np[s]
    t0 = int(m["baseline_offset"]) - bo0 + int(m["time_offset"])
    nt = int(m["nr_timesteps"])
    sc = 2 * np.pi / IS
    uo = (int(m["x"]) + S // 2 - G // 2) * sc
    vo = (int(m["y"]) + S // 2 - G // 2) * sc
    poff = uo * L + vo * M
    acc = np.zeros((4, S * S), complex)
    for t in range(nt):
        u, v = uvw[t0 + t, 0], uvw[t0 + t, 1]
        pidx = u * L + v * M
        ph = np.exp(1j * (poff[None, :] - pidx[None, :] * k[:, None]))   # [C, P]
        acc += (vis[t0 + t].T @ ph)                                        # [4, P]
    got = r0[s, :, :, 0] + 1j * r0[s, :, :, 1]
    err = np.abs(got - acc).max(axis=1) / np.abs(acc).max()
    print("subgrid", s, "exact-vs-dump rel err per pol", err)
