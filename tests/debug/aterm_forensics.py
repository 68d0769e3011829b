"""Debug aid: for mismatching pixels, which wrong formula reproduces the MFMA
output (P from an identity-A-term run, A-terms applied in numpy)."""
import itertools, os, sys
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
ident = np.zeros_like(a["aterms"]); iv = ident.reshape(-1, 4, 2); iv[:, 0, 0] = 1; iv[:, 3, 0] = 1
ones = torch.ones_like(dev["spheroidal"])
def run(impl, at):
    os.environ["IDG_GRIDDER_IMPL"] = impl
    g = torch.zeros_like(dev["subgrids"])
    idg_amd.gridder_launch(*p, dev["uvw"], dev["wavenumbers"], dev["visibilities"], ones,
                           torch.from_numpy(at).cuda(), md, g)
    torch.cuda.synchronize()
    r = g.cpu().numpy().reshape(ns, 4, S * S, 2).astype(np.float64)
    return r[..., 0] + 1j * r[..., 1]
P = run("valu", ident)
V = run("valu", a["aterms"])
M = run("mfma", a["aterms"])
mag = np.abs(V).reshape(ns, -1).max(axis=1)
err = np.abs(M - V) / mag[:, None, None]
bad = np.argwhere(err > 1e-4)
print("bad (s, corr, pix) count", len(bad), "corr hist", np.bincount(bad[:, 1], minlength=4))
at = a["aterms"].reshape(-1, st, S, S, 4, 2)
at = at[..., 0] + 1j * at[..., 1]
def aterm(Pv, A1, A2):
    Pm = Pv.reshape(2, 2); return (A1.reshape(2, 2).conj().T @ Pm @ A2.reshape(2, 2)).reshape(4)
shown = 0
for s, q, pix in bad[:400]:
    m = a["metadata"][s]
    y, x = divmod(int(pix), S)
    A1 = at[int(m["aterm_index"]), int(m["station1"]), y, x]
    A2 = at[int(m["aterm_index"]), int(m["station2"]), y, x]
    Pv = P[s, :, pix]
    ref = aterm(Pv, A1, A2)
    got = M[s, q, pix]
    hyp = {}
    for perm in itertools.permutations(range(4)):
        hyp[f"Pperm{perm}"] = aterm(Pv[list(perm)], A1, A2)[q]
    hyp["A1=A2=A1"] = aterm(Pv, A1, A1)[q]
    hyp["A1=A2=A2"] = aterm(Pv, A2, A2)[q]
    hyp["swapA"] = aterm(Pv, A2, A1)[q]
    for k in range(4):
        Pz = Pv.copy(); Pz[k] = 0; hyp[f"P{k}=0"] = aterm(Pz, A1, A2)[q]
    best = sorted(hyp.items(), key=lambda kv: abs(kv[1].real - got.real))[:3]
    if shown < 6:
        print(f"s {s} corr {q} pix {pix}: valu {ref[q]:.6f} (gpu-valu {V[s,q,pix]:.6f}) mfma {got:.6f}")
        print("   P", Pv, "\n   best re-match:", [(k, f"{v:.6f}") for k, v in best])
        shown += 1

print("---- partial products / cross-pixel hypotheses ----")
shown = 0
for s, q, pix in bad[:400]:
    if q != 2 or shown >= 6:
        continue
    shown += 1
    m = a["metadata"][s]
    y, x = divmod(int(pix), S)
    A1 = at[int(m["aterm_index"]), int(m["station1"]), y, x]
    A2 = at[int(m["aterm_index"]), int(m["station2"]), y, x]
    Pv = P[s, :, pix]
    a1h = A1.reshape(2, 2).conj().T
    tmp = (a1h @ Pv.reshape(2, 2)).reshape(4)
    terms = {"t2r*A20r": tmp[2].real * A2[0].real, "t2i*A20i": -tmp[2].imag * A2[0].imag,
             "t3r*A22r": tmp[3].real * A2[2].real, "t3i*A22i": -tmp[3].imag * A2[2].imag}
    d = M[s, q, pix].real - V[s, q, pix].real
    print(f"s {s} pix {pix} delta {d:.6f} terms", {k: round(v, 6) for k, v in terms.items()})
    # P from another pixel, A from this pixel
    cands = []
    for pp in range(S * S):
        o = (A1.reshape(2, 2).conj().T @ P[s, :, pp].reshape(2, 2) @ A2.reshape(2, 2)).reshape(4)[2]
        cands.append((abs(o.real - M[s, q, pix].real), pp, "P@"))
        yy, xx = divmod(pp, S)
        B1 = at[int(m["aterm_index"]), int(m["station1"]), yy, xx]
        B2 = at[int(m["aterm_index"]), int(m["station2"]), yy, xx]
        o = (B1.reshape(2, 2).conj().T @ Pv.reshape(2, 2) @ B2.reshape(2, 2)).reshape(4)[2]
        cands.append((abs(o.real - M[s, q, pix].real), pp, "A@"))
    cands.sort()
    print("   closest cross-pixel:", [(f"{c[0]:.2e}", c[1], c[2]) for c in cands[:3]])
