"""Debug aid (CPU): the gridder of one subgrid with the reference's f32
phase rounding but fp64 accumulation, to separate accumulation error from
phase error.  Compares the oracle and saved GPU outputs against it."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "ska-sdp-idg-bench_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import idg_amd
import oracle as orc

f32 = np.float32


def fma32(a, b, c):
    return (np.float64(a) * np.float64(b) + np.float64(c)).astype(f32)


def grid_fp64(a, s, G, S, C, img=float(np.float32(0.01))):
    m = a["metadata"][s]
    T = int(m["nr_timesteps"])
    rows = slice(int(m["time_offset"]), int(m["time_offset"]) + T)
    uvw = a["uvw"].reshape(-1, 3)[rows]
    vis = a["visibilities"].reshape(-1, C, 4, 2)[rows]
    vis = vis[..., 0].astype(np.float64) + 1j * vis[..., 1]
    k = a["wavenumbers"]
    idx = (np.arange(S) + 0.5 - S // 2) * img / S
    lm = idx.astype(f32)
    l = lm[None, :].repeat(S, 0)
    mm = lm[:, None].repeat(S, 1)
    scale = 2 * np.pi / img
    uo = f32((int(m["x"]) + S // 2 - G // 2) * scale)
    vo = f32((int(m["y"]) + S // 2 - G // 2) * scale)
    poff = fma32(uo, l, (vo * mm).astype(f32))        # w_offset = 0
    P = np.zeros((4, S, S), complex)
    for t in range(T):
        u, v = uvw[t, 0], uvw[t, 1]
        pidx = fma32(u, l, (v * mm).astype(f32))       # w = 0
        for c in range(C):
            ph = fma32(-pidx, k[c], poff).astype(np.float64)
            phasor = np.cos(ph) + 1j * np.sin(ph)
            P += vis[t, c][:, None, None] * phasor[None]
    A = a["aterms"]
    A = A[..., 0].astype(np.float64) + 1j * A[..., 1]   # [ts][st][S][S][4]
    a1 = A[int(m["aterm_index"]), int(m["station1"])]
    a2 = A[int(m["aterm_index"]), int(m["station2"])]
    J = lambda q: q.reshape(S, S, 2, 2)
    Pm = np.moveaxis(P, 0, -1).reshape(S, S, 2, 2)
    out = np.conj(np.swapaxes(J(a1), -1, -2)) @ Pm @ J(a2)
    out = out.reshape(S, S, 4) * a["spheroidal"][..., None]
    return np.moveaxis(out, -1, 0)


def err(cand, ref):
    return np.sqrt((np.abs(cand - ref) ** 2).sum() / (np.abs(ref) ** 2).sum())


if __name__ == "__main__":
    C = int(os.environ.get("C", 256))
    st, ts, T, G, S = 50, 1, 128, 1024, 32
    a = idg_amd.generate(st, ts, T, C, G, S, nthreads=8)
    print("aterms shape", a["aterms"].shape)
    path = os.path.join(REPO, "gpurun_out", f"c{C}_grid.npz")
    saved = np.load(path) if os.path.exists(path) else None
    o = orc.Oracle()
    for s in (0, 1):
        ref = grid_fp64(a, s, G, S, C)
        go = np.zeros((1, 4, S, S, 2), f32)
        o.gridder(1, G, S, 0.01, 0.0, C, st, a["uvw"], a["wavenumbers"],
                  a["visibilities"], a["spheroidal"], a["aterms"],
                  a["metadata"][s:s + 1], go)
        cz = lambda x: x[0, ..., 0].astype(np.float64) + 1j * x[0, ..., 1]
        msg = "subgrid %d oracle vs fp64 %.3e" % (s, err(cz(go), ref))
        if saved is not None:
            msg += " valu vs fp64 %.3e mfma vs fp64 %.3e" % (
                err(cz(saved[f"valu_{s}"]), ref),
                err(cz(saved[f"mfma_{s}"]), ref))
        print(msg)
