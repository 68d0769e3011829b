"""Debug aid (CPU): the gridder's phase-reduction tail, emulated exactly and
accumulated in double, scored in the reference metric (A-term and taper in
double) against exact accumulation of the reference's f32 phases.

  none      r = fma(ph, 1/2pi_hi, -m); only the phase_offset tail restored
            after the sum (round 2)
  block     + c = -k_b phase_index (1/2pi - 1/2pi_hi) added to every r of the
            16-channel block (round 3: one v_pk_add per two phasors)
  mean      no per-phasor add: the pixel's whole tail is restored after the
            sum as one phasor exp(i tau (phase_offset - kbar pidx_bar)),
            kbar the mean wavenumber, pidx_bar the phase index at the
            subgrid's mean (u, v, w)
  sparseN   the block's tail added to one channel quad in N (N x c on quads
            q % N == 0, nothing on the others): the same sum of corrections
            over the block, 1/N of the adds
  altN      the same per channel: N x c on channels k % N == 0

    python tests/emul/tail_mean_emul.py [C] [T]
DESIGN.md §3.3.
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for _p in ("ska-sdp-idg-bench_amd", "oracle", "tools/debug"):
    sys.path.insert(0, os.path.join(REPO, _p))
import idg_amd  # noqa: E402
import oracle as orc  # noqa: E402
from mfma_accum_emul import IH, IH_LO, TAIL, f32, f64, fma32  # noqa: E402


def emulate(C, T, nthreads=8):
    """{model: distance to the exact sum in the reference metric} for the
    two subgrids of the -c geometry at C channels and T timesteps."""
    S, G = 32, 1024
    a = idg_amd.generate(2, 2, T, C, G, S, nthreads=nthreads)
    ns = a["metadata"].size
    img = f32(idg_amd.IMAGE_SIZE)
    k = a["wavenumbers"].astype(f32)
    npix = S * S
    idx = ((np.arange(S) + 0.5 - S / 2) * f64(img) / S).astype(f32)
    l = np.broadcast_to(idx[None, :], (S, S)).astype(f32).ravel()
    m = np.broadcast_to(idx[:, None], (S, S)).astype(f32).ravel()
    at = a["aterms"].reshape(-1, 2, S, S, 4, 2)
    at = at[..., 0].astype(f64) + 1j * at[..., 1]
    sph = a["spheroidal"].reshape(npix).astype(f64)
    models = ("none", "block", "mean", "sparse2", "sparse4", "alt2", "alt4",
              "alt8", "alt16")
    outs = {x: np.zeros((ns, 4, S, S, 2), f32) for x in models + ("exact",)}
    for s in range(ns):
        md = a["metadata"][s]
        su = 2 * np.pi / f64(img)
        uo = f32((int(md["x"]) + S // 2 - G // 2) * su)
        vo = f32((int(md["y"]) + S // 2 - G // 2) * su)
        poff = fma32(uo, l, (vo * m).astype(f32))
        rows = slice(int(md["time_offset"]), int(md["time_offset"]) + T)
        uvw = a["uvw"].reshape(-1, 3)[rows]
        vis = a["visibilities"].reshape(-1, C, 4, 2)[rows]
        V = vis[..., 0].astype(f64) + 1j * vis[..., 1]
        P = {x: np.zeros((npix, 4), complex) for x in models + ("exact",)}
        kb = k[(np.arange(C) // 16) * 16]
        for t in range(T):
            pidx = fma32(uvw[t, 0], l, (uvw[t, 1] * m).astype(f32))
            ph = fma32(-pidx[None, :], k[:, None], poff[None, :])  # [C][npix]
            P["exact"] += np.exp(1j * ph.astype(f64)).T @ V[t]
            A = fma32(-pidx[None, :], kb[:, None], poff[None, :])
            nm = -np.rint((A * IH).astype(f32))
            r0 = fma32(ph, IH, nm)
            cr = (-pidx[None, :] * (kb * IH_LO).astype(f32)[:, None]).astype(f32)
            rb = (r0 + cr).astype(f32)
            quad = (np.arange(C) // 4)[:, None]
            rs2 = np.where(quad % 2 == 0, (r0 + (2 * cr).astype(f32)).astype(f32), r0)
            rs4 = np.where(quad % 4 == 0, (r0 + (4 * cr).astype(f32)).astype(f32), r0)
            ch = np.arange(C)[:, None]
            ra2 = np.where(ch % 2 == 0, (r0 + (2 * cr).astype(f32)).astype(f32), r0)
            ra4 = np.where(ch % 4 == 0, (r0 + (4 * cr).astype(f32)).astype(f32), r0)
            for x, r in (("none", r0), ("block", rb), ("mean", r0),
                         ("sparse2", rs2), ("sparse4", rs4), ("alt2", ra2),
                         ("alt4", ra4),
                         ("alt8", np.where(ch % 8 == 0, (r0 + (8 * cr).astype(f32)).astype(f32), r0)),
                         ("alt16", np.where(ch % 16 == 0, (r0 + (16 * cr).astype(f32)).astype(f32), r0))):
                P[x] += np.exp(2j * np.pi * r.astype(f64)).T @ V[t]
        tail = np.exp(1j * poff.astype(f64) * f64(TAIL))
        ubar, vbar = uvw[:, 0].astype(f64).mean(), uvw[:, 1].astype(f64).mean()
        pbar = ubar * l.astype(f64) + vbar * m.astype(f64)
        kbar = k.astype(f64).mean()
        rot = {"none": tail, "block": tail, "sparse2": tail, "sparse4": tail,
               "alt2": tail, "alt4": tail, "alt8": tail, "alt16": tail,
               "mean": np.exp(1j * f64(TAIL) * (poff.astype(f64) - kbar * pbar))}
        a1 = at[int(md["aterm_index"]), int(md["station1"])].reshape(npix, 2, 2)
        a2 = at[int(md["aterm_index"]), int(md["station2"])].reshape(npix, 2, 2)
        for x in P:
            Px = P[x] * (rot[x][:, None] if x in rot else 1.0)
            Q = np.conj(np.transpose(a1, (0, 2, 1))) @ Px.reshape(npix, 2, 2) @ a2
            Q = Q.reshape(npix, 4) * sph[:, None]
            outs[x][s, ..., 0] = Q.real.T.reshape(4, S, S)
            outs[x][s, ..., 1] = Q.imag.T.reshape(4, S, S)
    o = orc.Oracle()
    return {x: float(o.check_error(outs[x], outs["exact"])[0]) for x in models}


def main():
    C = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 128
    errs = emulate(C, T)
    print(f"C={C} T={T}, 2 subgrids: emulated reduction vs exact "
          "(double sums), reference metric")
    for x, e in errs.items():
        print(f"  {x:7s} {e:.3e}")


if __name__ == "__main__":
    main()
