"""Debug aid (CPU): numpy emulation of the mirror MFMA gridder's arithmetic on
one subgrid of the -c NR_CHANNELS=256 case (T = 128), scored in the
reference metric against exact accumulation of the reference's f32 phases.
Each model changes one ingredient, so the error budget can be read off:

  phasor    exact f32 reference phase -> kernel's r = fma(ph, 1/2pi_hi, -m)
            + c -> cos/sin (correctly rounded f32), unsplit, sums in double
  split     + the two-term f16 split of the phasor and of the scaled
            visibilities, sums in double
  rne       + one round-to-nearest-even f32 rounding per MFMA (K-step)
  rtz       + one round-toward-zero rounding per MFMA instead
  seq       + the 32 products of a K-step added to the accumulator one at a
            time in f32 (RNE)
  flushN    rne, but the accumulator is added to an f32 master and cleared
            every N K-steps (blocked summation)

    python tools/debug/mfma_accum_emul.py [C] [subgrid]
DESIGN.md §3.1.
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for _p in ("ska-sdp-idg-bench_amd", "oracle", "tests", "tools/debug"):
    sys.path.insert(0, os.path.join(REPO, _p))
import idg_amd  # noqa: E402
import oracle as orc  # noqa: E402

f32, f16, f64 = np.float32, np.float16, np.float64
IH = f32(float.fromhex("0x1.45f306p-3"))
IH_LO = f32(float.fromhex("0x1.b9391p-28"))
TAIL = f32(float.fromhex("0x1.5a892p-25"))


def fma32(a, b, c):
    return (f64(a) * f64(b) + f64(c)).astype(f32)


def split(x):
    """(hi, lo) of f32 x as float64 values of f16 numbers."""
    x = np.asarray(x, f32)
    hi = x.astype(f16).astype(f32)
    lo = (x - hi).astype(f16)  # x - hi exact in f32
    return hi.astype(f64), lo.astype(f64)


def rtz32(x):
    r = x.astype(f32)
    over = np.abs(r.astype(f64)) > np.abs(x)
    r[over] = np.nextafter(r[over], f32(0))
    return r


def main():
    C = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    s = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    T, S, G = 128, 32, 1024
    a = idg_amd.generate(2, 2, T, C, G, S, nthreads=8)
    img = f32(idg_amd.IMAGE_SIZE)
    k = a["wavenumbers"].astype(f32)
    md = a["metadata"][s]
    npix, half = S * S, S * S // 2
    idx = ((np.arange(S) + 0.5 - S / 2) * f64(img) / S).astype(f32)
    l = np.broadcast_to(idx[None, :], (S, S)).astype(f32).ravel()
    m = np.broadcast_to(idx[:, None], (S, S)).astype(f32).ravel()
    scale_uv = 2 * np.pi / f64(img)
    uo = f32((int(md["x"]) + S // 2 - G // 2) * scale_uv)
    vo = f32((int(md["y"]) + S // 2 - G // 2) * scale_uv)
    poff = fma32(uo, l, (vo * m).astype(f32))
    lb, mb, pb = l[:half], m[:half], poff[:half]
    rows = slice(int(md["time_offset"]), int(md["time_offset"]) + T)
    uvw = a["uvw"].reshape(-1, 3)[rows]
    vis = a["visibilities"].reshape(-1, C, 4, 2)[rows].astype(f32)  # [T][C][4][2]
    # B columns (re, im per correlation): Bc = (re, im), Bs = (-im, re)
    e = np.frexp(np.abs(vis[:4]).max())[1]
    sc = f32(2.0 ** -e)
    bc = (vis.reshape(T, C, 8) * sc).astype(f32)
    bs = np.empty_like(bc)
    bs[..., 0::2] = -vis[..., 1] * sc
    bs[..., 1::2] = vis[..., 0] * sc
    Bc = split(bc)
    Bs = split(bs)
    Vc = vis[..., 0].astype(f64) + 1j * vis[..., 1]  # [T][C][4]

    models = ["phasor", "split", "rne", "rtz", "seq", "flush32", "flush8"]
    acc = {mname: np.zeros((4, half, 8), f32) for mname in models}  # X hi, X lo, Y hi, Y lo columns
    dsum = {mname: np.zeros((2, half, 8), f64) for mname in ("phasor", "split")}
    master = {mname: np.zeros((4, half, 8), f32) for mname in ("flush32", "flush8")}
    exact = np.zeros((2, half, 4), complex)  # base, mirror
    nkst = 0
    for q in range(T // 4):
        ts = slice(4 * q, 4 * q + 4)
        pidx = fma32(uvw[ts, 0, None], lb[None, :], (uvw[ts, 1, None] * mb[None, :]).astype(f32))
        npi = -pidx  # [4][half]
        ph = fma32(npi[:, None, :], k[None, :, None], pb[None, None, :])  # [4][C][half]
        # exact (double phasor of the f32 phase)
        ex = np.exp(1j * ph.astype(f64))
        exact[0] += np.einsum("tcp,tcj->pj", ex, Vc[ts])
        exact[1] += np.einsum("tcp,tcj->pj", np.conj(ex), Vc[ts])
        kb = k[(np.arange(C) // 16) * 16]
        A = fma32(npi[:, None, :], kb[None, :, None], pb[None, None, :])
        nm = -np.rint((A * IH).astype(f32))
        fk = (kb * IH_LO).astype(f32)
        cr = (npi[:, None, :] * fk[None, :, None]).astype(f32)
        r = (fma32(ph, IH, nm) + cr).astype(f32)
        cs = np.cos(2 * np.pi * r.astype(f64)).astype(f32)
        sn = np.sin(2 * np.pi * r.astype(f64)).astype(f32)
        # the phase-offset tail is restored after the sum (in double here)
        ach, acl = split(cs)
        ash, asl = split(sn)
        ac = ach + acl
        as_ = ash + asl
        ncq = C // 4
        rs = lambda x: x.reshape(4, ncq, 4, -1)  # noqa: E731
        # per K-step sums [cq][pixel][col]: X hi/lo cols, Y hi/lo cols
        kx_h = np.einsum("tqkp,tqkj->qpj", rs(ac), rs(Bc[0][ts]))
        kx_l = np.einsum("tqkp,tqkj->qpj", rs(ac), rs(Bc[1][ts]))
        ky_h = np.einsum("tqkp,tqkj->qpj", rs(as_), rs(Bs[0][ts]))
        ky_l = np.einsum("tqkp,tqkj->qpj", rs(as_), rs(Bs[1][ts]))
        kall = np.stack([kx_h, kx_l, ky_h, ky_l], 1)  # [cq][4][half][8]
        # unsplit phasor, exact B, double sums
        dsum["phasor"][0] += np.einsum("tcp,tcj->pj", cs.astype(f64), bc.astype(f64)[ts])
        dsum["phasor"][1] += np.einsum("tcp,tcj->pj", sn.astype(f64), bs.astype(f64)[ts])
        dsum["split"][0] += kall[:, 0].sum(0) + kall[:, 1].sum(0)
        dsum["split"][1] += kall[:, 2].sum(0) + kall[:, 3].sum(0)
        # item products of one K-step, for the sequential model
        for cq in range(ncq):
            ks = kall[cq]
            acc["rne"] = (acc["rne"].astype(f64) + ks.reshape(acc["rne"].shape)).astype(f32)
            acc["rtz"] = rtz32(acc["rtz"].astype(f64) + ks.reshape(acc["rtz"].shape))
            for fl, N in (("flush32", 32), ("flush8", 8)):
                acc[fl] = (acc[fl].astype(f64) + ks.reshape(acc[fl].shape)).astype(f32)
                if (nkst + 1) % N == 0:
                    master[fl] = (master[fl] + acc[fl].reshape(master[fl].shape)).astype(f32)
                    acc[fl][:] = 0
            nkst += 1
        # sequential: 32 products per K-step in a fixed order (t, channel, hi/lo)
        acs = acc["seq"].reshape(4, half, 8)
        for cq in range(ncq):
            for t in range(4):
                for j in range(4):
                    c = 4 * cq + j
                    for av in (ach[t, c], acl[t, c]):
                        acs[0] = (acs[0] + (av[:, None] * Bc[0][4 * q + t, c][None, :])).astype(f32)
                        acs[1] = (acs[1] + (av[:, None] * Bc[1][4 * q + t, c][None, :])).astype(f32)
                    for av in (ash[t, c], asl[t, c]):
                        acs[2] = (acs[2] + (av[:, None] * Bs[0][4 * q + t, c][None, :])).astype(f32)
                        acs[3] = (acs[3] + (av[:, None] * Bs[1][4 * q + t, c][None, :])).astype(f32)
        acc["seq"] = acs.reshape(acc["seq"].shape)

    unscale = 2.0 ** e
    tail = np.exp(1j * pb.astype(f64) * f64(TAIL))  # per base pixel

    def finish(X, Y):
        """X, Y [half][8] -> base, mirror complex [half][4] (double)."""
        xc = X[:, 0::2] + 1j * X[:, 1::2]
        yc = Y[:, 0::2] + 1j * Y[:, 1::2]
        base = (xc + yc) * unscale * tail[:, None]
        mir = (xc - yc) * unscale * np.conj(tail)[:, None]
        return base, mir

    res = {}
    for mname in ("phasor", "split"):
        res[mname] = finish(dsum[mname][0], dsum[mname][1])
    for mname in ("rne", "rtz", "seq"):
        A4 = acc[mname].reshape(4, half, 8)
        X = (A4[0] + A4[1]).astype(f32).astype(f64)
        Y = (A4[2] + A4[3]).astype(f32).astype(f64)
        res[mname] = finish(X, Y)
    for fl in ("flush32", "flush8"):
        A4 = (master[fl] + acc[fl].reshape(4, half, 8)).astype(f32)
        X = (A4[0] + A4[1]).astype(f32).astype(f64)
        Y = (A4[2] + A4[3]).astype(f32).astype(f64)
        res[fl] = finish(X, Y)

    # A1^H P A2 and the taper in double (the same for every model), into
    # the [1][4][S][S][2] subgrid layout
    at = a["aterms"].reshape(-1, 2, S, S, 4, 2)  # [slot][station][y][x][4]
    at = at[..., 0].astype(f64) + 1j * at[..., 1]
    slot = int(md["aterm_index"])
    a1 = at[slot, int(md["station1"])].reshape(npix, 2, 2)
    a2 = at[slot, int(md["station2"])].reshape(npix, 2, 2)
    sph = a["spheroidal"].reshape(npix).astype(f64)

    def lay(base, mir):
        out = np.zeros((npix, 4), complex)
        out[:half] = base
        out[half:] = mir[::-1]
        P = out.reshape(npix, 2, 2)
        P = np.conj(np.transpose(a1, (0, 2, 1))) @ P @ a2
        out = (P.reshape(npix, 4) * sph[:, None]).T
        z = np.zeros((1, 4, S, S, 2), f32)
        z[0, ..., 0] = out.real.reshape(4, S, S)
        z[0, ..., 1] = out.imag.reshape(4, S, S)
        return z
    o = orc.Oracle()
    ez = lay(exact[0], exact[1])
    print(f"C={C} T={T} subgrid {s}: output vs exact, reference metric")
    for mname in models:
        err = o.check_error(lay(*res[mname]), ez)[0]
        print(f"  {mname:8s} {err:.3e}")


if __name__ == "__main__":
    main()
