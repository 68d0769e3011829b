"""Debug aid (CPU): numpy emulation of phase -> revolutions reductions for the
gridder / degridder, scored with the reference metric against the golden
reference outputs (tests/golden).  Exact f32 emulation: products of two
floats and sums with small integers are exact in float64, so
fma32(a, b, c) = f32(a*b + c) here is the device's fmaf.

  anchor : current kernels -- r = fma(ph - A, 1/2pi_hi, R), A the block's
           first-channel phase, R = revolutions(A) with the Dekker tail
  int_px : r = fma(ph, 1/2pi_hi, -m_p), m_p = rint(poff * 1/2pi_hi) per
           pixel; the tail ph * (1/2pi - 1/2pi_hi) is applied as one per-pixel
           phasor e^{i 2pi poff (1/2pi - 1/2pi_hi)} (k*P part dropped)
  int_pt : as int_px with m per (pixel, timestep, 16-channel block)
Hardware sin/cos error is modelled as uniform noise of +-hw on each output.
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import oracle as orc  # noqa: E402
from conftest import load_case  # noqa: E402

f32 = np.float32
IH = f32(float.fromhex("0x1.45f306p-3"))
IH_LO = f32(float.fromhex("0x1.b9391p-28"))
TAIL = 1.0 / (2.0 * np.pi) - float(IH)        # exact-ish 1/2pi - IH


def fma32(a, b, c):
    return (np.float64(a) * np.float64(b) + np.float64(c)).astype(f32)


def geometry(p, a, s):
    S, G = p["subgrid_size"], p["grid_size"]
    img = f32(p["image_size"])
    m = a["metadata"][s]
    idx = ((np.arange(S) + 0.5 - S / 2) * np.float64(img) / S).astype(f32)
    l = np.broadcast_to(idx[None, :], (S, S)).astype(f32)
    mm = np.broadcast_to(idx[:, None], (S, S)).astype(f32)
    scale = 2 * np.pi / np.float64(img)
    uo = f32((int(m["x"]) + S // 2 - G // 2) * scale)
    vo = f32((int(m["y"]) + S // 2 - G // 2) * scale)
    poff = fma32(uo, l, (vo * mm).astype(f32))
    T = int(m["nr_timesteps"])
    rows = slice(int(m["time_offset"]), int(m["time_offset"]) + T)
    uvw = a["uvw"].reshape(-1, 3)[rows]
    pidx = np.stack([fma32(uvw[t, 0], l, (uvw[t, 1] * mm).astype(f32))
                     for t in range(T)])                      # [T][S][S]
    return poff, pidx, rows


def revs(x):
    hi = (x * IH).astype(f32)
    lo = fma32(x, IH, -hi)
    lo = fma32(x, IH_LO, lo)
    return ((hi - np.rint(hi)).astype(f32) + lo).astype(f32)


def phasors(kind, poff, pidx, k, sign, hw, rng):
    """exp(i * phase) for every (t, c, y, x); gridder sign +1 (phase =
    fma(-pidx, k, poff)), degridder -1 (phase = fma(pidx, k, -poff))."""
    T, C = pidx.shape[0], k.size
    if sign > 0:
        ph = np.stack([fma32(-pidx, k[c], poff) for c in range(C)], 1)
    else:
        ph = np.stack([fma32(pidx, k[c], -poff) for c in range(C)], 1)
    if kind == "exact":
        ang = ph.astype(np.float64)
        z = np.exp(1j * ang)
    else:
        if kind == "anchor":
            r = np.empty_like(ph)
            for c0 in range(0, C, 16):
                A = ph[:, c0:c0 + 1]
                R = revs(A)
                d = (ph[:, c0:c0 + 16] - A).astype(f32)
                r[:, c0:c0 + 16] = fma32(d, IH, R)
            corr = 1.0
        else:
            if kind == "int_px":
                m = np.rint((sign * poff).astype(np.float64) * float(IH))
                m = np.broadcast_to(m, ph.shape)
            else:
                m = np.empty(ph.shape)
                for c0 in range(0, C, 16):
                    m[:, c0:c0 + 16] = np.rint(
                        ph[:, c0:c0 + 1].astype(np.float64) * float(IH))
            r = (ph.astype(np.float64) * float(IH) - m).astype(f32)
            corr = np.exp(2j * np.pi * TAIL * sign * poff.astype(np.float64))
        z = np.exp(2j * np.pi * r.astype(np.float64)) * corr
    if hw:
        z = z + rng.uniform(-hw, hw, z.shape) + 1j * rng.uniform(-hw, hw,
                                                                   z.shape)
    return z


def to_c(x):
    return x[..., 0].astype(np.float64) + 1j * x[..., 1]


def jones(a, s, p, S):
    m = a["metadata"][s]
    A = to_c(a["aterms"])
    a1 = A[int(m["aterm_index"]), int(m["station1"])].reshape(S, S, 2, 2)
    a2 = A[int(m["aterm_index"]), int(m["station2"])].reshape(S, S, 2, 2)
    return a1, a2


def gridder(kind, p, a, hw, rng):
    S, C = p["subgrid_size"], p["nr_channels"]
    k = a["wavenumbers"]
    out = []
    for s in range(p["nr_subgrids"]):
        poff, pidx, rows = geometry(p, a, s)
        z = phasors(kind, poff, pidx, k, +1, hw, rng)         # [T][C][S][S]
        vis = to_c(a["visibilities"].reshape(-1, C, 4, 2)[rows])  # [T][C][4]
        P = np.einsum("tcq,tcyx->yxq", vis, z).reshape(S, S, 2, 2)
        a1, a2 = jones(a, s, p, S)
        P = np.conj(np.swapaxes(a1, -1, -2)) @ P @ a2
        P = P.reshape(S, S, 4) * a["spheroidal"][..., None]
        out.append(np.moveaxis(P, -1, 0))
    return np.stack(out)


def degridder(kind, p, a, hw, rng):
    S, C = p["subgrid_size"], p["nr_channels"]
    k = a["wavenumbers"]
    out = []
    for s in range(p["nr_subgrids"]):
        poff, pidx, rows = geometry(p, a, s)
        z = phasors(kind, poff, pidx, k, -1, hw, rng)
        sg = np.moveaxis(to_c(a["subgrids"][s]), 0, -1)       # [S][S][4]
        sg = sg * a["spheroidal"][..., None]
        a1, a2 = jones(a, s, p, S)
        P = a1 @ sg.reshape(S, S, 2, 2) @ np.conj(np.swapaxes(a2, -1, -2))
        out.append(np.einsum("yxq,tcyx->tcq", P.reshape(S, S, 4), z))
    return np.stack(out)


def as_pairs(z):
    return np.stack([z.real, z.imag], -1).astype(f32)


if __name__ == "__main__":
    o = orc.Oracle()
    rng = np.random.default_rng(0)
    hw = float(os.environ.get("HW", "1.2e-7"))
    for case in sys.argv[1:] or ["c_default", "s64", "c256"]:
        p, a = load_case(case)
        a["metadata"] = np.ascontiguousarray(a["metadata"]).view(
            np.dtype([(n, "<i4") for n in ("baseline_offset", "time_offset",
                                           "nr_timesteps", "aterm_index",
                                           "station1", "station2", "x", "y",
                                           "z")])).reshape(-1)
        for kind in ("exact", "anchor", "int_px", "int_pt"):
            g = as_pairs(gridder(kind, p, a, hw, rng))
            d = degridder(kind, p, a, hw, rng)
            d = as_pairs(d).reshape(a["degridder_out"].shape)
            eg = o.check_error(g.reshape(a["gridder_out"].shape),
                               a["gridder_out"])[0]
            ed = o.check_error(d, a["degridder_out"])[0]
            print(f"{case:10s} {kind:7s} gridder {eg:.3e} degridder {ed:.3e}")
