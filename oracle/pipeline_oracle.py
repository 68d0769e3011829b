"""CPU oracle for the pipeline steps either side of the gridder / degridder
(SURVEY.md §8f rows 1-3): subgrid FFT, adder and splitter.

TEST INFRASTRUCTURE ONLY -- imported by tests/ as the checker, never by the
product path (ska-sdp-idg-bench_amd/), which runs the HIP kernels of
csrc/hip/kernels/pipeline_mi355x.hip.cpp and has no CPU fallback.

The reference has no adder, splitter or subgrid FFT (its `Grid` type,
app/common/types.hpp:358-370, is never used), so there is nothing to be
bit-compatible with: PARITY UNPINNED against the reference.  The conventions
are pinned instead by the path they complete, against the reference-faithful
C oracle (oracle/idg_oracle.c) -- tests/test_pipeline.py:
  * gridding: a unit visibility whose uv lies exactly on grid cell (U, V)
    grids (oracle gridder -> subgrid_fft(+1) -> adder) to S^2 at (U, V);
  * degridding: a unit grid cell degrids (splitter -> subgrid_fft(-1, 1/S^2)
    -> oracle degridder) to 1 for a visibility at that cell;
  * the splitter is the adjoint of the adder's placement.
"""
import numpy as np


def subgrid_fft(subgrids, sign, scale=1.0):
    """2-D DFT of every [S][S] plane of a complex [NS, 4, S, S] array:
    out[k][l] = scale * sum in[y][x] exp(sign 2 pi i (k y + l x) / S)."""
    S = subgrids.shape[-1]
    if sign > 0:
        out = np.fft.ifft2(subgrids, axes=(-2, -1)) * (S * S)
    else:
        out = np.fft.fft2(subgrids, axes=(-2, -1))
    return out * scale


def shift_phasor(S, sgn):
    """exp(i sgn pi ((x + y)(S + 1)/S - 1)) over the subgrid pixels [y, x]."""
    y, x = np.mgrid[0:S, 0:S]
    return np.exp(1j * sgn * np.pi * ((x + y) * (S + 1) / S - 1))


def _fits(m, G, S, W):
    return (0 <= m["x"] and m["x"] + S <= G and 0 <= m["y"]
            and m["y"] + S <= G and 0 <= m["z"] < W)


def adder(grid, metadata, subgrids):
    """grid[z, pol, y0 + y, x0 + x] += phasor * F[s, pol, (y+S/2)%S, (x+S/2)%S]
    (complex grid [W, 4, G, G]; subgrids wholly outside are skipped)."""
    W, _, G, _ = grid.shape
    S = subgrids.shape[-1]
    ph = shift_phasor(S, +1.0)
    shifted = np.roll(subgrids, (-(S // 2), -(S // 2)), axis=(-2, -1))
    for s, m in enumerate(metadata):
        if not _fits(m, G, S, W):
            continue
        y0, x0, z = int(m["y"]), int(m["x"]), int(m["z"])
        grid[z, :, y0:y0 + S, x0:x0 + S] += ph * shifted[s]
    return grid


def splitter(grid, metadata, S):
    """F[s, pol, (y+S/2)%S, (x+S/2)%S] = conj(phasor) * grid[z, pol, y0+y,
    x0+x]; zero for subgrids not wholly inside the grid."""
    W, _, G, _ = grid.shape
    ph = shift_phasor(S, -1.0)
    out = np.zeros((len(metadata), 4, S, S), complex)
    for s, m in enumerate(metadata):
        if not _fits(m, G, S, W):
            continue
        y0, x0, z = int(m["y"]), int(m["x"]), int(m["z"])
        out[s] = ph * grid[z, :, y0:y0 + S, x0:x0 + S]
    return np.roll(out, (S // 2, S // 2), axis=(-2, -1))


def to_complex(a):
    """[..., 2] float32 -> complex128."""
    a = np.asarray(a, dtype=np.float64)
    return a[..., 0] + 1j * a[..., 1]


def to_pairs(c):
    """complex -> [..., 2] float32."""
    return np.stack([c.real, c.imag], axis=-1).astype(np.float32)
