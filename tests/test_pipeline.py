"""Pipeline steps either side of the gridder/degridder (SURVEY.md §8f rows
1-3): conventions of the subgrid FFT, adder and splitter, pinned against the
reference-faithful C oracle's gridder and degridder (CPU, no GPU needed).

The reference has no adder/splitter/FFT, so these are "parity unpinned"
against it; what is pinned is that the pipeline does the physically right
thing with the oracle's own gridder/degridder conventions
(oracle/pipeline_oracle.py docstring)."""
import numpy as np
import pytest

import pipeline_oracle as pl
from oracle import METADATA_DTYPE

IMAGE_SIZE = 0.01


def _one_subgrid(S, xc, yc, st=2):
    md = np.zeros(1, METADATA_DTYPE)
    md["nr_timesteps"] = 1
    md["station1"], md["station2"] = 0, 1
    md["x"], md["y"] = xc, yc
    at = np.zeros((1, st, S, S, 4, 2), np.float32)
    at[..., 0, 0] = 1.0
    at[..., 3, 0] = 1.0
    return md, at, np.ones((S, S), np.float32)


def _uvw_at(Ux, Uy, G):
    u, v = (Ux - G / 2) / IMAGE_SIZE, (Uy - G / 2) / IMAGE_SIZE
    return np.array([[u, v, 0.0]], np.float32).reshape(1, 1, 3)


@pytest.mark.parametrize("S", [32, 64])
def test_unit_visibility_grids_to_its_cell(oracle_lib, S):
    G, st, xc, yc = 256, 2, 100, 60
    md, at, sph = _one_subgrid(S, xc, yc, st)
    wn = np.array([2 * np.pi], np.float32)  # k = 2 pi: uvw in wavelengths
    vis = np.zeros((1, 1, 1, 4, 2), np.float32)
    vis[..., 0, 0] = 1.0
    vis[..., 3, 0] = 1.0
    for Ux, Uy in ((xc, yc), (xc + 13, yc + 11), (xc + S - 1, yc + 5),
                   (xc + 7, yc + S - 2)):
        sg = np.zeros((1, 4, S, S, 2), np.float32)
        oracle_lib.gridder(1, G, S, IMAGE_SIZE, 0.0, 1, st, _uvw_at(Ux, Uy, G),
                           wn, vis, sph, at, md, sg)
        F = pl.subgrid_fft(pl.to_complex(sg), +1)
        grid = pl.adder(np.zeros((1, 4, G, G), complex), md, F)
        assert np.argmax(np.abs(grid[0, 0])) == Uy * G + Ux
        np.testing.assert_allclose(grid[0, 0, Uy, Ux], S * S, rtol=1e-6)
        np.testing.assert_allclose(grid[0, 3, Uy, Ux], S * S, rtol=1e-6)
        assert np.abs(grid[0, 1]).max() == 0.0


@pytest.mark.parametrize("S", [32, 64])
def test_unit_cell_degrids_to_one(oracle_lib, S):
    G, st, xc, yc = 256, 2, 100, 60
    md, at, sph = _one_subgrid(S, xc, yc, st)
    wn = np.array([2 * np.pi], np.float32)
    for Ux, Uy in ((xc + 13, yc + 11), (xc + 25, yc + 30), (xc + 17, yc + 6)):
        grid = np.zeros((1, 4, G, G), complex)
        grid[0, 0, Uy, Ux] = 1.0
        grid[0, 3, Uy, Ux] = 2.0 - 1.0j
        F = pl.subgrid_fft(pl.splitter(grid, md, S), -1, 1.0 / (S * S))
        vis = np.zeros((1, 1, 1, 4, 2), np.float32)
        oracle_lib.degridder(1, G, S, IMAGE_SIZE, 0.0, 1, st,
                             _uvw_at(Ux, Uy, G), wn, vis, sph, at, md,
                             pl.to_pairs(F))
        v = pl.to_complex(vis)[0, 0, 0]
        np.testing.assert_allclose(v, [1.0, 0.0, 0.0, 2.0 - 1.0j], atol=3e-6)


def test_splitter_is_adjoint_of_adder():
    rng = np.random.default_rng(3)
    G, S, W, ns = 96, 16, 2, 9
    md = np.zeros(ns, METADATA_DTYPE)
    md["x"] = rng.integers(-4, G - S + 4, ns)
    md["y"] = rng.integers(-4, G - S + 4, ns)
    md["z"] = rng.integers(0, W + 1, ns)   # some out of range -> skipped
    X = rng.normal(size=(ns, 4, S, S)) + 1j * rng.normal(size=(ns, 4, S, S))
    g = rng.normal(size=(W, 4, G, G)) + 1j * rng.normal(size=(W, 4, G, G))
    lhs = np.vdot(g, pl.adder(np.zeros_like(g), md, X))
    rhs = np.vdot(pl.splitter(g, md, S), X)
    np.testing.assert_allclose(lhs, rhs, rtol=1e-12)


def test_fft_sign_and_scale():
    rng = np.random.default_rng(5)
    x = rng.normal(size=(2, 4, 8, 8)) + 1j * rng.normal(size=(2, 4, 8, 8))
    S = 8
    k = np.arange(S)
    E = np.exp(2j * np.pi * np.outer(k, k) / S)       # sign +1 DFT matrix
    ref = np.einsum("ky,...yx,lx->...kl", E, x, E)
    np.testing.assert_allclose(pl.subgrid_fft(x, +1), ref, atol=1e-10)
    np.testing.assert_allclose(pl.subgrid_fft(pl.subgrid_fft(x, +1), -1,
                                              1.0 / S**2), x, atol=1e-12)
