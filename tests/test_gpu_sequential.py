"""The order-preserving kernels (IDG_GRIDDER_IMPL / IDG_DEGRIDDER_IMPL =
sequential, csrc/hip/kernels/sequential_mi355x.hip.cpp): the reference CPU
path's arithmetic in its own order, so the bar is BIT-EXACT equality with the
reference's outputs (tests/golden/, oracle/_ref) and with the oracle, which is
itself bit-exact to the reference (tests/test_oracle.py) -- not a tolerance.
Run on the GPU box: -m gpu.
"""
import os
import subprocess

import numpy as np
import pytest

from conftest import CASES, REPO, TOLERANCE, load_case

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def idg():
    import torch
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    import idg_amd
    return idg_amd


@pytest.fixture
def sequential(monkeypatch):
    monkeypatch.setenv("IDG_GRIDDER_IMPL", "sequential")
    monkeypatch.setenv("IDG_DEGRIDDER_IMPL", "sequential")


def _params(p):
    return (p["nr_subgrids"], p["grid_size"], p["subgrid_size"],
            p["image_size"], p["w_step_in_lambda"], p["nr_channels"],
            p["nr_stations"])


def _grid(idg, p, a, md=None):
    out = np.zeros((p["nr_subgrids"], 4, p["subgrid_size"],
                    p["subgrid_size"], 2), np.float32)
    idg.c_run_gridder(*_params(p), a["uvw"], a["wavenumbers"],
                      a["visibilities"], a["spheroidal"], a["aterms"],
                      a["metadata"] if md is None else md, out)
    return out


def _degrid(idg, p, a, md=None):
    out = np.zeros(a["uvw"].shape[:2] + (p["nr_channels"], 4, 2), np.float32)
    idg.c_run_degridder(*_params(p), a["uvw"], a["wavenumbers"], out,
                        a["spheroidal"], a["aterms"],
                        a["metadata"] if md is None else md, a["subgrids"])
    return out


def _oracle(oracle_lib, p, a, md=None):
    md = a["metadata"] if md is None else md
    g = np.zeros((p["nr_subgrids"], 4, p["subgrid_size"], p["subgrid_size"],
                  2), np.float32)
    oracle_lib.gridder(*_params(p), a["uvw"], a["wavenumbers"],
                       a["visibilities"], a["spheroidal"], a["aterms"], md, g,
                       nthreads=min(16, os.cpu_count() or 1))
    d = np.zeros(a["uvw"].shape[:2] + (p["nr_channels"], 4, 2), np.float32)
    oracle_lib.degridder(*_params(p), a["uvw"], a["wavenumbers"], d,
                         a["spheroidal"], a["aterms"], md, a["subgrids"],
                         nthreads=min(16, os.cpu_count() or 1))
    return g, d


def _mismatch(x, y):
    return int((x.view(np.uint32) != y.view(np.uint32)).sum())


@pytest.mark.parametrize("case", CASES)
def test_sequential_bit_exact_to_reference_golden(idg, sequential, case):
    p, a = load_case(case)
    g = _grid(idg, p, a)
    d = _degrid(idg, p, a)
    assert _mismatch(g, a["gridder_out"]) == 0, case
    assert _mismatch(d, a["degridder_out"]) == 0, case


SWEEP = [
    # (stations, timeslots, T, C, G, S)
    (2, 1, 1, 1, 64, 8),
    (2, 2, 9, 7, 256, 24),
    (2, 1, 3, 5, 1024, 64),     # S = 64: several pixel passes / LDS chunks
    (2, 1, 4, 300, 1024, 32),   # many channels
    (2, 1, 700, 2, 1024, 32),   # many timesteps (> 256 x 4 degridder items)
    (2, 1, 7, 3, 256, 33),      # odd S: no mirror pairs
    (2, 1, 6, 5, 128, 15),      # odd S, S^2 < one pixel pass
    (2, 2, 128, 256, 1024, 32), # the -c NR_CHANNELS=256 shape (T x C 32,768)
    (2, 1, 3, 2, 1024, 128),    # S = 128 (runtime S)
    (5, 1, 4, 3, 999, 20),      # odd G, 10 baselines
]


@pytest.mark.parametrize("geom", SWEEP)
def test_sequential_bit_exact_to_oracle_sweep(idg, oracle_lib, sequential,
                                              geom):
    st, ts, T, C, G, S = geom
    a = idg.generate(st, ts, T, C, G, S, nthreads=8)
    p = dict(nr_subgrids=idg.nr_subgrids_for(st, ts), grid_size=G,
             subgrid_size=S, image_size=idg.IMAGE_SIZE, w_step_in_lambda=0.0,
             nr_channels=C, nr_stations=st)
    go, do = _oracle(oracle_lib, p, a)
    assert _mismatch(_grid(idg, p, a), go) == 0
    assert _mismatch(_degrid(idg, p, a), do) == 0


@pytest.mark.parametrize("geom", [(3, 2, 16, 8, 512, 32), (2, 1, 5, 3, 256, 33),
                                  (2, 1, 3, 5, 1024, 64)])
def test_sequential_bit_exact_with_w_terms(idg, oracle_lib, sequential, geom):
    st, ts, T, C, G, S = geom
    a = idg.generate(st, ts, T, C, G, S)
    rng = np.random.default_rng(3)
    a["uvw"][..., 2] = rng.uniform(-200, 200, a["uvw"].shape[:2])
    md = a["metadata"].copy()
    md["z"] = rng.integers(-3, 4, md.size)
    p = dict(nr_subgrids=md.size, grid_size=G, subgrid_size=S,
             image_size=idg.IMAGE_SIZE, w_step_in_lambda=2.5, nr_channels=C,
             nr_stations=st)
    go, do = _oracle(oracle_lib, p, a, md)
    assert _mismatch(_grid(idg, p, a, md), go) == 0
    assert _mismatch(_degrid(idg, p, a, md), do) == 0


def test_sequential_bit_exact_with_baseline_offsets(idg, oracle_lib,
                                                    sequential):
    # metadata[0].baseline_offset != 0, offsets varying by subgrid, negative
    # time offsets: the reference's time index, bit for bit
    from test_gpu import _rebase
    st, ts, T, C, G, S = 3, 2, 16, 8, 512, 32
    a = idg.generate(st, ts, T, C, G, S)
    md = _rebase(a["metadata"])
    p = dict(nr_subgrids=md.size, grid_size=G, subgrid_size=S,
             image_size=idg.IMAGE_SIZE, w_step_in_lambda=0.0, nr_channels=C,
             nr_stations=st)
    go, do = _oracle(oracle_lib, p, a, md)
    assert _mismatch(_grid(idg, p, a, md), go) == 0
    assert _mismatch(_degrid(idg, p, a, md), do) == 0


@pytest.mark.parametrize("image_size", [0.002, 0.08])
def test_sequential_bit_exact_at_other_image_sizes(idg, oracle_lib,
                                                   sequential, image_size):
    st, ts, T, C, G, S = 3, 2, 16, 8, 512, 32
    a = idg.generate(st, ts, T, C, G, S)
    p = dict(nr_subgrids=idg.nr_subgrids_for(st, ts), grid_size=G,
             subgrid_size=S, image_size=image_size, w_step_in_lambda=0.0,
             nr_channels=C, nr_stations=st)
    go, do = _oracle(oracle_lib, p, a)
    assert _mismatch(_grid(idg, p, a), go) == 0
    assert _mismatch(_degrid(idg, p, a), do) == 0


def test_sequential_mirror_fallback_on_mixed_w(idg, oracle_lib, sequential):
    # w != 0 on some subgrids only: mirror and single-pixel subgrids in one
    # launch; plus empty and ragged subgrids
    st, ts, T, C, G, S = 4, 2, 24, 6, 512, 32
    a = idg.generate(st, ts, T, C, G, S)
    a["uvw"][1::3, :, 2] = 37.5
    md = a["metadata"].copy()
    md["nr_timesteps"][2] = 0
    md["nr_timesteps"][5] = 7
    p = dict(nr_subgrids=md.size, grid_size=G, subgrid_size=S,
             image_size=idg.IMAGE_SIZE, w_step_in_lambda=0.0, nr_channels=C,
             nr_stations=st)
    go, do = _oracle(oracle_lib, p, a, md)
    assert _mismatch(_grid(idg, p, a, md), go) == 0
    # the degridder writes only the rows its subgrids cover
    d = _degrid(idg, p, a, md)
    rows = np.zeros(a["uvw"].shape[:2], bool)
    for s in range(md.size):
        rows[s, :md["nr_timesteps"][s]] = True
    assert _mismatch(d[rows], do[rows]) == 0


@pytest.mark.parametrize("lo,hi,stride", [
    (0, 0x46000000, 3),            # |y| < 2^13: every IDG phase, 1 in 3
    (0x46000000, 0x47000000, 1),   # [2^13, 2^15): every float (the device's
                                   # immediate-select table branch; G = 8192)
    (0, 0x7F800000, 61)])          # every finite float class, 1 in 61
def test_restated_sincosf_on_the_gpu_bit_exact_to_glibc(lo, hi, stride):
    # the device build of csrc/common/sincosf_glibc.hpp (its own table
    # lookup and int64 -> double conversion) against the host's glibc, and
    # the kernels' one-polynomial form sincosf_glibc_dev beside it
    path = os.path.join(REPO, "tests", "harness", "bin", "sincosf_gpu_check")
    assert os.path.exists(path), "build the harness: make -C tests/harness"
    r = subprocess.run([path, hex(lo), hex(hi), str(stride)],
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " mismatch 0 " in r.stdout, r.stdout
    assert " mismatch_dev 0" in r.stdout, r.stdout


REF_HARNESS = os.path.join(REPO, "oracle", "_ref")
HARNESS = os.path.join(REPO, "tests", "harness", "bin")


@pytest.mark.parametrize("exe", ["hip-gridder_mi355x", "hip-degridder_mi355x"])
@pytest.mark.parametrize("env", [{}, {"NR_CHANNELS": "256"},
                                 {"SUBGRID_SIZE": "64",
                                  "NR_TIMESTEPS_SUBGRID": "32"}],
                         ids=["default", "c256_t128", "s64"])
def test_reference_harness_sequential_error_zero(exe, env):
    """The reference's own unmodified harness (oracle/_ref, tests/
    {gridder,degridder}_common.cpp) with the sequential kernels: PASSED with
    error 0 -- including -c NR_CHANNELS=256 at the default T = 128, where the
    default MFMA gridder prints FAILED 1.30e-5."""
    path = os.path.join(REF_HARNESS, exe)
    if not os.path.exists(path):
        pytest.skip("oracle/_ref harness not built (needs /root/reference "
                    "at build time)")
    r = subprocess.run([path, "-c"], env=dict(
        os.environ, IDG_GRIDDER_IMPL="sequential",
        IDG_DEGRIDDER_IMPL="sequential", **env),
        capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert ">>> Result PASSED" in r.stdout, r.stdout[-3000:]
    assert ">>> Error: 0\n" in r.stdout, r.stdout[-3000:]


@pytest.mark.parametrize("exe", ["hip-gridder_mi355x", "hip-degridder_mi355x"])
def test_restated_harness_sequential_c256(exe):
    path = os.path.join(HARNESS, exe)
    assert os.path.exists(path), "build the harness: make -C tests/harness"
    r = subprocess.run([path, "-c"], env=dict(
        os.environ, IDG_QUIET="1", IDG_GRIDDER_IMPL="sequential",
        IDG_DEGRIDDER_IMPL="sequential", NR_CHANNELS="256"),
        capture_output=True, text=True, timeout=300)
    assert ">>> Result PASSED" in r.stdout, r.stdout[-2000:] + r.stderr
    assert r.returncode == 0


@pytest.mark.timeout(600)
def test_sequential_full_configs4_batch_samples_bit_exact(idg, oracle_lib,
                                                          sequential):
    """BASELINE configs[4] at full size (S = 64, 24,500 subgrids) on the
    sequential kernels through the device entries: sampled subgrids and
    their visibility rows bit-exact to the oracle (itself bit-exact to
    app/CPU)."""
    import torch
    st, ts, T, C, G, S = 50, 20, 128, 16, 1024, 64
    a = idg.generate(st, ts, T, C, G, S, nthreads=16)
    ns = idg.nr_subgrids_for(st, ts)
    p = dict(nr_subgrids=ns, grid_size=G, subgrid_size=S,
             image_size=idg.IMAGE_SIZE, w_step_in_lambda=0.0, nr_channels=C,
             nr_stations=st)
    dev = {k: torch.from_numpy(v).cuda() for k, v in a.items()
           if k not in ("metadata", "frequencies")}
    dev["metadata"] = torch.from_numpy(
        a["metadata"].view(np.int32).reshape(-1, 9).copy()).cuda()
    g_dev = torch.empty_like(dev["subgrids"])
    idg.gridder_launch(*_params(p), dev["uvw"], dev["wavenumbers"],
                       dev["visibilities"], dev["spheroidal"], dev["aterms"],
                       dev["metadata"], g_dev)
    d_dev = torch.empty_like(dev["visibilities"])
    idg.degridder_launch(*_params(p), dev["uvw"], dev["wavenumbers"], d_dev,
                         dev["spheroidal"], dev["aterms"], dev["metadata"],
                         dev["subgrids"])
    torch.cuda.synchronize()
    q = dict(p, nr_subgrids=1)
    for s in (0, ns // 2 + 3, ns - 1):
        md0 = a["metadata"][s:s + 1].copy()
        md0["time_offset"] = 0
        uvw = np.ascontiguousarray(a["uvw"][s])
        go = np.zeros((1, 4, S, S, 2), np.float32)
        oracle_lib.gridder(*_params(q), uvw, a["wavenumbers"],
                           np.ascontiguousarray(a["visibilities"][s]),
                           a["spheroidal"], a["aterms"], md0, go)
        do = np.zeros((1, T, C, 4, 2), np.float32)
        oracle_lib.degridder(*_params(q), uvw, a["wavenumbers"], do,
                             a["spheroidal"], a["aterms"], md0,
                             np.ascontiguousarray(a["subgrids"][s:s + 1]))
        assert _mismatch(g_dev[s:s + 1].cpu().numpy(), go) == 0, s
        assert _mismatch(d_dev[s:s + 1].cpu().numpy(), do) == 0, s
