"""The CPU oracle pinned against the reference's golden vectors (CPU only).

tests/golden/*.npz were produced by the reference's own CPU path
(oracle/_ref/libidgref.so, built from /root/reference/app/{common,CPU} with
the reference's flags; tests/golden/make_golden.py).  The plain-C restatement
(oracle/idg_oracle.c) must reproduce them far inside the repo tolerance.
"""
import os

import numpy as np
import pytest

import oracle as orc
from conftest import CASES, TOLERANCE, load_case

# The restatement reproduces the reference's FMA fusion pattern exactly, so
# it is bit-exact (test_oracle_bit_exact_to_reference_golden); the metric bar
# below is the weaker claim kept beside it (rounds 1-4: 5.5e-8 .. 4.1e-7).
ORACLE_BAR = 1e-6


def _run(o, p, a):
    ns, G, S = p["nr_subgrids"], p["grid_size"], p["subgrid_size"]
    C, st = p["nr_channels"], p["nr_stations"]
    img, ws = p["image_size"], p["w_step_in_lambda"]
    g = np.zeros_like(a["gridder_out"])
    o.gridder(ns, G, S, img, ws, C, st, a["uvw"], a["wavenumbers"],
              a["visibilities"], a["spheroidal"], a["aterms"], a["metadata"],
              g)
    d = np.zeros_like(a["degridder_out"])
    o.degridder(ns, G, S, img, ws, C, st, a["uvw"], a["wavenumbers"], d,
                a["spheroidal"], a["aterms"], a["metadata"], a["subgrids"])
    return g, d


@pytest.mark.parametrize("case", CASES)
def test_oracle_matches_reference_golden(oracle_lib, case):
    p, a = load_case(case)
    g, d = _run(oracle_lib, p, a)
    eg, _ = oracle_lib.check_error(g, a["gridder_out"])
    ed, _ = oracle_lib.check_error(d, a["degridder_out"])
    assert eg < ORACLE_BAR, f"gridder {case}: {eg}"
    assert ed < ORACLE_BAR, f"degridder {case}: {ed}"


@pytest.mark.parametrize("case", CASES)
def test_oracle_bit_exact_to_reference_golden(oracle_lib, case):
    # with GCC's per-site complex-product forms (idg_oracle.c header) the
    # restatement computes the reference's bits, not just its values: every
    # output of every golden case, both directions (same glibc sincosf)
    p, a = load_case(case)
    g, d = _run(oracle_lib, p, a)
    assert np.array_equal(g, a["gridder_out"]), case
    assert np.array_equal(d, a["degridder_out"]), case


@pytest.mark.skipif(not orc.Reference.available(portable=True),
                    reason="oracle/_ref not built (needs /root/reference)")
def test_oracle_bit_exact_to_reference_at_T128_C256(oracle_lib):
    # the -c NR_CHANNELS=256 shape (T x C = 32,768 sequential adds per pixel)
    # that the reference's own build is 1.27e-5 from exact at
    import idg_amd
    a = idg_amd.generate(2, 2, 128, 256, 1024, 32, nthreads=8)
    ns = a["metadata"].size
    args = (ns, 1024, 32, idg_amd.IMAGE_SIZE, 0.0, 256, 2)
    ref, ours = orc.Reference(portable=True), np.zeros((ns, 4, 32, 32, 2),
                                                       np.float32)
    r = np.zeros_like(ours)
    ref.gridder(*args, a["uvw"], a["wavenumbers"], a["visibilities"],
                a["spheroidal"], a["aterms"], a["metadata"], r)
    oracle_lib.gridder(*args, a["uvw"], a["wavenumbers"], a["visibilities"],
                       a["spheroidal"], a["aterms"], a["metadata"], ours,
                       nthreads=8)
    assert np.array_equal(ours, r)


def test_oracle_multithreaded_identical(oracle_lib):
    p, a = load_case("multi")
    ns, G, S = p["nr_subgrids"], p["grid_size"], p["subgrid_size"]
    C, st = p["nr_channels"], p["nr_stations"]
    g1 = np.zeros_like(a["gridder_out"])
    g4 = np.zeros_like(a["gridder_out"])
    for out, nt in ((g1, 1), (g4, 4)):
        oracle_lib.gridder(ns, G, S, p["image_size"], p["w_step_in_lambda"],
                           C, st, a["uvw"], a["wavenumbers"],
                           a["visibilities"], a["spheroidal"], a["aterms"],
                           a["metadata"], out, nthreads=nt)
    assert np.array_equal(g1, g4)


def test_cpu_baseline_threads_compute_the_whole_batch():
    # bench.py's 16-thread cpu_baseline runs the reference kernel on disjoint
    # subgrid ranges; with equal baseline offsets (the synthetic batch) the
    # ranges' outputs are exactly the whole run's
    import bench
    import idg_amd
    os.environ["IDG_CPU_BASELINE_THREADS"] = "3"
    w = dict(bench.WORKLOADS["default"], nr_stations=4, nr_timeslots=2,
             nr_timesteps=8, nr_channels=4, grid_size=256, subgrid_size=16)
    a = idg_amd.generate(4, 2, 8, 4, 256, 16)
    try:
        r = bench.cpu_baseline(w, a, 4)
    finally:
        del os.environ["IDG_CPU_BASELINE_THREADS"]
    assert r["cores"] == 3 and r["single_thread"]["cores"] == 1
    assert r["value"] > 0 and r["unit"] == "Mvis/s"
    outs = bench.cpu_baseline_threads.last_outputs
    ns = outs["subgrids"].shape[0]
    g = np.zeros_like(outs["subgrids"])
    impl = orc.Reference(portable=True) if orc.Reference.available() \
        else orc.Oracle()
    impl.gridder(ns, 256, 16, 0.01, 0.0, 4, 4, a["uvw"], a["wavenumbers"],
                 a["visibilities"], a["spheroidal"], a["aterms"],
                 a["metadata"][:ns], g)
    assert np.array_equal(g, outs["subgrids"])
    d = np.zeros_like(outs["visibilities"])
    impl.degridder(ns, 256, 16, 0.01, 0.0, 4, 4, a["uvw"], a["wavenumbers"],
                   d, a["spheroidal"], a["aterms"], a["metadata"][:ns],
                   np.ascontiguousarray(a["subgrids"][:ns]))
    assert np.array_equal(d, outs["visibilities"])


def test_metric_matches_numpy_twin(oracle_lib):
    rng = np.random.default_rng(0)
    b = rng.normal(size=(1000, 2)).astype(np.float32) * 50
    a = b + rng.normal(size=b.shape).astype(np.float32) * 1e-3
    b[::7] = 0.0  # entries with |B| == 0 are excluded (nnz)
    e1, nnz = oracle_lib.check_error(a, b)
    e2 = orc.check_error(a, b)
    assert nnz == 1000 - len(range(0, 1000, 7))
    assert abs(e1 - e2) <= 1e-9 * max(1.0, e1)


def test_metric_semantics():
    # identical -> 0; a uniform offset d on every element with r_max = 1
    # -> sqrt(d^2 + d^2)
    b = np.ones((10, 2), np.float32) * 0.5
    assert orc.check_error(b, b) == 0.0
    a = b + np.float32(1e-3)
    assert abs(orc.check_error(a, b) - np.sqrt(2) * 1e-3) < 1e-7
    # the pass threshold is 1e-5 (tests/test_util.hpp:84)
    assert TOLERANCE == 1e-5


@pytest.mark.skipif(not orc.Reference.available(portable=True) or
                    not orc.Reference.available(portable=False),
                    reason="oracle/_ref not built (no /root/reference here)")
def test_reference_builds_agree_bitwise():
    # the -march=x86-64-v3 build that travels to the GPU box computes the
    # same bits as the -march=native build that made the golden vectors
    p, a = load_case("c_default")
    ns, G, S = p["nr_subgrids"], p["grid_size"], p["subgrid_size"]
    ref = orc.Reference(portable=True)
    g = np.zeros_like(a["gridder_out"])
    ref.gridder(ns, G, S, p["image_size"], p["w_step_in_lambda"],
                p["nr_channels"], p["nr_stations"], a["uvw"],
                a["wavenumbers"], a["visibilities"], a["spheroidal"],
                a["aterms"], a["metadata"], g)
    assert np.array_equal(g, a["gridder_out"])


# --------------------------------------------------------------------------
# The exact-accumulation twins (oracle_*_exact): the instrument of the
# large-T x C error split (tests/accuracy.py, tests/test_gpu_accuracy.py)
# --------------------------------------------------------------------------
def _exact(o, p, a):
    ns, G, S = p["nr_subgrids"], p["grid_size"], p["subgrid_size"]
    C, st = p["nr_channels"], p["nr_stations"]
    img, ws = p["image_size"], p["w_step_in_lambda"]
    g = np.zeros(a["gridder_out"].shape, np.float64)
    o.gridder_exact(ns, G, S, img, ws, C, st, a["uvw"], a["wavenumbers"],
                    a["visibilities"], a["spheroidal"], a["aterms"],
                    a["metadata"], g, nthreads=4)
    d = np.zeros(a["degridder_out"].shape, np.float64)
    o.degridder_exact(ns, G, S, img, ws, C, st, a["uvw"], a["wavenumbers"],
                      d, a["spheroidal"], a["aterms"], a["metadata"],
                      a["subgrids"], nthreads=4)
    return g, d


@pytest.mark.parametrize("case", CASES)
def test_exact_twins_agree_with_reference_golden(oracle_lib, case):
    # at golden sizes (T x C <= 4,096) the reference's f32 sums are within
    # a few 1e-6 of the exact accumulation of its own phases
    p, a = load_case(case)
    g, d = _exact(oracle_lib, p, a)
    assert oracle_lib.check_error(a["gridder_out"], g.astype(np.float32))[0] \
        <= 5e-6
    assert oracle_lib.check_error(a["degridder_out"],
                                  d.astype(np.float32))[0] <= 5e-6


def test_exact_gridder_matches_numpy_fp64_restatement(oracle_lib):
    # an independent numpy restatement (tests/emul/grid_fp64.py: the same f32
    # phase rounding, float64 everything else) of one subgrid
    import importlib.util
    import idg_amd
    spec = importlib.util.spec_from_file_location(
        "grid_fp64", os.path.join(os.path.dirname(__file__), "emul",
                                  "grid_fp64.py"))
    gf = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gf)
    st, ts, T, C, G, S = 2, 1, 8, 4, 1024, 32
    a = idg_amd.generate(st, ts, T, C, G, S, nthreads=2)
    g = np.zeros((1, 4, S, S, 2), np.float64)
    oracle_lib.gridder_exact(1, G, S, idg_amd.IMAGE_SIZE, 0.0, C, st,
                             a["uvw"], a["wavenumbers"], a["visibilities"],
                             a["spheroidal"], a["aterms"], a["metadata"][:1],
                             g)
    ref = gf.grid_fp64(a, 0, G, S, C)
    got = g[0, ..., 0] + 1j * g[0, ..., 1]
    assert np.abs(got - ref).max() <= 1e-9 * np.abs(ref).max()


@pytest.mark.skipif(not orc.Reference.available(portable=True),
                    reason="oracle/_ref not built (needs /root/reference)")
def test_reference_itself_misses_the_bar_at_large_TxC(oracle_lib):
    """The fact behind the stated configs[2] deviation: at
    T x C = 32,768 (-c with NR_CHANNELS=256, T = 128) the reference's own
    CPU gridder output is more than 1e-5 from the exact sum of its own
    phases in its own metric, while at the -c defaults it is ~1e-6."""
    import idg_amd
    ref = orc.Reference(portable=True)
    errs = {}
    for C in (16, 256):
        a = idg_amd.generate(2, 2, 128, C, 1024, 32, nthreads=8)
        ns = a["metadata"].size
        args = (ns, 1024, 32, idg_amd.IMAGE_SIZE, 0.0, C, 2)
        r = np.zeros((ns, 4, 32, 32, 2), np.float32)
        ref.gridder(*args, a["uvw"], a["wavenumbers"], a["visibilities"],
                    a["spheroidal"], a["aterms"], a["metadata"], r)
        e = np.zeros(r.shape, np.float64)
        oracle_lib.gridder_exact(*args, a["uvw"], a["wavenumbers"],
                                 a["visibilities"], a["spheroidal"],
                                 a["aterms"], a["metadata"], e,
                                 nthreads=min(8, os.cpu_count() or 1))
        errs[C] = oracle_lib.check_error(r, e.astype(np.float32))[0]
    assert errs[16] < 2e-6, errs
    assert errs[256] > TOLERANCE, errs


@pytest.mark.parametrize("C", [16, 64])
def test_reduction_tail_on_one_channel_per_quad_emulated(C):
    """The gridder's phase-reduction tail, emulated exactly with double sums
    (tests/emul/tail_mean_emul.py): without it the
    coherent sums keep a systematic phase error; added as 4c to the first
    channel of every quad (kPrecTailAlt, IDG_PREC=4; the default until
    round 5, when channel-incoherent data showed it losing to the
    reference's own sum, tests/test_gpu_accuracy.py) it is as close
    to the exact sum as the every-phasor add within 2x, and at least 4x
    closer than none -- while a per-quad pattern or one channel in 16 is
    worse than one in 4."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "emul"))
    from tail_mean_emul import emulate
    e = emulate(C, 128, nthreads=4)
    assert e["alt4"] <= 2.0 * e["block"], e
    assert e["alt4"] * 4.0 <= e["none"], e
    assert e["alt4"] < e["sparse4"] and e["alt4"] < e["alt16"], e
