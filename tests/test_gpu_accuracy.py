"""Large T x C accuracy, checked as an error split (run on the GPU box: -m gpu).

BASELINE configs[2] (C = 256, T = 128) puts T x C = 32,768 visibilities into
every gridded pixel.  The reference's metric (tests/test_util.hpp:28-92) grows
with sqrt(|pixel|), and there the reference's own CPU output is ~1.3e-5 from
the exact sum of its own phases: the 1e-5 bar is below the reference's own
accumulation error.  These tests record the verdict the reference's harness
prints at that configuration and check the claim that replaces it
(tests/accuracy.py): our output is closer to exact accumulation than the
reference's, and our distance to the reference is at most 1.5x the
reference's own error.  DESIGN.md §3.1 and INTEGRATION.md list this as a
stated deviation, with the numbers these tests print.
"""
import json
import os
import re
import subprocess

import numpy as np
import pytest

from accuracy import error_split, fmt, split_holds
from conftest import REPO, TOLERANCE

pytestmark = pytest.mark.gpu

HARNESS = os.path.join(REPO, "tests", "harness", "bin")
REF_HARNESS = os.path.join(REPO, "oracle", "_ref")
RECORD = os.path.join(REPO, "gpurun_out", "accuracy")


@pytest.fixture(scope="module")
def idg():
    import torch
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    import idg_amd
    return idg_amd


@pytest.fixture(scope="module")
def ref_cpu(oracle_lib):
    """The reference's own CPU path (oracle/_ref, built from /root/reference
    sources) when present, else the pinned restatement."""
    import oracle as orc
    if orc.Reference.available(portable=True):
        return "reference app/CPU (oracle/_ref)", orc.Reference(portable=True)
    return "oracle restatement", oracle_lib


def _record(name, data):
    os.makedirs(RECORD, exist_ok=True)
    with open(os.path.join(RECORD, name + ".json"), "w") as f:
        json.dump(data, f, indent=1)


def _harness_c(path, env):
    r = subprocess.run([path, "-c"], env=dict(os.environ, IDG_QUIET="1",
                                              **env),
                       capture_output=True, text=True, timeout=600)
    verdict = re.search(r">>> Result (PASSED|FAILED)", r.stdout)
    err = re.search(r">>> Error: ([-+0-9.eE]+)", r.stdout)
    assert verdict and err, r.stdout[-2000:] + r.stderr[-2000:]
    return {"verdict": verdict.group(1), "error": float(err.group(1)),
            "exit_code": r.returncode}


def _cpu_threads():
    return max(1, min(16, os.cpu_count() or 1))


# -c at NR_CHANNELS=256 with the harness' default NR_TIMESTEPS_SUBGRID=128
# (tests/gridder_common.cpp:54-60): NR_STATIONS=2, NR_TIMESLOTS=2 -> 2
# subgrids, 65,536 visibilities each.
C256_ENV = {"NR_CHANNELS": "256"}
C256 = dict(st=2, ts=2, T=128, C=256, G=1024, S=32)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("direction", ["gridder", "degridder"])
def test_c256_default_timesteps_harness_verdict_and_error_split(
        idg, oracle_lib, ref_cpu, direction):
    exe = f"hip-{direction}_mi355x"
    harness = {}
    for tag, root in (("reference_harness", REF_HARNESS),
                      ("restated_harness", HARNESS)):
        path = os.path.join(root, exe)
        if os.path.exists(path):
            harness[tag] = _harness_c(path, C256_ENV)
    assert "restated_harness" in harness, "build the harness first"

    # the harness' inputs, in-process (srand(0), reference generators)
    c = C256
    a = idg.generate(c["st"], c["ts"], c["T"], c["C"], c["G"], c["S"],
                     nthreads=8)
    ns = a["metadata"].size
    args = (ns, c["G"], c["S"], idg.IMAGE_SIZE, idg.W_STEP, c["C"], c["st"])
    ref_name, ref_lib = ref_cpu
    nt = _cpu_threads()
    if direction == "gridder":
        ours = np.zeros((ns, 4, c["S"], c["S"], 2), np.float32)
        idg.c_run_gridder(*args, a["uvw"], a["wavenumbers"],
                          a["visibilities"], a["spheroidal"], a["aterms"],
                          a["metadata"], ours)
        ref = np.zeros_like(ours)
        ref_lib.gridder(*args, a["uvw"], a["wavenumbers"], a["visibilities"],
                        a["spheroidal"], a["aterms"], a["metadata"], ref)
        orc_out = np.zeros_like(ours)
        oracle_lib.gridder(*args, a["uvw"], a["wavenumbers"],
                           a["visibilities"], a["spheroidal"], a["aterms"],
                           a["metadata"], orc_out, nthreads=nt)
        exact = np.zeros(ours.shape, np.float64)
        oracle_lib.gridder_exact(*args, a["uvw"], a["wavenumbers"],
                                 a["visibilities"], a["spheroidal"],
                                 a["aterms"], a["metadata"], exact,
                                 nthreads=nt)
    else:
        ours = np.zeros_like(a["visibilities"])
        idg.c_run_degridder(*args, a["uvw"], a["wavenumbers"], ours,
                            a["spheroidal"], a["aterms"], a["metadata"],
                            a["subgrids"])
        ref = np.zeros_like(ours)
        ref_lib.degridder(*args, a["uvw"], a["wavenumbers"], ref,
                          a["spheroidal"], a["aterms"], a["metadata"],
                          a["subgrids"])
        orc_out = np.zeros_like(ours)
        oracle_lib.degridder(*args, a["uvw"], a["wavenumbers"], orc_out,
                             a["spheroidal"], a["aterms"], a["metadata"],
                             a["subgrids"], nthreads=nt)
        exact = np.zeros(ours.shape, np.float64)
        oracle_lib.degridder_exact(*args, a["uvw"], a["wavenumbers"], exact,
                                   a["spheroidal"], a["aterms"],
                                   a["metadata"], a["subgrids"], nthreads=nt)
    split = error_split(oracle_lib, ours, ref, exact)
    split["ours_vs_oracle"] = float(oracle_lib.check_error(ours, orc_out)[0])
    rec = {"config": "-c NR_CHANNELS=256 (T=128 default): 2 subgrids",
           "direction": direction, "reference_cpu": ref_name,
           "harness": harness, "split": split}
    _record(f"c256_T128_{direction}", rec)
    print(f"{direction} C=256 T=128 -c: harness {harness}; {fmt(split)}")

    # The harnesses measured the same outputs: the restated harness compares
    # ours with the restatement over every output; the reference's harness
    # with the reference CPU path, over the first quarter of the
    # visibilities (its compare_visibilities passes the Visibility count as
    # the complex count, tests/test_util.hpp:94-99).
    assert harness["restated_harness"]["error"] == pytest.approx(
        split["ours_vs_oracle"], rel=1e-3)
    if "reference_harness" in harness:
        if direction == "gridder":
            seen = split["ours_vs_ref"]
        else:
            n = ours.size // 2 // 4
            seen = oracle_lib.check_error(ours.reshape(-1, 2)[:n],
                                          ref.reshape(-1, 2)[:n])[0]
        assert harness["reference_harness"]["error"] == pytest.approx(
            seen, rel=1e-3)
    if direction == "degridder":
        # the degridder's sums are not coherent (its error is per-phasor, not
        # accumulation): the reference metric holds unchanged
        assert split["ours_vs_ref"] <= TOLERANCE
        assert harness["restated_harness"]["verdict"] == "PASSED"
    else:
        assert split_holds(split), fmt(split)
        # and the bar itself against exact accumulation, which the
        # reference's own output misses here (ref_vs_exact ~1.3e-5)
        assert split["ours_vs_exact"] <= TOLERANCE, fmt(split)


# The -c defaults (tests/gridder_common.cpp:54-60: NR_STATIONS=2,
# NR_TIMESLOTS=2, NR_TIMESTEPS_SUBGRID=128, NR_CHANNELS=16): the gridder
# must be at least as close to the exact accumulation of the reference's own
# f32 phases as the reference's CPU output is.
@pytest.mark.parametrize("direction", ["gridder", "degridder"])
def test_c_defaults_closer_to_exact_than_the_reference(idg, oracle_lib,
                                                       ref_cpu, direction):
    st, ts, T, C, G, S = 2, 2, 128, 16, 1024, 32
    a = idg.generate(st, ts, T, C, G, S, nthreads=8)
    ns = a["metadata"].size
    args = (ns, G, S, idg.IMAGE_SIZE, idg.W_STEP, C, st)
    ref_name, ref_lib = ref_cpu
    nt = _cpu_threads()
    if direction == "gridder":
        ours = np.zeros((ns, 4, S, S, 2), np.float32)
        idg.c_run_gridder(*args, a["uvw"], a["wavenumbers"],
                          a["visibilities"], a["spheroidal"], a["aterms"],
                          a["metadata"], ours)
        ref = np.zeros_like(ours)
        ref_lib.gridder(*args, a["uvw"], a["wavenumbers"], a["visibilities"],
                        a["spheroidal"], a["aterms"], a["metadata"], ref)
        exact = np.zeros(ours.shape, np.float64)
        oracle_lib.gridder_exact(*args, a["uvw"], a["wavenumbers"],
                                 a["visibilities"], a["spheroidal"],
                                 a["aterms"], a["metadata"], exact,
                                 nthreads=nt)
    else:
        ours = np.zeros_like(a["visibilities"])
        idg.c_run_degridder(*args, a["uvw"], a["wavenumbers"], ours,
                            a["spheroidal"], a["aterms"], a["metadata"],
                            a["subgrids"])
        ref = np.zeros_like(ours)
        ref_lib.degridder(*args, a["uvw"], a["wavenumbers"], ref,
                          a["spheroidal"], a["aterms"], a["metadata"],
                          a["subgrids"])
        exact = np.zeros(ours.shape, np.float64)
        oracle_lib.degridder_exact(*args, a["uvw"], a["wavenumbers"], exact,
                                   a["spheroidal"], a["aterms"],
                                   a["metadata"], a["subgrids"], nthreads=nt)
    split = error_split(oracle_lib, ours, ref, exact)
    _record(f"c_default_{direction}", {"config": "-c defaults",
                                        "direction": direction,
                                        "reference_cpu": ref_name,
                                        "split": split})
    print(f"{direction} -c defaults: {fmt(split)}")
    assert split["ours_vs_ref"] <= TOLERANCE, fmt(split)
    if direction == "gridder":
        assert split["ours_vs_exact"] <= split["ref_vs_exact"], fmt(split)
    else:
        # the degridder: 3.9e-7 against the reference's 4.1e-7 since its
        # B operand sits high in the f16 range (1.0e-6 with
        # the lo parts of small pixels in f16 subnormals): held to 1.25x
        assert split["ours_vs_exact"] <= 1.25 * split["ref_vs_exact"], \
            fmt(split)


@pytest.mark.parametrize("C", [16, 64, 128])
def test_tail_patterns_on_channel_incoherent_visibilities(idg, oracle_lib,
                                                          ref_cpu, C,
                                                          monkeypatch):
    """Every channel of every timestep gets an independent random phase: a
    worst case for the one-channel-per-quad tail (kPrecTailAlt, 4x the
    reduction tail on one channel of four), which cancels only where a
    quad's four terms are coherent, as on the reference's synthetic data
    (DESIGN.md §3.3).  Round 5 measured it here at 1.31e-6 / 2.43e-6 from
    exact at C = 16 / 64, farther than the reference's own f32 sum (0.79e-6
    / 2.21e-6), so since round 6 the default gridder puts the tail on every
    phasor (kPrecTail).  Held here:
      * the default's distance to exact <= the reference's own (the error
        split's first half, tests/accuracy.py) at every C;
      * the default within the reference's bar of app/CPU itself (oracle/_ref
        when built, else the pinned restatement), in the reference metric,
        at T x C >= 8,192 (C = 64, 128);
      * the every-phasor tail no farther from exact than no tail."""
    import torch
    st, ts, T, G, S = 2, 2, 128, 1024, 32
    a = idg.generate(st, ts, T, C, G, S)
    rng = np.random.default_rng(23)
    ph = rng.uniform(0.0, 2 * np.pi, a["visibilities"].shape[:3])
    rot = np.stack([np.cos(ph), np.sin(ph)], -1).astype(np.float32)
    v = a["visibilities"]  # [..., C, 4, 2]: rotate every (t, c) by its phase
    vr, vi = v[..., 0].copy(), v[..., 1].copy()
    c_, s_ = rot[..., None, 0], rot[..., None, 1]
    v[..., 0] = vr * c_ - vi * s_
    v[..., 1] = vr * s_ + vi * c_
    ns = a["metadata"].size
    p = (ns, G, S, idg.IMAGE_SIZE, 0.0, C, st)
    exact = np.zeros((ns, 4, S, S, 2), np.float64)
    oracle_lib.gridder_exact(*p, a["uvw"], a["wavenumbers"], v,
                             a["spheroidal"], a["aterms"], a["metadata"],
                             exact, nthreads=8)
    ex32 = exact.astype(np.float32)
    errs, outs = {}, {}
    for name, bits in (("default", None), ("tail_alt", "4"),
                       ("tail_every", "1"), ("none", "0")):
        if bits is None:
            monkeypatch.delenv("IDG_PREC", raising=False)
        else:
            monkeypatch.setenv("IDG_PREC", bits)
        out = np.zeros((ns, 4, S, S, 2), np.float32)
        idg.c_run_gridder(*p, a["uvw"], a["wavenumbers"], v, a["spheroidal"],
                          a["aterms"], a["metadata"], out)
        errs[name] = oracle_lib.check_error(out, ex32)[0]
        outs[name] = out
    src, impl = ref_cpu
    ref = np.zeros((ns, 4, S, S, 2), np.float32)
    impl.gridder(*p, a["uvw"], a["wavenumbers"], v, a["spheroidal"],
                 a["aterms"], a["metadata"], ref)
    errs["reference_order_f32"] = oracle_lib.check_error(ref, ex32)[0]
    errs["default_vs_reference"] = oracle_lib.check_error(outs["default"],
                                                          ref)[0]
    errs["reference_source"] = src
    print(f"C={C} channel-incoherent visibilities:",
          {k: (f"{e:.3e}" if isinstance(e, float) else e)
           for k, e in errs.items()})
    _record(f"tail_patterns_incoherent_c{C}", errs)
    assert errs["default"] <= errs["reference_order_f32"], errs
    if T * C >= 8192:
        assert errs["default_vs_reference"] <= TOLERANCE, errs
    for k in ("default", "tail_alt", "tail_every", "none"):
        assert errs[k] <= 0.5 * TOLERANCE, errs
    # the every-phasor tail removes the systematic part on any data
    assert errs["tail_every"] <= errs["none"], errs
