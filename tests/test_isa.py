"""Static checks of the shipped gfx950 kernels' ISA (CPU only: hipcc
cross-compiles the listing with the library's own flags, `make isa`).

* Wait states around the inline-asm f16 splits that feed the MFMAs
  (tools/probes/hazard_check.py): every v_mfma SrcA/SrcB
  written by a VALU has >= 2 wait states before it, every VALU read of a
  v_sin/v_cos result >= 1, on every control-flow path.
* Register spills stay out of the MFMA loops: no scratch access inside any
  basic block that issues an MFMA (DESIGN.md §4.1-4.2 document the few
  cold spills of the prologue/epilogue).
"""
import os
import re
import subprocess
import sys

import pytest

from conftest import PKG, REPO

sys.path.insert(0, os.path.join(REPO, "tools", "probes"))
import hazard_check as hc  # noqa: E402

ISA = os.path.join(PKG, "build", "isa")


@pytest.fixture(scope="module")
def listings():
    subprocess.run(["make", "-C", PKG, "isa"], check=True,
                   capture_output=True, timeout=600)
    return {k: os.path.join(ISA, f"{k}_mi355x.s")
            for k in ("gridder", "degridder")}


SYNTH = """
_Zkernel:
\tv_cvt_pk_f16_f32 v10, v1, v2
\t{pad}
\tv_mfma_f32_16x16x32_f16 v[0:3], v[10:13], v[20:23], v[0:3]
\ts_endpgm
.Lfunc_end0:
"""


@pytest.mark.parametrize("pad,bad", [("s_nop 1", False), ("s_nop 0", True),
                                     ("v_add_f32 v30, v31, v32", True),
                                     ("s_nop 0\n\tv_add_f32 v30, v31, v32",
                                      False)])
def test_checker_counts_valu_to_mfma_wait_states(pad, bad):
    f = hc.parse_functions(SYNTH.format(pad=pad))["_Zkernel"]
    assert bool(hc.check_function(f)) == bad


def test_checker_follows_branches_into_a_loop_head():
    # the producer sits at the end of the loop body, the MFMA at its head:
    # only the back edge connects them
    src = """
_Zk:
\ts_nop 4
.LBB0_1:
\tv_mfma_f32_16x16x32_f16 v[0:3], v[10:13], v[20:23], v[0:3]
\ts_nop 7
\tv_cvt_pk_f16_f32 v11, v1, v2
\ts_cbranch_scc1 .LBB0_1
\ts_endpgm
.Lfunc_end0:
"""
    v = hc.check_function(hc.parse_functions(src)["_Zk"])
    assert [k for k, *_ in v] == ["valu->mfma_src"]


def test_checker_trans_forwarding():
    src = """
_Zk:
\tv_sin_f32_e32 v5, v4
\tv_fma_mixlo_f16 v7, v6, -1.0, v5 op_sel_hi:[1,0,0]
\ts_endpgm
.Lfunc_end0:
"""
    v = hc.check_function(hc.parse_functions(src)["_Zk"])
    assert [k for k, *_ in v] == ["trans->valu"]


@pytest.mark.parametrize("kernel", ["gridder", "degridder"])
def test_shipped_kernels_have_no_operand_hazards(listings, kernel):
    res = hc.check_file(listings[kernel])
    mfma_kernels = {n: r for n, r in res.items() if r["mfma"]}
    assert mfma_kernels, "no MFMA kernel found in the listing"
    bad = {n[:60]: r["violations"][:3] for n, r in res.items()
           if r["violations"]}
    assert not bad, bad


@pytest.mark.parametrize("kernel", ["gridder", "degridder"])
def test_no_scratch_access_in_mfma_loops(listings, kernel):
    # Every kernel but the queue-fed general gridder, which only runs on
    # batches that mix w = 0 and w != 0 subgrids with W_STEP = 0 (its loop
    # over queued subgrids reloads one spilled pointer in an MFMA block;
    # DESIGN.md §4.1).
    import mfma_spills
    from resources import short
    res = mfma_spills.per_kernel(open(listings[kernel]).read())
    assert res
    bad = {short(n): v for n, v in res.items()
           if v[1] and not short(n).startswith("gridder_general<")}
    assert not bad, bad


def test_l2_prefetch_is_not_drained_before_the_mfma_loop(listings):
    # The gridder pulls each next fill's rows into L2 with a 4-byte LDS-DMA
    # issued as inline asm after the fill barrier.  A
    # compiler vmcnt wait between it and the MFMA loop (e.g. for a spill
    # reload) would expose its whole latency once per fill.
    # Required of every mirror-path kernel and of the S = 32 general one;
    # the S = 64 / runtime-S general-only kernels (w-terms at those sizes)
    # reload a spill before one of their MFMA loops.
    import dma_drain_check as ddc
    from resources import short
    res = ddc.check(open(listings["gridder"]).read())
    checked = []
    for name, total, drained, _ in res:
        k = short(name)
        if k.startswith("gridder_general<") and not k.startswith(
                "gridder_general<32,"):
            continue
        checked.append(k)
        assert total > 0 and drained == 0, (k, total, drained)
    # every precision variant (the last template argument, device.hpp kPrec*)
    # (the mirror kernel's last argument is SPLIT, its workgroups per
    # subgrid: 1 at S = 32)
    for form, tail in (("gridder_mirror<32,16,4,", ",1>"),
                       ("gridder_general<32,16,4,", ">")):
        for prec in ("0", "1", "3"):
            assert form + prec + tail in checked, checked


def test_lds_dma_m0_wait_state_checker():
    import dma_drain_check as ddc
    src = """
_Zk:
\ts_mov_b32 m0, s5
{pad}\tglobal_load_lds_dword v[2:3], off
\ts_endpgm
"""
    bad = ddc.check(src.format(pad=""), with_m0=True)
    ok = ddc.check(src.format(pad="\ts_nop 0\n"), with_m0=True)
    assert bad[0][4] == 1 and ok[0][4] == 0


def test_shipped_lds_dma_has_m0_wait_state(listings):
    # the asm's SALU write of M0 needs one wait state before the
    # LDS-DMA that reads it; the compiler cannot pad inside the asm string.
    import dma_drain_check as ddc
    res = ddc.check(open(listings["gridder"]).read(), with_m0=True)
    assert res, "no kernel with an LDS-DMA"
    for name, total, _, _, m0 in res:
        assert total > 0 and m0 == 0, (name[:60], total, m0)


def test_dpp_moves_of_vector_elements(tmp_path):
    # hipcc (ROCm 7.2) emits one DPP move of element 0 for a loop of
    # update_dpp over a float4's elements written inline (loop_form); the
    # kernels go through device.hpp row_ror8 on named scalars (scalar_form),
    # which must stay four moves (tools/probes/dpp_vector_probe.hip).
    out = tmp_path / "dpp.s"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3",
                    "-ffp-contract=off", "-I", os.path.join(PKG, "csrc"),
                    "--cuda-device-only", "-S", "-o", str(out),
                    os.path.join(REPO, "tools", "probes",
                                 "dpp_vector_probe.hip")],
                   check=True, capture_output=True, timeout=300)
    text = out.read_text()
    scalar = text[text.index("_Z11scalar_form"):]
    scalar = scalar[:scalar.index("s_endpgm")]
    assert scalar.count("row_ror:8") == 4
