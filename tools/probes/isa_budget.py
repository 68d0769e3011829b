"""Instruction budget of one phasor in the default gridder's MFMA loop: every
instruction of the hot loop body, its class and its role, and the issue
cycles per phasor-wave at the measured costs.

    python tools/probes/isa_budget.py ska-sdp-idg-bench_amd/build/isa/gridder_mi355x.s \
        kernel_gridder_mirror_mi355xILi32ELi16ELi4ELb0ELi1ELi1E [--json OUT]

The loop is the basic block with the most v_mfma (one K-step of every tile
pair of a wave).  Roles:
  trans      v_sin_f32 / v_cos_f32 of the revolutions (the floor: one pair
             per phasor of the reference's exact f32 phase)
  split      v_cvt_pk_f16_f32 (hi parts, then lo parts of two values) and
             v_fma_mix_f32 (the exact f32 residual x - hi): the two-term f16
             operand of the matrix core, 4 per two values
  phase      the reference's phase fma(-phase_index, k, phase_offset) and
             its revolutions fma(phase, 1/2pi_hi, -m): v_pk_fma_f32 / v_fma_f32
  tail       the reduction tail r + c (v_pk_add_f32 / v_add_f32)
  anchor     the block's revolution count m: v_pk_mul_f32, v_rndne_f32
  mfma       v_mfma_f32_16x16x32_f16
  wait       s_nop (wait states the hazard rules require between dependent
             packed / transcendental / MFMA-operand instructions)
  memory     ds_read (B fragments from LDS), s_waitcnt
  control    scalar loop / branch instructions
Costs (cycles per wave64 instruction, 8 waves per SIMD;
profiles/r02/rates/instr_rates_probe.txt, profiles/r06/rates/):
trans 8.35, cvt 4.5, fma_mix 4.46, packed f32 4.78, plain f32 2.7,
rndne 4.43, f16 MFMA 4.7 (its issue beside the split), s_nop 1 per wait
state not hidden by another wave (reported, not priced).
"""
import json
import re
import sys
from collections import Counter

COST = {"v_sin_f32_e32": 8.35, "v_cos_f32_e32": 8.35,
        "v_cvt_pk_f16_f32": 4.5, "v_fma_mix_f32": 4.46,
        "v_pk_fma_f32": 4.78, "v_pk_add_f32": 4.67, "v_pk_mul_f32": 4.7,
        "v_fma_f32": 2.7, "v_add_f32_e64": 2.5, "v_add_f32_e32": 2.5,
        "v_rndne_f32_e64": 4.43, "v_mfma_f32_16x16x32_f16": 4.7}
ROLE = {"v_sin_f32_e32": "trans", "v_cos_f32_e32": "trans",
        "v_cvt_pk_f16_f32": "split", "v_fma_mix_f32": "split",
        "v_pk_fma_f32": "phase", "v_fma_f32": "phase",
        "v_pk_add_f32": "tail", "v_add_f32_e64": "tail",
        "v_add_f32_e32": "tail", "v_pk_mul_f32": "anchor",
        "v_rndne_f32_e64": "anchor", "v_mfma_f32_16x16x32_f16": "mfma",
        "s_nop": "wait", "ds_read_b128": "memory", "ds_read_b64": "memory",
        "s_waitcnt": "memory"}


def hot_loop(src, pat):
    for f in re.split(r"\n(?=_Z\w+:)", src):
        if pat not in f.split(":")[0]:
            continue
        best = None
        for b in re.split(r"\n(?=\.LBB\d+_\d+:)", f):
            ins = [l.strip() for l in b.split("\n")[1:]
                   if l.strip() and not l.strip().startswith((".", ";", "//"))]
            n = sum("v_mfma" in l for l in ins)
            if n and (best is None or n > best[0]):
                best = (n, b.split("\n")[0].split(":")[0], ins)
        return best
    raise SystemExit(f"{pat}: not found")


def main():
    src = open(sys.argv[1]).read()
    nm, label, ins = hot_loop(src, sys.argv[2])
    c = Counter(l.split()[0] for l in ins)
    phasors = (c["v_sin_f32_e32"] + c["v_cos_f32_e32"]) // 2
    roles, cyc = Counter(), Counter()
    for k, v in c.items():
        r = ROLE.get(k, "control" if k.startswith("s_") else "other")
        roles[r] += v
        cyc[r] += v * COST.get(k, 0.0)
    per = {r: round(roles[r] / phasors, 3) for r in roles}
    cycles = {r: round(cyc[r] / phasors * 64 / 64, 2) for r in cyc if cyc[r]}
    total = sum(cyc.values()) / phasors
    out = {"block": label, "phasors_per_lane": phasors, "mfma": nm,
           "instructions": dict(sorted(c.items(), key=lambda x: -x[1])),
           "per_phasor": per,
           "issue_cycles_per_phasor_wave": cycles,
           "issue_cycles_total": round(total, 2)}
    print(json.dumps(out, indent=1))
    if "--json" in sys.argv:
        with open(sys.argv[sys.argv.index("--json") + 1], "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
