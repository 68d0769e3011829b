"""Static wait-state check of the shipped gfx950 kernels (ISA listing from
`make -C ska-sdp-idg-bench_amd isa`, the same flags as the library build).

hipcc pads the hazards of the instructions it emits, but models an inline asm
statement as one opaque instruction and pads nothing inside it
(cdna_hip_programming.md §5.7 item 2).  The MFMA A operands of the gridder
and degridder come out of inline-asm f16 splits (kernels/mfma.hpp), so the
wait states there are hand-placed; this checker verifies them on the final
listing, over every control-flow path into each consumer:

  * VALU write of a VGPR -> v_mfma_* reading it as SrcA or SrcB: >= 2 wait
    states (cdna_asm_programming.md Table 38; DESIGN.md §4.4 is the
    accumulator corruption this caused);
  * transcendental (v_sin/v_cos/v_exp/...) write -> VALU read: >= 1 wait
    state (gfx940+ trans forwarding).

Wait states between producer and consumer: `s_nop N` counts N + 1, every
other instruction 1.  Paths are followed backwards through labels into every
branch that targets them.

    python tools/probes/hazard_check.py build/isa/gridder_mi355x.s [...]
"""
import re
import sys
from collections import defaultdict

MFMA_SRC_STATES = 2
TRANS_STATES = 1
TRANS_OPS = ("v_sin_", "v_cos_", "v_exp_", "v_log_", "v_rcp_", "v_rsq_",
             "v_sqrt_")
_REG = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+)(?!\w))")


def regs_of(tok):
    """Register names ('v12', 'a3') an operand token covers."""
    out = set()
    for m in _REG.finditer(tok):
        kind = m.group(1)
        if m.group(4) is not None:
            out.add(f"{kind}{m.group(4)}")
        else:
            for r in range(int(m.group(2)), int(m.group(3)) + 1):
                out.add(f"{kind}{r}")
    return out


def parse_functions(text):
    """{function name: [("label", name) | ("inst", mnemonic, operands)]}"""
    funcs = {}
    cur = None
    for raw in text.split("\n"):
        line = raw.split(";")[0].rstrip()
        s = line.strip()
        if not s:
            continue
        m = re.match(r"^(_Z\w+):", line)
        if m:
            cur = funcs.setdefault(m.group(1), [])
            continue
        if cur is None:
            continue
        if s.startswith(".Lfunc_end"):
            cur = None
            continue
        m = re.match(r"^(\.LBB\w+):", s)
        if m:
            cur.append(("label", m.group(1)))
            continue
        if s.startswith("."):
            continue
        parts = s.split(None, 1)
        ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 \
            else []
        cur.append(("inst", parts[0], ops))
    return funcs


def _states(item):
    if item[1] == "s_nop":
        return int(item[2][0], 0) + 1
    return 1


def _is_valu(mn):
    return mn.startswith("v_") and not mn.startswith(
        ("v_mfma", "v_readfirstlane", "v_readlane", "v_cmp", "v_accvgpr_read"))


def _written(item):
    mn, ops = item[1], item[2]
    if not ops:
        return set()
    return regs_of(ops[0])


def check_function(body):
    """List of (kind, consumer index, producer index, states found)."""
    branches = defaultdict(list)   # label -> indices of branches to it
    for i, it in enumerate(body):
        if it[0] == "inst" and it[1].startswith(("s_branch", "s_cbranch")):
            if it[2]:
                branches[it[2][0]].append(i)
    viol = []

    def scan(start, need, regs, is_producer, kind, consumer):
        seen = set()
        stack = [(start, 0)]
        while stack:
            j, got = stack.pop()
            while j >= 0:
                if (j, got) in seen:
                    break
                seen.add((j, got))
                it = body[j]
                if it[0] == "label":
                    for b in branches.get(it[1], []):
                        stack.append((b, got))
                    prev = j - 1
                    if prev >= 0 and body[prev][0] == "inst" and \
                            body[prev][1] in ("s_branch", "s_endpgm"):
                        break
                    j -= 1
                    continue
                if is_producer(it) and (_written(it) & regs):
                    viol.append((kind, consumer, j, got))
                    break
                got += _states(it)
                if got >= need:
                    break
                j -= 1

    for i, it in enumerate(body):
        if it[0] != "inst":
            continue
        mn, ops = it[1], it[2]
        if mn.startswith("v_mfma") and len(ops) >= 3:
            src = regs_of(ops[1]) | regs_of(ops[2])
            scan(i - 1, MFMA_SRC_STATES, src,
                 lambda x: x[0] == "inst" and _is_valu(x[1]),
                 "valu->mfma_src", i)
        elif _is_valu(mn) and len(ops) >= 2:
            src = set()
            for o in ops[1:]:
                src |= regs_of(o)
            # v_fma_mix{lo,hi} and other partial writes also read their dst
            scan(i - 1, TRANS_STATES, src,
                 lambda x: x[0] == "inst" and x[1].startswith(TRANS_OPS),
                 "trans->valu", i)
    return viol


def check_file(path, name_filter=""):
    text = open(path).read()
    out = {}
    for name, body in parse_functions(text).items():
        if name_filter not in name:
            continue
        n_mfma = sum(1 for it in body if it[0] == "inst" and
                     it[1].startswith("v_mfma"))
        v = check_function(body)
        out[name] = {"mfma": n_mfma, "violations": [
            (k, body[c][1] + " " + ", ".join(body[c][2]),
             body[p][1] + " " + ", ".join(body[p][2]), got)
            for k, c, p, got in v]}
    return out


if __name__ == "__main__":
    bad = 0
    for path in sys.argv[1:]:
        for name, r in check_file(path).items():
            print(f"{path}: {name[:70]}: {r['mfma']} MFMA, "
                  f"{len(r['violations'])} violations")
            for v in r["violations"][:10]:
                print("   ", v)
            bad += len(r["violations"])
    sys.exit(1 if bad else 0)
