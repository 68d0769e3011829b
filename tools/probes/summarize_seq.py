"""Per-kernel summary of tools/debug/r06_seq_prof.sh output (the kernel trace
and the SQ class passes of the bit-exact "sequential" kernels, merged back
under gpurun_out/), with the issue model those kernels are priced on.

    python tools/probes/summarize_seq.py gpurun_out/r06_seq_TAG [--out F.json]
        [--traffic profiles/traffic.json --workload default]

Per kernel (gridder_sequential / degridder_sequential): the rocprof mean
duration, every SQ counter as its mean per dispatch, and
  * the VALU mix per class: f64 (FMA/MUL/ADD_F64), CVT, INT32 / INT64, the
    f32 classes, TRANS, and the rest;
  * issue model: each class at its measured wave64 issue cost on one SIMD
    with 8 waves resident (tools/probes/seq_rates_probe.hip,
    instr_rates_probe.hip; profiles/r06/rates/): the VOP3-only "quarter"
    instructions -- f64 FMA/MUL/ADD, conversions, integer multiplies, bit-field
    ops, packed f32 -- 4.4-5.0 cycles, the "plain" f32 / VOP2 integer ones
    (v_fma_f32, v_add_f32, v_add_u32, v_mov, logic) 2.5-3.0;
    t_issue = sum(class count x cost) / 1024 SIMDs / 2.4 GHz and
    frac = t_issue / measured duration (how close the kernel runs to its own
    instruction stream's issue floor).
SQ_INSTS_VALU_INT32 counts every 32-bit integer VALU op (adds, shifts, logic,
compares, multiplies) and the f32 classes count a packed v_pk_fma_f32 as one
instruction like a plain v_fma_f32; the split between quarter-rate
(multiplies, bfe) and plain int32, and between packed and plain f32, is taken
from the ISA listing of the inner loop (`--frac-int32-quarter`,
`--frac-f32-packed`).
"""
import argparse
import csv
import glob
import json
import os
import subprocess
import tempfile
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(
    __file__))))
ROCPD2CSV = "/opt/rocm/bin/rocpd2csv"
CLOCK_HZ, N_SIMD = 2.4e9, 1024
# measured issue cost per wave64 instruction (8 waves per SIMD),
# profiles/r06/rates/seq_rates.txt and profiles/r02/rates/instr_rates_probe.txt
COST = {"f64": 4.75, "cvt": 4.4, "int32_quarter": 4.55, "int32_plain": 2.6,
        "int64": 4.65, "fma_f32_pk": 4.75, "f32_plain": 2.75, "trans": 8.35,
        "other": 2.75}


def to_csv(db, kind):
    out = tempfile.mkdtemp(prefix="rocpd_")
    subprocess.run([ROCPD2CSV, "-i", db, "-d", out], check=True,
                   stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    want = {"kernel": "out_kernel_trace.csv",
            "counter": "out_counter_collection_trace.csv"}[kind]
    return os.path.join(out, want)


def rows(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def short(name):
    for tag in ("kernel_gridder_sequential_mi355x",
                "kernel_degridder_sequential_mi355x"):
        if tag in name:
            s = name.split(tag + "<", 1)[1].split(">", 1)[0]
            sz = {"32": "s32", "64": "s64"}.get(s.strip(), "generic")
            return tag[len("kernel_"):] + "_" + sz
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out")
    ap.add_argument("--traffic", help="merge each kernel's issue model into "
                    "this traffic.json (bench.py reads it)")
    ap.add_argument("--workload", default="default")
    ap.add_argument("--note", default=None)
    ap.add_argument("--nr-subgrids", type=int, default=None,
                    help="subgrids of the profiled launch (bench.py scales "
                         "the issue model to its own launch by it)")
    ap.add_argument("--frac-int32-quarter", type=float, default=0.35)
    ap.add_argument("--frac-f32-packed", type=float, default=None,
                    help="override both kernels' packed share of the f32 "
                         "class (default: gridder 0.9 -- per mirror pair "
                         "20 packed MAC ops beside 2 plain phase FMAs --, "
                         "degridder 0.75 -- per phasor 12 packed beside 4 "
                         "plain: phase_index and phase)")
    args = ap.parse_args()
    dur = defaultdict(list)
    for db in glob.glob(os.path.join(args.dir, "ktrace", "**", "*.db"),
                        recursive=True):
        for r in rows(to_csv(db, "kernel")):
            k = short(r["Kernel_Name"])
            if k:
                dur[k].append(int(r["End_Timestamp"]) -
                              int(r["Start_Timestamp"]))
    per = defaultdict(lambda: defaultdict(float))
    for db in sorted(glob.glob(os.path.join(args.dir, "p*", "**", "*.db"),
                               recursive=True)):
        for r in rows(to_csv(db, "counter")):
            k = short(r["Kernel_Name"])
            if k:
                per[(k, db, r["Dispatch_Id"])][r["Counter_Name"]] += \
                    float(r["Counter_Value"])
    cnt = defaultdict(lambda: defaultdict(list))
    for (k, _, _), cs in per.items():
        for c, v in cs.items():
            cnt[k][c].append(v)
    out = {}
    for k in sorted(set(dur) | set(cnt)):
        c = {n: sum(v) / len(v) for n, v in cnt[k].items()}
        d = dur.get(k, [])
        e = {"launches": len(d),
             "mean_ms": round(sum(d) / len(d) / 1e6, 4) if d else None,
             "counters": {n: round(v) for n, v in sorted(c.items())}}
        if "SQ_INSTS_VALU" in c and d:
            f64 = sum(c.get(n, 0) for n in ("SQ_INSTS_VALU_FMA_F64",
                                            "SQ_INSTS_VALU_MUL_F64",
                                            "SQ_INSTS_VALU_ADD_F64",
                                            "SQ_INSTS_VALU_TRANS_F64"))
            cvt = c.get("SQ_INSTS_VALU_CVT", 0)
            i32 = c.get("SQ_INSTS_VALU_INT32", 0)
            i64 = c.get("SQ_INSTS_VALU_INT64", 0)
            f32 = sum(c.get(n, 0) for n in ("SQ_INSTS_VALU_FMA_F32",
                                            "SQ_INSTS_VALU_ADD_F32",
                                            "SQ_INSTS_VALU_MUL_F32"))
            trans = c.get("SQ_INSTS_VALU_TRANS_F32", 0)
            other = c["SQ_INSTS_VALU"] - f64 - cvt - i32 - i64 - f32 - trans
            q = args.frac_int32_quarter
            pk = args.frac_f32_packed
            if pk is None:
                pk = 0.9 if k.startswith("gridder") else 0.75
            cyc = (f64 * COST["f64"] + cvt * COST["cvt"] +
                   i32 * (q * COST["int32_quarter"] +
                          (1 - q) * COST["int32_plain"]) +
                   i64 * COST["int64"] +
                   f32 * (pk * COST["fma_f32_pk"] + (1 - pk) * COST["f32_plain"]) +
                   trans * COST["trans"] + max(other, 0) * COST["other"])
            t_issue = cyc / N_SIMD / CLOCK_HZ
            t = e["mean_ms"] / 1e3
            e["valu_mix"] = {"f64": f64, "cvt": cvt, "int32": i32,
                             "int64": i64, "f32": f32, "trans_f32": trans,
                             "other": other, "total": c["SQ_INSTS_VALU"]}
            e["issue_model"] = {
                "t_issue_ms": round(t_issue * 1e3, 4),
                "frac": round(t_issue / t, 4),
                "costs": COST, "frac_int32_quarter": q,
                "frac_f32_packed": pk,
                "note": "class counts x measured issue cost / 1024 SIMDs / "
                        "2.4 GHz over the rocprof mean duration; the SQ "
                        "classes do not tell packed from plain f32 or "
                        "quarter-rate from plain int32, so those splits come "
                        "from the inner loop's ISA listing"}
            if "GRBM_GUI_ACTIVE" in c and "SQ_BUSY_CYCLES" in c:
                e["sq_busy_frac"] = round(c["SQ_BUSY_CYCLES"] /
                                          max(c["GRBM_GUI_ACTIVE"], 1), 4)
        out[k] = e
    text = json.dumps(out, indent=1)
    if args.out:
        with open(args.out, "w") as f:
            f.write(text + "\n")
    if args.traffic:
        with open(args.traffic) as f:
            tj = json.load(f)
        wl = tj.setdefault(args.workload, {})
        src = os.path.relpath(args.out, REPO) if args.out else args.dir
        for k, e in out.items():
            if "issue_model" not in e:
                continue
            ent = wl.setdefault(k, {})
            ent.update({"issue_model": dict(e["issue_model"], source=src,
                                            valu_mix=e["valu_mix"]),
                        "mean_ms_under_rocprof": e["mean_ms"]})
            if args.note:
                ent["workload"] = args.note
            if args.nr_subgrids:
                ent["nr_subgrids"] = args.nr_subgrids
        with open(args.traffic, "w") as f:
            json.dump(tj, f, indent=1)
    print(text)


if __name__ == "__main__":
    main()
