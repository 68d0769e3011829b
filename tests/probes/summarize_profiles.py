"""Turn the rocprofv3 databases of tests/probes/profile_round.sh and
tests/probes/pmc_sq.sh (merged back under gpurun_out/) into the committed
profile summaries and profiles/traffic.json, which bench.py reads for
`roofline.traffic` and `roofline.issue_bound`.

    python tests/probes/summarize_profiles.py --prof gpurun_out/prof_TAG \
        --pmc gpurun_out/pmc_TAG --out profiles/r01/final [--workload default]

Per kernel (the MFMA gridder/degridder of the workload):
  * mean / min / max duration over the kernel-trace launches;
  * HBM bytes per launch: FETCH_SIZE x 2 + WRITE_SIZE (KiB), the gfx950
    correction of MI355X_MICROARCH.md (vector loads tallied at 64 B per
    128-B request), calibrated in profiles/r01/traffic_calibration.md;
  * VALU-issue utilisation: (trans x 8.35 + f16 MFMA x 4.7 + other VALU x 4.46
    cycles, tests/probes/instr_rates_probe.hip) / 1024 SIMDs / (GRBM_GUI_ACTIVE / 8
    XCDs).
"""
import argparse
import csv
import glob
import json
import os
import shutil
import subprocess
import tempfile
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(
    __file__))))
ROCPD2CSV = "/opt/rocm/bin/rocpd2csv"
CYC_TRANS, CYC_MFMA_F16, CYC_VALU = 8.35, 4.7, 4.46
N_SIMD, N_XCD = 1024, 8


def short_name(kernel_name):
    """'void idg_mi355x::kernel_gridder_mi355x<32, 4, 16, 1, 4>(...)' ->
    ('gridder', 32, MODE); None for other kernels."""
    for d, mode_arg in (("gridder", 3), ("degridder", 2)):
        tag = f"kernel_{d}_mi355x<"
        if tag in kernel_name:
            args = kernel_name.split(tag, 1)[1].split(">", 1)[0].split(",")
            return d, int(args[0]), int(args[mode_arg])
    return None


def bench_name(d, S):
    return f"{d}_mi355x_{'s%d' % S if S in (32, 64) else 'generic'}"


def to_csv(db, kind):
    """Convert one rocpd database; returns the path of the wanted CSV."""
    out = tempfile.mkdtemp(prefix="rocpd_")
    subprocess.run([ROCPD2CSV, "-i", db, "-d", out], check=True,
                   stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    want = {"kernel": "out_kernel_trace.csv",
            "counter": "out_counter_collection_trace.csv"}[kind]
    path = os.path.join(out, want)
    if not os.path.exists(path):
        raise SystemExit(f"{db}: no {want}")
    return path


def read_rows(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def kernel_stats(rows):
    acc = defaultdict(list)
    for r in rows:
        k = short_name(r["Kernel_Name"])
        if k and k[2] == 1:
            acc[bench_name(k[0], k[1])].append(
                int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return {n: {"launches": len(v), "mean_ns": sum(v) / len(v),
                "min_ns": min(v), "max_ns": max(v)} for n, v in acc.items()}


def counters(rows):
    """{kernel: {counter: mean over launches}} (values summed per dispatch
    over the rows rocprofv3 writes per dimension)."""
    per = defaultdict(lambda: defaultdict(float))
    for r in rows:
        k = short_name(r["Kernel_Name"])
        if not (k and k[2] == 1):
            continue
        per[(bench_name(k[0], k[1]), r["Dispatch_Id"])][r["Counter_Name"]] += \
            float(r["Counter_Value"])
    out = defaultdict(lambda: defaultdict(list))
    for (name, _), cs in per.items():
        for c, v in cs.items():
            out[name][c].append(v)
    return {n: {c: sum(v) / len(v) for c, v in cs.items()}
            for n, cs in out.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prof", required=True)
    ap.add_argument("--pmc", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--workload", default="default")
    ap.add_argument("--traffic", default=os.path.join(REPO, "profiles",
                                                      "traffic.json"))
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)

    ktrace = to_csv(glob.glob(os.path.join(args.prof, "ktrace", "**",
                                           "*.db"), recursive=True)[0],
                    "kernel")
    shutil.copy(ktrace, os.path.join(args.out, "kernel_trace.csv"))
    stats = kernel_stats(read_rows(ktrace))

    traffic = {}
    for cname, sub in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
        db = glob.glob(os.path.join(args.prof, sub, "**", "*.db"),
                       recursive=True)[0]
        path = to_csv(db, "counter")
        shutil.copy(path, os.path.join(args.out,
                                       f"{sub}_counter_collection.csv"))
        for n, cs in counters(read_rows(path)).items():
            traffic.setdefault(n, {})[cname] = cs[cname]

    sq = defaultdict(dict)
    for db in sorted(glob.glob(os.path.join(args.pmc, "p*", "**", "*.db"),
                               recursive=True)):
        for n, cs in counters(read_rows(to_csv(db, "counter"))).items():
            sq[n].update(cs)

    with open(args.traffic) as f:
        tj = json.load(f)
    wl = tj.setdefault(args.workload, {})
    summary = {"counters": sq, "issue_bound": {}}
    lines = [f"{'kernel':28s} {'launches':>8s} {'mean ms':>9s} {'min ms':>8s} "
             f"{'max ms':>8s} {'HBM GB':>8s} {'VALU issue':>10s}"]
    for n in sorted(stats):
        st = stats[n]
        t = traffic.get(n, {})
        hbm = None
        if "FETCH_SIZE" in t and "WRITE_SIZE" in t:
            hbm = int((2 * t["FETCH_SIZE"] + t["WRITE_SIZE"]) * 1024)
        c = sq.get(n, {})
        issue = None
        if all(k in c for k in ("SQ_INSTS_VALU", "SQ_INSTS_VALU_TRANS_F32",
                                "SQ_INSTS_VALU_MFMA_F16", "GRBM_GUI_ACTIVE")):
            other = (c["SQ_INSTS_VALU"] - c["SQ_INSTS_VALU_TRANS_F32"]
                     - c["SQ_INSTS_VALU_MFMA_F16"])
            cyc = (c["SQ_INSTS_VALU_TRANS_F32"] * CYC_TRANS
                   + c["SQ_INSTS_VALU_MFMA_F16"] * CYC_MFMA_F16
                   + other * CYC_VALU) / N_SIMD
            per_simd = c["GRBM_GUI_ACTIVE"] / N_XCD
            issue = {
                "resource": "VALU issue per SIMD",
                "utilization": round(cyc / per_simd, 3),
                "model": ("(trans x 8.35 + f16 MFMA x 4.7 + other VALU x 4.46 "
                          "cycles, tests/probes/instr_rates_probe.hip) / "
                          "(GRBM_GUI_ACTIVE / 8 XCDs), summed over 1024 SIMDs"),
                "insts_valu": c["SQ_INSTS_VALU"],
                "insts_trans": c["SQ_INSTS_VALU_TRANS_F32"],
                "insts_mfma_f16": c["SQ_INSTS_VALU_MFMA_F16"],
                "cycles_per_simd": per_simd,
                "source": os.path.relpath(
                    os.path.join(args.out, "pmc_sq_summary.json"), REPO),
            }
            summary["issue_bound"][n] = issue
        entry = wl.setdefault(n, {})
        if hbm is not None:
            entry.update({
                "hbm_bytes_per_launch": hbm,
                "fetch_kib_raw": t["FETCH_SIZE"],
                "write_kib_raw": t["WRITE_SIZE"],
                "source": os.path.relpath(args.out, REPO)
                + "/fetch_counter_collection.csv + write_counter_collection.csv",
            })
        if issue:
            entry["issue_bound"] = issue
        entry["mean_ms_under_rocprof"] = round(st["mean_ns"] / 1e6, 4)
        lines.append(
            f"{n:28s} {st['launches']:8d} {st['mean_ns'] / 1e6:9.4f} "
            f"{st['min_ns'] / 1e6:8.4f} {st['max_ns'] / 1e6:8.4f} "
            f"{(hbm or 0) / 1e9:8.3f} "
            f"{issue['utilization'] if issue else float('nan'):10.3f}")
    with open(os.path.join(args.out, "pmc_sq_summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    with open(os.path.join(args.out, "kernel_stats_summary.txt"), "w") as f:
        f.write(f"rocprofv3 --kernel-trace --stats of bench.py ({args.workload} "
                "workload); per-launch means over the traced launches\n")
        f.write("\n".join(lines) + "\n")
    with open(args.traffic, "w") as f:
        json.dump(tj, f, indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
