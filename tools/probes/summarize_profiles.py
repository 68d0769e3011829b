"""Turn the rocprofv3 databases of tools/probes/profile_round.sh and
tools/probes/pmc_sq.sh (merged back under gpurun_out/) into the committed
profile summaries and profiles/traffic.json, which bench.py reads for
`roofline.traffic` and `roofline.issue_bound`.

    python tools/probes/summarize_profiles.py --prof gpurun_out/prof_TAG \
        --pmc gpurun_out/pmc_TAG --out profiles/r01/final [--workload default]

Per kernel (the MFMA gridder/degridder of the workload):
  * mean / min / max duration over the kernel-trace launches;
  * HBM bytes per launch: FETCH_SIZE x 2 + WRITE_SIZE (KiB), the gfx950
    correction of MI355X_MICROARCH.md (vector loads tallied at 64 B per
    128-B request), calibrated in profiles/r01/traffic_calibration.md;
  * VALU-issue utilisation: (trans x 8.35 + f16 MFMA x 4.7 + other VALU x 4.46
    cycles, tools/probes/instr_rates_probe.hip) / 1024 SIMDs / (GRBM_GUI_ACTIVE / 8
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
# Round 4: with the VALU class counters (pmc_sq.sh's optional passes) the
# "other" VALU is priced per class: v_cvt_pk_f16_f32 (CVT) 4.5, the FMA_F32
# class 4.58 (v_fma_mix_f32 4.46 and v_pk_fma_f32 4.8 in the loops' 2:1
# mix, tools/probes/isa_loops.py), everything else at the plain f32 /
# integer rate 2.6 (v_fma_f32, v_add_f32, v_mov_b32 2.5-2.7 in
# instr_rates_probe.hip).
CYC_CLASS = {"SQ_INSTS_VALU_CVT": 4.5, "SQ_INSTS_VALU_FMA_F32": 4.58}
CYC_PLAIN = 2.6
N_SIMD, N_XCD = 1024, 8


KERNELS = (  # name tag -> (direction, variant); S is the first template arg
    ("kernel_gridder_mirror_mi355x<", "gridder", "mirror"),
    ("kernel_gridder_general_mi355x<", "gridder", "general_queue"),
    ("kernel_gridder_mi355x<", "gridder", "combined"),
    ("kernel_degridder_mirror_mi355x<", "degridder", "mirror"),
    ("kernel_degridder_general_direct_mi355x<", "degridder", "general_direct"),
    ("kernel_degridder_general_mi355x<", "degridder", "general_queue"),
    ("kernel_degridder_mi355x<", "degridder", "combined"),
)
PIPELINE = ("kernel_subgrid_fft_reg", "kernel_subgrid_fft2", "kernel_subgrid_dft",
            "kernel_home_count", "kernel_home_place", "kernel_home_scan",
            "kernel_home_key",
            "kernel_adder_bin_scan", "kernel_adder_bin", "kernel_adder",
            "kernel_splitter_key", "kernel_splitter_pairs", "kernel_splitter",
            "kernel_splitter_fft")


def short_name(kernel_name):
    """'void idg_mi355x::kernel_gridder_mirror_mi355x<32, 16, 4>(...)' ->
    ('gridder', 32, 'mirror'); the combined kernel's VALU instantiation
    (MODE 0) and other kernels -> None."""
    for tag, d, variant in KERNELS:
        if tag in kernel_name:
            args = kernel_name.split(tag, 1)[1].split(">", 1)[0].split(",")
            if args[-1].strip() == "true":  # FFT epilogue: a pipeline kernel
                return None
            if variant == "combined":
                mode = int(args[3] if d == "gridder" else args[2])
                if mode != 1:
                    return None
            return d, int(args[0]), variant
    return None


def pipeline_name(kernel_name):
    for tag, d, variant in KERNELS:  # the gridder's FFT-epilogue kernels
        if d == "gridder" and tag in kernel_name and \
                kernel_name.split(tag, 1)[1].split(">", 1)[0].endswith("true"):
            return "gridder_fft_" + variant
    for tag in PIPELINE:
        if "::" + tag + "<" in kernel_name or "::" + tag + "(" in kernel_name:
            return tag[len("kernel_"):]
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
    """{(bench kernel, variant): duration stats} and the pipeline kernels'
    {name: stats}."""
    acc, pipe = defaultdict(list), defaultdict(list)
    for r in rows:
        dt = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        k = short_name(r["Kernel_Name"])
        if k:
            acc[(bench_name(k[0], k[1]), k[2])].append(dt)
        else:
            pn = pipeline_name(r["Kernel_Name"])
            if pn:
                pipe[pn].append(dt)

    def st(v):
        return {"launches": len(v), "mean_ns": sum(v) / len(v),
                "min_ns": min(v), "max_ns": max(v)}
    return ({k: st(v) for k, v in acc.items()},
            {k: st(v) for k, v in pipe.items()})


def counters(rows):
    """{(bench kernel, variant) or pipeline name: {counter: mean over
    launches}} (values summed per dispatch over the rows rocprofv3 writes
    per dimension)."""
    per = defaultdict(lambda: defaultdict(float))
    for r in rows:
        k = short_name(r["Kernel_Name"])
        key = (bench_name(k[0], k[1]), k[2]) if k else \
            pipeline_name(r["Kernel_Name"])
        if key is None:
            continue
        per[(key, r["Dispatch_Id"])][r["Counter_Name"]] += \
            float(r["Counter_Value"])
    out = defaultdict(lambda: defaultdict(list))
    for (key, _), cs in per.items():
        for c, v in cs.items():
            out[key][c].append(v)
    return {n: {c: sum(v) / len(v) for c, v in cs.items()}
            for n, cs in out.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prof", required=True)
    ap.add_argument("--pmc", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--workload", default="default")
    ap.add_argument("--nr-subgrids", type=int, default=None,
                    help="subgrids of the profiled launch (bench.py scales "
                         "the per-launch figures to its own launch by it)")
    ap.add_argument("--note", default=None,
                    help="the profiled workload, stored with each entry")
    ap.add_argument("--traffic", default=os.path.join(REPO, "profiles",
                                                      "traffic.json"))
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)

    ktrace = to_csv(glob.glob(os.path.join(args.prof, "ktrace", "**",
                                           "*.db"), recursive=True)[0],
                    "kernel")
    shutil.copy(ktrace, os.path.join(args.out, "kernel_trace.csv"))
    vstats, pstats = kernel_stats(read_rows(ktrace))

    traffic = {}
    for cname, sub in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
        db = glob.glob(os.path.join(args.prof, sub, "**", "*.db"),
                       recursive=True)[0]
        path = to_csv(db, "counter")
        shutil.copy(path, os.path.join(args.out,
                                       f"{sub}_counter_collection.csv"))
        for n, cs in counters(read_rows(path)).items():
            traffic.setdefault(n, {})[cname] = cs[cname]

    sq_v = defaultdict(dict)
    for db in sorted(glob.glob(os.path.join(args.pmc, "p*", "**", "*.db"),
                               recursive=True)):
        for n, cs in counters(read_rows(to_csv(db, "counter"))).items():
            sq_v[n].update(cs)

    # One step launches every variant of a direction at most once: the
    # direction's per-launch figures are the sums over its variants.
    stats, sq, vtraffic = {}, defaultdict(lambda: defaultdict(float)), \
        defaultdict(lambda: defaultdict(float))
    for (n, variant), st in vstats.items():
        s0 = stats.setdefault(n, {"launches": 0, "mean_ns": 0.0,
                                  "min_ns": 0.0, "max_ns": 0.0,
                                  "variants": {}})
        s0["launches"] = max(s0["launches"], st["launches"])
        for key in ("mean_ns", "min_ns", "max_ns"):
            s0[key] += st[key]
        s0["variants"][variant] = round(st["mean_ns"] / 1e6, 4)
    for key, cs in sq_v.items():
        if isinstance(key, tuple):
            for c, v in cs.items():
                sq[key[0]][c] += v
    for key, cs in traffic.items():
        if isinstance(key, tuple):
            for c, v in cs.items():
                vtraffic[key[0]][c] += v

    with open(args.traffic) as f:
        tj = json.load(f)
    wl = tj.setdefault(args.workload, {})
    summary = {"counters": sq, "issue_bound": {}}
    lines = [f"{'kernel':28s} {'launches':>8s} {'mean ms':>9s} {'min ms':>8s} "
             f"{'max ms':>8s} {'HBM GB':>8s} {'VALU issue':>10s}"]
    for n in sorted(stats):
        st = stats[n]
        t = vtraffic.get(n, {})
        hbm = None
        if "FETCH_SIZE" in t and "WRITE_SIZE" in t:
            hbm = int((2 * t["FETCH_SIZE"] + t["WRITE_SIZE"]) * 1024)
        c = sq.get(n, {})
        issue = None
        if all(k in c for k in ("SQ_INSTS_VALU", "SQ_INSTS_VALU_TRANS_F32",
                                "SQ_INSTS_VALU_MFMA_F16", "GRBM_GUI_ACTIVE")):
            other = (c["SQ_INSTS_VALU"] - c["SQ_INSTS_VALU_TRANS_F32"]
                     - c["SQ_INSTS_VALU_MFMA_F16"])
            classed = all(k in c for k in CYC_CLASS)
            if classed:
                cls = {k: c[k] for k in CYC_CLASS}
                plain = other - sum(cls.values())
                other_cyc = (sum(c[k] * v for k, v in CYC_CLASS.items())
                             + plain * CYC_PLAIN)
                model = ("(trans x 8.35 + f16 MFMA x 4.7 + CVT x 4.5 + FMA_F32 "
                         "x 4.58 + the rest x 2.6 cycles, tools/probes/"
                         "instr_rates_probe.hip) / (GRBM_GUI_ACTIVE / 8 XCDs), "
                         "summed over 1024 SIMDs")
            else:
                other_cyc = other * CYC_VALU
                model = ("(trans x 8.35 + f16 MFMA x 4.7 + other VALU x 4.46 "
                         "cycles, tools/probes/instr_rates_probe.hip) / "
                         "(GRBM_GUI_ACTIVE / 8 XCDs), summed over 1024 SIMDs")
            cyc = (c["SQ_INSTS_VALU_TRANS_F32"] * CYC_TRANS
                   + c["SQ_INSTS_VALU_MFMA_F16"] * CYC_MFMA_F16
                   + other_cyc) / N_SIMD
            per_simd = c["GRBM_GUI_ACTIVE"] / N_XCD
            issue = {
                "resource": "VALU issue per SIMD",
                "utilization": round(cyc / per_simd, 3),
                "model": model,
                "insts_valu": c["SQ_INSTS_VALU"],
                "insts_trans": c["SQ_INSTS_VALU_TRANS_F32"],
                "insts_mfma_f16": c["SQ_INSTS_VALU_MFMA_F16"],
                "cycles_per_simd": per_simd,
                "source": os.path.relpath(
                    os.path.join(args.out, "pmc_sq_summary.json"), REPO),
            }
            if classed:
                issue["insts_class"] = dict(cls, plain=plain)
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
        if args.nr_subgrids:
            entry["nr_subgrids"] = args.nr_subgrids
        if args.note:
            entry["workload"] = args.note
        lines.append(
            f"{n:28s} {st['launches']:8d} {st['mean_ns'] / 1e6:9.4f} "
            f"{st['min_ns'] / 1e6:8.4f} {st['max_ns'] / 1e6:8.4f} "
            f"{(hbm or 0) / 1e9:8.3f} "
            f"{issue['utilization'] if issue else float('nan'):10.3f}")
        lines.append("    variants (mean ms): " + ", ".join(
            f"{v} {ms}" for v, ms in sorted(st["variants"].items())))
    # the pipeline steps either side of the path
    lines.append("")
    lines.append(f"{'pipeline kernel':28s} {'launches':>8s} {'mean ms':>9s} "
                 f"{'min ms':>8s} {'HBM GB':>8s} {'GB/s':>8s}")
    pipe = {}
    for n in sorted(pstats):
        st = pstats[n]
        t = traffic.get(n, {})
        hbm = None
        if "FETCH_SIZE" in t and "WRITE_SIZE" in t:
            hbm = int((2 * t["FETCH_SIZE"] + t["WRITE_SIZE"]) * 1024)
        pipe[n] = {"mean_ms": round(st["mean_ns"] / 1e6, 4),
                   "hbm_bytes_per_launch": hbm}
        lines.append(f"{n:28s} {st['launches']:8d} {st['mean_ns'] / 1e6:9.4f} "
                     f"{st['min_ns'] / 1e6:8.4f} {(hbm or 0) / 1e9:8.3f} "
                     f"{(hbm or 0) / st['mean_ns']:8.1f}")
    summary["pipeline"] = pipe
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
