#!/usr/bin/env python3
"""bench.py -- IDG gridder + degridder throughput on MI355X (BASELINE.json metric).

One step = one gridder pass + one degridder pass over one batch of the
workload, both kernels on the same HIP stream, inputs resident in HBM.  The
batch is BASELINE.json configs[1], the reference's perf defaults
(app/HIP/util.cpp:181-187): NR_STATIONS=50, NR_TIMESLOTS=20,
NR_TIMESTEPS_SUBGRID=128, NR_CHANNELS=16, SUBGRID_SIZE=32, GRID_SIZE=1024
-> 24,500 subgrids, 50.176 M visibilities, made by the reference's own
synthetic generators (srand(0)).

With N GPUs (one process per GPU, torchrun) the ONE batch is sharded
(BASELINE configs[3]): idg_amd.shard.plan_shards cuts the subgrids into N
contiguous ranges of equal cost, every rank uploads only its range's
metadata (rebased), uvw and visibility rows and degridder-input subgrids, and
grids / degrids just those (3,062-3,063 subgrids per GPU at N = 8).  No
collective on the data path; `value` = the batch's visibilities / the max
over ranks of the timed region (strong scaling).  The per-rank full-batch
(replicated, weak-scaling) figure is measured too and reported beside it as
`weak_scaling`; `--mode replicated` makes it the headline instead.

`value` counts a visibility once per step (it is gridded AND degridded);
per-kernel Mvis/s are reported alongside.  `roofline` is for the dominant
(slower) kernel -- see roofline_for() and DESIGN.md §4.3: the hardware floor
is the transcendental unit (v_sin + v_cos of the reference's exact f32 phase
for every phasor), so `frac` is that floor's time over the measured time;
the kernel's issue efficiency (its own instruction stream at the measured
issue costs), the f16-MFMA and the FP32-equivalent views sit beside it.
cpu_baseline times the reference's own CPU path (oracle/_ref) on a bounded
sample of the same batch, on the host cores this process may use and on one
thread as the reference builds it.

Beside `value` (never in it), a one-GPU default run also times: the `wterm`
batch; the bit-exact order-preserving kernels (`sequential`, with their own
issue-model roofline, and `sequential.configs2`: configs[2] at NR_TIMESLOTS=4
with the order-preserving gridder); and BASELINE configs[2] (`configs2`, C =
256 at NR_TIMESLOTS=4) and configs[4] (`configs4`, S = 64, the full batch) on
the default kernels, each with its roofline, counter traffic and issue
efficiency priced from the committed profile of the same launch
(profiles/traffic.json).

    python bench.py [--gpus N --steps K --warmup W] [--workload default]
                    [--mode sharded|replicated] [--dump DIR]

`--gpus N` with N > 1 works both under torchrun (one rank per GPU, RANK /
LOCAL_RANK / WORLD_SIZE / MASTER_* from the environment) and as a plain
command: without WORLD_SIZE the process touches no device, starts
`torch.distributed.run --nproc-per-node N` on itself as a child (rendezvous
on 127.0.0.1), and exits with its exit code (non-zero if any rank failed);
rank 0's JSON line is the output.  `--plan-only` stops each rank after the
rendezvous and the shard plan (no device needed: the launcher and sharding
rehearsed on CPU with IDG_DIST_BACKEND=gloo, tests/test_distributed.py).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "ska-sdp-idg-bench_amd"))

METRIC = "Mvisibilities/s (gridder & degridder) at 1/2/4/8 GPUs; % HBM roofline"
CLOCK_HZ = 2.4e9            # MI355X_MICROARCH.md: max engine clock
FP32_PEAK_TFLOPS = 157.3    # MI355X_MICROARCH.md: FP32 vector = FP32 matrix
F16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: BF16/F16 MFMA, dense
HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# Issue cost per wave64 instruction on one SIMD, in cycles at 2.4 GHz, the
# lower end of the isolated-probe costs (profiles/r02/rates/): v_sin/v_cos
# 8.35 (instr_rates_probe.hip), "other" = the VOP3/VOP3P class that makes up
# 97% of the MFMA loops' remaining VALU (v_cvt_pk_f16_f32 4.5, v_fma_mix_f32
# 4.46, v_pk_fma_f32 4.8), f16 MFMA 4.7 beside the split that feeds it
# (split_rates_probe.hip: split + 2 dependent MFMAs - split alone, per MFMA).
ISSUE_CYC = {"trans": 8.35, "mfma_f16": 4.7, "other": 4.46,
             # per-class prices (round 4): v_cvt_pk_f16_f32; the FMA_F32
             # class = v_fma_mix_f32 4.46 and v_pk_fma_f32 4.8 in the loops'
             # 2:1 mix; plain f32 / integer VALU (v_fma_f32, v_add_f32,
             # v_mov_b32: 2.5-2.7)
             "cvt": 4.5, "fma_f32": 4.58, "plain": 2.6}
MFMA_F16_FLOP = 16 * 16 * 32 * 2  # v_mfma_f32_16x16x32_f16
NR_SIMDS = 1024

WORKLOADS = {
    # BASELINE.json configs[1] (the metric's config)
    "default": dict(nr_stations=50, nr_timeslots=20, nr_timesteps=128,
                    nr_channels=16, grid_size=1024, subgrid_size=32),
    # configs[2]: large channel count (25.7 GB of visibilities per batch)
    "c256": dict(nr_stations=50, nr_timeslots=20, nr_timesteps=128,
                 nr_channels=256, grid_size=1024, subgrid_size=32),
    # configs[4]: large subgrid, A-term + spheroidal
    "s64": dict(nr_stations=50, nr_timeslots=20, nr_timesteps=128,
                nr_channels=16, grid_size=1024, subgrid_size=64),
    # the default batch with w-terms -- w ~ U(-200, 200)
    # per timestep, W_STEP = 2.5 and w-layers z in [0, 7) -- so every
    # subgrid takes the general (non-mirror) path
    "wterm": dict(nr_stations=50, nr_timeslots=20, nr_timesteps=128,
                  nr_channels=16, grid_size=1024, subgrid_size=32,
                  w_range=200.0, w_step=2.5, w_layers=7),
}
BASELINE_CONFIG = {"default": "configs[1]", "c256": "configs[2]",
                   "s64": "configs[4]", "wterm": "SURVEY.md §8f row 4"}


def apply_wterms(w, a):
    """w-terms of the 'wterm' workload, in place (seeded, numpy)."""
    import numpy as np
    if not w.get("w_range"):
        return
    rng = np.random.default_rng(7)
    a["uvw"][..., 2] = rng.uniform(-w["w_range"], w["w_range"],
                                   a["uvw"].shape[:2])
    a["metadata"]["z"] = rng.integers(0, w["w_layers"], a["metadata"].size)


def progress(msg):
    """One progress line on stderr (a long workload's phases: batch
    generation, upload, timing, pipeline, CPU baseline), so a run that
    takes minutes is seen to be alive."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr,
          flush=True)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="must equal the torchrun world size (1 without it)")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    # 5 s: long enough that a sampler of GPU activity at a few-second
    # interval sees the device busy before the timed steps (1 s: 3,292 /
    # 3,287 Mvis/s, 5 s: 3,289 / 3,281, same box, profiles/r06/warmup/)
    ap.add_argument("--min-warmup-s", type=float, default=5.0,
                    help="continue the untimed warm-up to at least this many "
                         "seconds of back-to-back steps (clock ramp, "
                         "DESIGN.md section 6); 0 = exactly --warmup steps")
    ap.add_argument("--workload", default="default", choices=sorted(WORKLOADS))
    ap.add_argument("--mode", default="sharded",
                    choices=("sharded", "replicated"),
                    help="sharded: the one batch split over the ranks "
                         "(strong scaling, BASELINE configs[3]); replicated: "
                         "every rank processes the whole batch (weak)")
    ap.add_argument("--timeslots", type=int, default=None,
                    help="override NR_TIMESLOTS (batch size)")
    ap.add_argument("--cpu-sample-subgrids", type=int, default=128,
                    help="subgrids per host thread in the cpu_baseline at "
                         "C = 16, S = 32 (scaled to the same work for other "
                         "C and S)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="skip timing the FFT / adder / grid-sum / splitter")
    ap.add_argument("--no-weak", action="store_true",
                    help="skip the replicated (weak-scaling) side figure")
    ap.add_argument("--no-side", action="store_true",
                    help="skip the side legs of a one-GPU default run (the "
                         "wterm batch and the sequential kernels; profiling "
                         "runs pass it so only the headline launches are "
                         "counted)")
    ap.add_argument("--no-workload-legs", action="store_true",
                    help="skip the configs[2] / configs[4] side legs of a "
                         "one-GPU default run (the wterm and sequential "
                         "legs still run)")
    ap.add_argument("--dump", default=None,
                    help="rank 0 writes the gathered gridder subgrids, "
                         "degridded visibilities and summed uv grid here "
                         "(.npy; tests/test_gpu_dist.py)")
    ap.add_argument("--traffic-file", default=os.path.join(
        REPO, "profiles", "traffic.json"))
    ap.add_argument("--plan-only", action="store_true",
                    help="rendezvous, shard the batch and print the plan "
                         "line (value null); no device is touched")
    return ap.parse_args(argv)


def launch_ranks(args, argv):
    """`--gpus N` (N > 1) run as a plain command: start one rank per GPU
    with torch.distributed.run as a CHILD process (never exec: the parent
    has not touched the GPU, and on this pool a process that has must not
    be replaced) and return its exit code, which is non-zero when any rank
    failed.  The ranks inherit stdout, so rank 0's JSON line is this
    command's output."""
    import socket
    import subprocess
    argv = list(sys.argv[1:] if argv is None else argv)
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", str(args.gpus), "--master-addr", "127.0.0.1",
           "--master-port", str(port), os.path.abspath(__file__)] + argv
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    sys.stdout.flush()
    return subprocess.run(cmd, env=env).returncode


# ---------------------------------------------------------------------------
# Batch and shards (host side; imported by tests/test_distributed.py)
# ---------------------------------------------------------------------------
def workload(name, timeslots=None):
    w = dict(WORKLOADS[name])
    if timeslots:
        w["nr_timeslots"] = timeslots
    return w


def make_batch(w, nthreads=8):
    """The whole batch on the host: the reference generators (srand(0)),
    identical on every rank, plus the workload's w-terms."""
    import idg_amd
    a = idg_amd.generate(w["nr_stations"], w["nr_timeslots"],
                         w["nr_timesteps"], w["nr_channels"], w["grid_size"],
                         w["subgrid_size"], nthreads=nthreads)
    apply_wterms(w, a)
    return a


def shard_batch(a, rank, world, mode="sharded"):
    """This rank's part of the batch: subgrid range [s0, s1) of
    shard.plan_shards, its metadata rebased to its own row space
    (shard.shard), and ONLY the uvw / visibility rows and degridder-input
    subgrids that range reads.  Replicated, spheroidal / A-terms /
    wavenumbers.  mode="replicated" returns the whole batch."""
    import numpy as np
    from idg_amd import shard
    md = a["metadata"]
    C = a["wavenumbers"].size
    uvw_rows = a["uvw"].reshape(-1, 3)
    vis_rows = a["visibilities"].reshape(-1, C, 4, 2)
    if mode == "replicated" or world == 1:
        s0, s1 = 0, md.size
        sub, r0, r1 = shard.shard(md, s0, s1)
    else:
        s0, s1 = shard.plan_shards(md, world)[rank]
        sub, r0, r1 = shard.shard(md, s0, s1)
    return {
        "s0": s0, "s1": s1, "row0": r0, "row1": r1,
        "metadata": sub,
        "uvw": np.ascontiguousarray(uvw_rows[r0:r1]),
        "visibilities": np.ascontiguousarray(vis_rows[r0:r1]),
        "subgrids": np.ascontiguousarray(a["subgrids"][s0:s1]),
        "wavenumbers": a["wavenumbers"], "spheroidal": a["spheroidal"],
        "aterms": a["aterms"],
    }


def shard_counts(a, world, mode="sharded"):
    """Subgrids per rank, in rank order (for gathers)."""
    from idg_amd import shard
    if mode == "replicated" or world == 1:
        return [a["metadata"].size] * world
    return [s1 - s0 for s0, s1 in shard.plan_shards(a["metadata"], world)]


# ---------------------------------------------------------------------------
# CPU baseline (the reference's own CPU path; test infrastructure)
# ---------------------------------------------------------------------------
def host_cpus():
    """The host CPUs this process may use: the affinity mask, capped by a
    cgroup CPU quota when there is one (on the GPU box `nproc` shows the
    whole machine while the job gets a share of it)."""
    import math
    info = {"nproc": os.cpu_count()}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except Exception:
        info["affinity"] = os.cpu_count()
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
        if q != "max":
            quota = max(1, math.floor(int(q) / int(period)))
    except Exception:
        pass
    info["cgroup_quota"] = quota
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    info["model"] = line.split(":", 1)[1].strip()
                    break
    except Exception:
        pass
    usable = info["affinity"] or 1
    if quota:
        usable = min(usable, quota)
    info["usable"] = usable
    return info


def cpu_baseline(w, a, nsample):
    """Time the reference CPU path (oracle/_ref, else the oracle port) on
    a bounded sample of the batch: on every usable host core (`value`) and
    on one thread as the reference builds it (`single_thread`).  Test
    infrastructure only: the baseline the GPU number is reported beside,
    never the measured path."""
    import numpy as np
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as orc
    T, C, S = w["nr_timesteps"], w["nr_channels"], w["subgrid_size"]
    # the sample is sized for configs[1] (C = 16, S = 32: ~7 s on one core);
    # other workloads take the same work per thread (c256: 8 subgrids, s64: 32)
    nsample = max(8, nsample * 16 * 32 * 32 // (C * S * S))
    n = min(nsample, a["metadata"].size)
    md = a["metadata"][:n]
    args = (n, w["grid_size"], S, 0.01, w.get("w_step", 0.0), C,
            w["nr_stations"])
    if orc.Reference.available(portable=True):
        impl, kind = orc.Reference(portable=True), "reference"
        extra = {}
    else:
        impl, kind = orc.Oracle(), "port"
        extra = {"nthreads": 1}
    sg = np.zeros((n, 4, S, S, 2), np.float32)
    t0 = time.perf_counter()
    impl.gridder(*args, a["uvw"], a["wavenumbers"], a["visibilities"],
                 a["spheroidal"], a["aterms"], md, sg, **extra)
    t1 = time.perf_counter()
    vis = np.zeros((n, T, C, 4, 2), np.float32)
    impl.degridder(*args, a["uvw"], a["wavenumbers"], vis, a["spheroidal"],
                   a["aterms"], md, np.ascontiguousarray(a["subgrids"][:n]),
                   **extra)
    t2 = time.perf_counter()
    nvis = n * T * C
    src = ("oracle/_ref/libidgref_v3.so (reference app/CPU)"
           if kind == "reference" else "oracle/liboracle.so")
    single = {
        "value": round(nvis / (t2 - t0) / 1e6, 4),
        "cores": 1,
        "sample": (f"first {n} subgrids of the same batch ({nvis} vis), "
                   f"gridder {t1 - t0:.2f} s + degridder {t2 - t1:.2f} s, "
                   f"{src}, single thread as the reference builds it "
                   "(its OpenMP pragma is inert: no -fopenmp)"),
        "gridder_mvis_s": round(nvis / (t1 - t0) / 1e6, 4),
        "degridder_mvis_s": round(nvis / (t2 - t1) / 1e6, 4),
    }
    cpus = host_cpus()
    multi = cpu_baseline_threads(w, a, impl, kind, args, nsample, extra,
                                 cpus["usable"])
    out = dict(multi or single)
    out.update({"unit": "Mvis/s", "kind": kind, "host": cpus})
    if multi:
        out["single_thread"] = single
    return out


def cpu_baseline_threads(w, a, impl, kind, args, nsample, extra, cores):
    """The same CPU path on `cores` host threads, each running the
    reference's own kernel on its own contiguous range of `nsample`
    subgrids (ctypes drops the GIL during the call).  The ranges write
    disjoint subgrids / visibility rows.  Only valid when every subgrid has
    the same baseline_offset (the kernels rebase row indices on
    metadata[0].baseline_offset, gridder_reference.cpp:16-25) -- true for
    the synthetic batch; otherwise None."""
    import numpy as np
    from concurrent.futures import ThreadPoolExecutor
    md_all = a["metadata"]
    cores = int(os.environ.get("IDG_CPU_BASELINE_THREADS", cores))
    n = min(nsample * cores, md_all.size)
    if cores < 2 or n < 2 * cores or np.any(
            md_all["baseline_offset"][:n] != md_all["baseline_offset"][0]):
        return None
    T, C, S = w["nr_timesteps"], w["nr_channels"], w["subgrid_size"]
    bounds = np.linspace(0, n, cores + 1).astype(int)
    sg = np.zeros((n, 4, S, S, 2), np.float32)
    # visibilities are [rows / T][T][C][4] complex: the blocks the first n
    # subgrids' rows (time_offset + t) fall in
    rows = int(md_all[n - 1]["time_offset"]) + T
    vis = np.zeros(((rows + T - 1) // T,) + a["visibilities"].shape[1:],
                   np.float32)
    sub_in = np.ascontiguousarray(a["subgrids"][:n])

    def run(fn, i):
        lo, hi = bounds[i], bounds[i + 1]
        md = np.ascontiguousarray(md_all[lo:hi])
        targs = (hi - lo,) + args[1:]
        if fn == "g":
            impl.gridder(*targs, a["uvw"], a["wavenumbers"], a["visibilities"],
                         a["spheroidal"], a["aterms"], md, sg[lo:hi], **extra)
        else:
            impl.degridder(*targs, a["uvw"], a["wavenumbers"], vis,
                           a["spheroidal"], a["aterms"], md, sub_in[lo:hi],
                           **extra)

    with ThreadPoolExecutor(cores) as pool:
        t0 = time.perf_counter()
        list(pool.map(lambda i: run("g", i), range(cores)))
        t1 = time.perf_counter()
        list(pool.map(lambda i: run("d", i), range(cores)))
        t2 = time.perf_counter()
    nvis = n * T * C
    cpu_baseline_threads.last_outputs = {"subgrids": sg, "visibilities": vis}
    return {
        "value": round(nvis / (t2 - t0) / 1e6, 4),
        "cores": cores,
        "sample": (f"first {n} subgrids of the same batch ({nvis} vis) on "
                   f"{cores} host threads ({n // cores} subgrids each), "
                   f"gridder {t1 - t0:.2f} s + degridder {t2 - t1:.2f} s, "
                   + ("oracle/_ref/libidgref_v3.so (reference app/CPU)"
                      if kind == "reference" else "oracle/liboracle.so")),
        "gridder_mvis_s": round(nvis / (t1 - t0) / 1e6, 4),
        "degridder_mvis_s": round(nvis / (t2 - t1) / 1e6, 4),
    }


# ---------------------------------------------------------------------------
# Committed profile data (profiles/traffic.json)
# ---------------------------------------------------------------------------
def profile_entry(path, workload_name, kernel):
    try:
        with open(path) as f:
            return json.load(f)[workload_name][kernel]
    except Exception:
        return None


def transcendental_floor(w, nsub):
    """(wave-instructions, seconds) of the v_sin/v_cos a launch over nsub
    subgrids cannot avoid: one exact f32 phase per (pixel, timestep,
    channel) and its sin and cos (the reference's own arithmetic, §3), one
    pair per mirror pair of pixels where the pairing applies (even S, w = 0:
    every workload but 'wterm'), at the measured 8.35 cycles per wave64
    transcendental on each of the 1,024 SIMDs (profiles/r02/rates/)."""
    S, T, C = w["subgrid_size"], w["nr_timesteps"], w["nr_channels"]
    mirror = S % 2 == 0 and not w.get("w_range")
    pixels = S * S // 2 if mirror else S * S
    insts = 2.0 * nsub * pixels * T * C / 64
    return insts, insts * ISSUE_CYC["trans"] / NR_SIMDS / CLOCK_HZ


def roofline_for(entry, kernel, flops, nvis, t, nsub_launch, nsub_profiled,
                 w=None):
    """Roofline of the dominant kernel.

    The binding hardware resource is the transcendental unit: every
    phasor needs v_sin + v_cos of the reference's exact f32 phase (quarter
    rate, 8.35 cycles per wave64 instruction), and nothing else the path
    must do is as scarce.  So
        t_floor = 2 x phasors / 64 x 8.35 cycles / 1024 SIMDs / 2.4 GHz
    (transcendental_floor), achieved = the reference work model's FLOPs
    (app/common/common.cpp:100-129) / measured time, peak = the same FLOPs
    / t_floor, frac = t_floor / t.  Beside it:
      mfma             the work model against the dense f16 MFMA peak, and
                       the MFMA FLOPs actually executed (two-term split);
      issue_efficiency the kernel's own instruction stream at the measured
                       issue costs over its time (how well it issues what it
                       has; from the committed SQ profile,
                       profiles/traffic.json -> issue_bound);
      fp32_equivalent  the work model against the FP32 peak the reference
                       prices it on (> 1: the MAC runs on the matrix core)."""
    achieved = flops / t / 1e12
    out = {"bound": "mfma", "achieved": round(achieved, 3),
           "unit": "TFLOP/s", "kernel": kernel, "traffic": None}
    scale = nsub_launch / nsub_profiled if nsub_profiled else 1.0
    if entry and entry.get("hbm_bytes_per_launch"):
        out["traffic"] = int(entry["hbm_bytes_per_launch"] * scale)
    if w is not None:
        trans, t_floor = transcendental_floor(w, nsub_launch)
        out.update({
            "resource": "transcendental issue (v_sin + v_cos of the "
                        "reference's exact f32 phase, one pair per phasor)",
            "peak": round(flops / t_floor / 1e12, 3),
            "frac": round(t_floor / t, 4),
            "floor": {"t_floor_ms": round(t_floor * 1e3, 4),
                      "trans_wave_insts": trans,
                      "cycles_per_trans": ISSUE_CYC["trans"],
                      "simds": NR_SIMDS, "clock_ghz": CLOCK_HZ / 1e9},
        })
    out["mfma"] = {
        "work_model_frac": round(achieved / F16_MFMA_PEAK_TFLOPS, 4),
        "peak": F16_MFMA_PEAK_TFLOPS,
        "note": "the reference work model's FLOPs over the measured time "
                "against the dense f16 MFMA peak"}
    ib = (entry or {}).get("issue_bound")
    if ib and ib.get("insts_valu"):
        trans_i = ib["insts_trans"] * scale
        mfma = ib["insts_mfma_f16"] * scale
        other = ib["insts_valu"] * scale - trans_i - mfma
        cls = ib.get("insts_class")
        if cls:
            # per VALU class (round 4, SQ_INSTS_VALU_CVT / _FMA_F32 passes):
            # the f16-output converts and the mix / packed FMAs at their
            # measured VOP3 costs, every other VALU at the plain f32 rate
            other_cyc = (cls["SQ_INSTS_VALU_CVT"] * ISSUE_CYC["cvt"] +
                         cls["SQ_INSTS_VALU_FMA_F32"] * ISSUE_CYC["fma_f32"] +
                         cls["plain"] * ISSUE_CYC["plain"]) * scale
        else:
            other_cyc = other * ISSUE_CYC["other"]
        cyc = (trans_i * ISSUE_CYC["trans"] + mfma * ISSUE_CYC["mfma_f16"] +
               other_cyc) / NR_SIMDS
        t_issue = cyc / CLOCK_HZ
        out["issue_efficiency"] = {
            "frac": round(t_issue / t, 4),
            "t_issue_ms": round(t_issue * 1e3, 4),
            "insts_per_launch": {"trans": trans_i, "mfma_f16": mfma,
                                 "other_valu": other},
            "cycles": ISSUE_CYC, "clock_ghz": CLOCK_HZ / 1e9,
            "source": ib.get("source"),
            "note": "the kernel's own instruction stream (SQ counters) at "
                    "the measured issue costs, over the measured time"}
        mfma_tf = mfma * MFMA_F16_FLOP / t / 1e12
        out["mfma"].update({
            "executed_tflops": round(mfma_tf, 3),
            "executed_frac": round(mfma_tf / F16_MFMA_PEAK_TFLOPS, 4),
            "executed_note": "v_mfma_f32_16x16x32_f16 FLOPs executed (two-"
                             "term split: 4 f16 products per f32 MAC)"})
    if "frac" not in out:
        out.update({"peak": F16_MFMA_PEAK_TFLOPS,
                    "frac": round(achieved / F16_MFMA_PEAK_TFLOPS, 4),
                    "resource": "f16 MFMA dense peak"})
    out["fp32_equivalent"] = {
        "achieved": round(achieved, 3), "peak": FP32_PEAK_TFLOPS,
        "ratio": round(achieved / FP32_PEAK_TFLOPS, 4),
        "note": "the reference work model priced on the FP32 peak; > 1 "
                "because its complex MAC runs on the f16 matrix core"}
    out["note"] = (f"achieved = reference work model {flops / nvis:.0f} "
                   f"FLOP/vis x {nvis} vis per launch / mean kernel duration "
                   "(HIP events on the launch stream); peak = the same FLOPs "
                   "at the transcendental floor; frac = t_floor / t "
                   "(DESIGN.md §4.3)")
    return out


def roofline_seq(entry, kernel, flops, nvis, t, nsub_launch):
    """Roofline of an order-preserving (bit-exact) kernel:
    it repeats the reference's own arithmetic -- glibc's sincosf in f64 per
    phasor, f32 sums in the reference's order -- so its floor is the issue
    time of that instruction stream, not a tensor or transcendental unit:
        t_issue = sum over VALU classes (SQ counters) of count x measured
                  issue cost / 1024 SIMDs / 2.4 GHz
    (tools/probes/summarize_seq.py, the costs from
    tools/probes/seq_rates_probe.hip), frac = t_issue / t, achieved = the
    reference work model's FLOPs / t, peak = the same FLOPs / t_issue."""
    achieved = flops / t / 1e12
    out = {"bound": "valu-issue", "achieved": round(achieved, 3),
           "unit": "TFLOP/s", "kernel": kernel,
           "resource": "VALU issue of the kernel's own instruction stream "
                       "(glibc sincosf restated in f64, sums in the "
                       "reference's order)"}
    im = (entry or {}).get("issue_model")
    if im:
        scale = nsub_launch / entry.get("nr_subgrids", nsub_launch)
        t_issue = im["t_issue_ms"] / 1e3 * scale
        out.update({
            "peak": round(flops / t_issue / 1e12, 3),
            "frac": round(t_issue / t, 4),
            "t_issue_ms": round(t_issue * 1e3, 4),
            "valu_mix_per_launch": {k: int(v * scale) for k, v in
                                    im.get("valu_mix", {}).items()},
            "costs": im.get("costs"), "source": im.get("source"),
            "note": "class counts x measured issue cost / 1024 SIMDs / "
                    "2.4 GHz over the measured time (the SQ profile's "
                    "launch, scaled to this one's subgrids)"})
    else:
        out.update({"peak": None, "frac": None,
                    "note": "no committed SQ profile for this kernel"})
    out["fp32_equivalent"] = {
        "achieved": round(achieved, 3), "peak": FP32_PEAK_TFLOPS,
        "ratio": round(achieved / FP32_PEAK_TFLOPS, 4)}
    return out


def algorithmic_bytes(w, nsub):
    """Bytes a launch must move at least: the visibilities once, the subgrids
    once, the uvw rows once (the A-terms and taper are L2-resident)."""
    T, C, S = w["nr_timesteps"], w["nr_channels"], w["subgrid_size"]
    return nsub * T * C * 32 + nsub * 4 * S * S * 8 + nsub * T * 12


def time_workload(args, name, timeslots, stream, dist, steps, impl=None,
                  batch=None):
    """One of BASELINE.json's other single-GPU configs, timed beside `value`
    (never in it): its own batch from the reference generators (a timeslot
    subset where stated), the same timed step, per-kernel figures and the
    dominant kernel's roofline priced from the committed profile of the
    same launch (profiles/traffic.json[name]).  impl: IDG_GRIDDER_IMPL for
    the leg (e.g. "sequential").  Returns (leg, batch) so a second leg can
    reuse the batch."""
    import torch
    import idg_amd
    w = workload(name, timeslots)
    T, C, S = w["nr_timesteps"], w["nr_channels"], w["subgrid_size"]
    if batch is None:
        progress(f"side leg {name}: generating the batch")
        a = make_batch(w, nthreads=16)
        batch = (a, upload(shard_batch(a, 0, 1)))
    a, dev = batch
    nsub = int(a["metadata"].size)
    nvis = nsub * T * C
    saved = os.environ.get("IDG_GRIDDER_IMPL")
    if impl:
        os.environ["IDG_GRIDDER_IMPL"] = impl
    try:
        names = {d: idg_amd.kernel_name(d, S, C)
                 for d in ("gridder", "degridder")}
        el, tg, td, _, _, _ = time_steps(w, dev, nsub, steps, 1, stream,
                                         dist, min_warmup_s=0.5)
    finally:
        if saved is None:
            os.environ.pop("IDG_GRIDDER_IMPL", None)
        else:
            os.environ["IDG_GRIDDER_IMPL"] = saved
    flops = idg_amd.flops_gridder(C, nsub * T, nsub, S)
    times = {"gridder": tg, "degridder": td}
    dom = "gridder" if tg >= td else "degridder"
    entry = profile_entry(args.traffic_file, name, names[dom])
    if "sequential" in names[dom]:
        rl = roofline_seq(entry, names[dom], flops, nvis, times[dom], nsub)
    else:
        rl = roofline_for(entry, names[dom], flops, nvis, times[dom], nsub,
                          (entry or {}).get("nr_subgrids", nsub), w)
    rl["algorithmic_bytes"] = algorithmic_bytes(w, nsub)
    if rl.get("traffic"):
        rl["traffic_over_algorithmic"] = round(
            rl["traffic"] / rl["algorithmic_bytes"], 3)
    leg = {
        "value": round(nvis / (el / steps) / 1e6, 2), "unit": "Mvis/s",
        "steps": steps, "ms_per_step": round(el / steps * 1e3, 4),
        "kernels": {d: {"kernel": names[d], "ms": round(times[d] * 1e3, 4),
                        "mvis_s": round(nvis / times[d] / 1e6, 2)}
                    for d in names},
        "baseline_config": BASELINE_CONFIG[name],
        "workload": (f"{name}: NR_STATIONS={w['nr_stations']} "
                     f"NR_TIMESLOTS={w['nr_timeslots']} "
                     f"NR_TIMESTEPS_SUBGRID={T} NR_CHANNELS={C} "
                     f"SUBGRID_SIZE={S} GRID_SIZE={w['grid_size']}: "
                     f"{nsub} subgrids, {nvis} visibilities"),
        "roofline": rl,
    }
    if entry and entry.get("source"):
        leg["traffic_source"] = entry["source"]
    return leg, batch


# ---------------------------------------------------------------------------
# Side legs of a one-GPU default run (beside `value`, never in it)
# ---------------------------------------------------------------------------
def time_side_legs(args, w, a, dev, nsub, stream, dist, value):
    """Two figures the default line carries beside `value`:
      wterm       the same batch with the 'wterm' workload's w-terms (w ~
                  U(-200, 200), W_STEP = 2.5, 7 w-layers): every subgrid off
                  the mirror pairing the synthetic w = 0 data allows
                  (app/common/init.cpp:21), so `value` / this = the w = 0
                  mirror factor; roofline priced from its own SQ profile;
      sequential  the batch on the order-preserving kernels
                  (IDG_{GRIDDER,DEGRIDDER}_IMPL=sequential), bit-exact to the
                  reference's CPU output."""
    import numpy as np
    import torch
    import idg_amd
    T, C, S = w["nr_timesteps"], w["nr_channels"], w["subgrid_size"]
    nvis = nsub * T * C
    side = {}
    steps = max(1, min(args.steps, 5))
    # -- wterm: new uvw (w column) and metadata (w-layer), same visibilities
    ww = workload("wterm")
    aw = {"uvw": a["uvw"].copy(), "metadata": a["metadata"].copy()}
    apply_wterms(ww, aw)
    devw = dict(dev)
    devw["uvw"] = torch.from_numpy(aw["uvw"]).cuda()
    devw["metadata"] = torch.from_numpy(
        aw["metadata"].view(np.int32).reshape(-1, 9).copy()).cuda()
    el, tg, td, _, _, _ = time_steps(ww, devw, nsub, steps, 1, stream, dist,
                                     min_warmup_s=0.5)
    flops = idg_amd.flops_gridder(C, nsub * T, nsub, S)
    names = {d: idg_amd.kernel_name(d, S, C) for d in ("gridder", "degridder")}
    dom = "gridder" if tg >= td else "degridder"
    t_dom = max(tg, td)
    entry = profile_entry(args.traffic_file, "wterm", names[dom])
    rl = roofline_for(entry, names[dom], flops, nvis, t_dom, nsub,
                      nsub if entry else 0, ww)
    if entry and entry.get("algorithmic_bytes"):
        rl["algorithmic_bytes"] = int(entry["algorithmic_bytes"])
    wv = nvis / (el / steps) / 1e6
    side["wterm"] = {
        "value": round(wv, 2), "unit": "Mvis/s", "steps": steps,
        "ms_per_step": round(el / steps * 1e3, 4),
        "gridder_ms": round(tg * 1e3, 4), "degridder_ms": round(td * 1e3, 4),
        "kernels": names, "roofline": rl,
        "mirror_factor": round(value / wv, 3),
        "workload": (f"the default batch with W_STEP={ww['w_step']}, "
                     f"w~U(-{ww['w_range']:g},{ww['w_range']:g}), "
                     f"w-layers={ww['w_layers']} (bench.py apply_wterms)"),
        "note": "beside `value`, not in it: every subgrid on the general "
                "(non-mirror) path; mirror_factor = value / this"}
    del devw
    # -- sequential kernels on the default batch
    saved = {k: os.environ.get(k) for k in ("IDG_GRIDDER_IMPL",
                                            "IDG_DEGRIDDER_IMPL")}
    os.environ["IDG_GRIDDER_IMPL"] = "sequential"
    os.environ["IDG_DEGRIDDER_IMPL"] = "sequential"
    try:
        names_q = {d: idg_amd.kernel_name(d, S, C)
                   for d in ("gridder", "degridder")}
        qsteps = max(1, min(args.steps, 2))
        el, tg, td, _, _, _ = time_steps(w, dev, nsub, qsteps, 1, stream,
                                         dist, min_warmup_s=0.0)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    qv = nvis / (el / qsteps) / 1e6
    flops = idg_amd.flops_gridder(C, nsub * T, nsub, S)
    qdom = "gridder" if tg >= td else "degridder"
    side["sequential"] = {
        "value": round(qv, 2), "unit": "Mvis/s", "steps": qsteps,
        "ms_per_step": round(el / qsteps * 1e3, 4),
        "gridder_ms": round(tg * 1e3, 4), "degridder_ms": round(td * 1e3, 4),
        "gridder_mvis_s": round(nvis / tg / 1e6, 2),
        "degridder_mvis_s": round(nvis / td / 1e6, 2),
        "kernels": names_q, "slowdown_vs_value": round(value / qv, 2),
        "roofline": roofline_seq(
            profile_entry(args.traffic_file, "default", names_q[qdom]),
            names_q[qdom], flops, nvis, max(tg, td), nsub),
        "roofline_other": roofline_seq(
            profile_entry(args.traffic_file, "default",
                          names_q["degridder" if qdom == "gridder"
                                  else "gridder"]),
            names_q["degridder" if qdom == "gridder" else "gridder"], flops,
            nvis, min(tg, td), nsub),
        "note": "IDG_{GRIDDER,DEGRIDDER}_IMPL=sequential: the reference CPU "
                "path's rounding sequence (glibc sincosf restated, t-then-c "
                "f32 sums per pixel; y-then-x per visibility), bit-exact to "
                "app/CPU (tests/test_gpu_sequential.py); beside `value`"}
    if args.no_workload_legs:
        return side
    # -- BASELINE configs[2] and configs[4] on the default (MFMA) kernels, and
    #    configs[2] with the order-preserving gridder -- the mode that keeps
    #    the reference's own rounding at T x C = 32,768 --
    #    beside the default degridder, which meets the reference metric there
    wsteps = max(1, min(args.steps, 3))
    side["configs2"], batch = time_workload(args, "c256", 4, stream, dist,
                                            wsteps)
    side["configs2"]["note"] = ("BASELINE configs[2] (C = 256) at "
                                "NR_TIMESLOTS=4 (a fifth of the batch); "
                                "beside `value`, not in it")
    seq2, _ = time_workload(args, "c256", 4, stream, dist, 1,
                            impl="sequential", batch=batch)
    seq2["note"] = ("configs[2] at NR_TIMESLOTS=4 with the order-preserving "
                    "gridder (bit-exact to app/CPU) and the default "
                    "degridder (within the reference metric of app/CPU at "
                    "every config): the configuration that prints PASSED "
                    "under the reference's own harness at T x C = 32,768")
    side["sequential"]["configs2"] = seq2
    del batch, _
    torch.cuda.empty_cache()
    side["configs4"], batch = time_workload(args, "s64", None, stream, dist,
                                            wsteps)
    side["configs4"]["note"] = ("BASELINE configs[4] (S = 64, A-term + "
                                "spheroidal), the full batch; beside "
                                "`value`, not in it")
    del batch
    torch.cuda.empty_cache()
    return side


# ---------------------------------------------------------------------------
# Timed run
# ---------------------------------------------------------------------------
def dtype_label(kernels):
    """The arithmetic of the kernels this run selected (idg_amd.kernel_name:
    a `_valu` suffix is the all-VALU body, IDG_{GRIDDER,DEGRIDDER}_IMPL=valu,
    whose MAC is plain f32 FMA; the others run the complex MAC on the f16
    matrix core with two-term-split operands)."""
    valu = {d: k["kernel"].endswith("_valu") for d, k in kernels.items()}
    mfma = "f32 phase/accumulate, f16x2-split MFMA operands"
    if all(valu.values()):
        return "f32"
    if not any(valu.values()):
        return mfma
    return "; ".join(f"{d}: {'f32' if v else mfma}" for d, v in valu.items())


def upload(part):
    import numpy as np
    import torch
    dev = {k: torch.from_numpy(part[k]).cuda() for k in
           ("uvw", "wavenumbers", "visibilities", "spheroidal", "aterms",
            "subgrids")}
    dev["metadata"] = torch.from_numpy(
        part["metadata"].view(np.int32).reshape(-1, 9).copy()).cuda()
    return dev


def extra_warmup_steps(step_s, min_warmup_s):
    """Untimed steps (the pricing step included) that fill min_warmup_s at
    step_s seconds per step: at least one, and at most 10,001 (steps priced
    below 0.1 ms count as 0.1 ms)."""
    if min_warmup_s <= 0:
        return 0
    return 1 + int(min_warmup_s / max(step_s, 1e-4))


def time_steps(w, dev, nsub, steps, warmup, stream, dist, meter=None,
               min_warmup_s=0.0, info=None):
    """warmup untimed steps (more, up to min_warmup_s of GPU work, see
    below), then `steps` timed ones bracketed by barrier + synchronize.
    Returns (elapsed max over ranks, t_grid, t_degrid (mean per launch, max
    over ranks), joules, outputs); info["warmup_steps_run"] gets the
    untimed step count."""
    import torch
    import idg_amd
    S, C, G = w["subgrid_size"], w["nr_channels"], w["grid_size"]
    p = (nsub, G, S, idg_amd.IMAGE_SIZE, w.get("w_step", idg_amd.W_STEP), C,
         w["nr_stations"])
    grid_out = torch.empty_like(dev["subgrids"])
    degrid_out = torch.empty_like(dev["visibilities"])

    # ev = (start, middle, end) of a timed step; consecutive steps share
    # their boundary event (step k's end is step k+1's start), so a step
    # records two events, not three (each event record costs the stream
    # ~3.5 us: 3,062 subgrids at N = 8, 1.9527 / 1.9577 / 1.9641 ms per step
    # with 0 / 2 / 3 events, tools/debug/event_cost.py, profiles/r06/n8/)
    def step(ev=None):
        if nsub == 0:
            return
        if ev and ev[0] is not None:
            ev[0].record(stream)
        idg_amd.gridder_launch(*p, dev["uvw"], dev["wavenumbers"],
                               dev["visibilities"], dev["spheroidal"],
                               dev["aterms"], dev["metadata"], grid_out,
                               stream=stream)
        if ev:
            ev[1].record(stream)
        idg_amd.degridder_launch(*p, dev["uvw"], dev["wavenumbers"],
                                 degrid_out, dev["spheroidal"], dev["aterms"],
                                 dev["metadata"], dev["subgrids"],
                                 stream=stream)
        if ev:
            ev[2].record(stream)

    marks = [torch.cuda.Event(enable_timing=True)
             for _ in range(2 * steps + 1)]
    events = [(marks[2 * k] if k == 0 else None, marks[2 * k + 1],
               marks[2 * k + 2]) for k in range(steps)]
    bounds = [(marks[2 * k], marks[2 * k + 1], marks[2 * k + 2])
              for k in range(steps)]
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    # Clock ramp: the device leaves its idle clock state only
    # after sustained work, and drops back after an idle gap of 20 ms.  A
    # short shard (3,062 subgrids at N = 8: 2 ms per step) timed after W = 2
    # warm-up steps ran 10% slower than the same launches after a long
    # warm-up.  So the untimed warm-up continues for about min_warmup_s of
    # back-to-back steps (priced by one more step, after the first launches'
    # one-off costs), the same count on every rank (max over ranks, so that
    # none idles at the barrier), straight into the timed region.
    extra = 0
    if nsub and min_warmup_s > 0:
        t_w = time.perf_counter()
        step()
        torch.cuda.synchronize()
        extra = extra_warmup_steps(time.perf_counter() - t_w, min_warmup_s)
    extra = int(dist.max_over_ranks(extra))
    for _ in range(extra - (1 if nsub and min_warmup_s > 0 else 0)):
        step()
    if info is not None:
        info["warmup_steps_run"] = warmup + extra
    dist.barrier()
    torch.cuda.synchronize()
    if meter:
        meter.start()
    t0 = time.perf_counter()
    for k in range(steps):
        step(events[k])
    torch.cuda.synchronize()
    dist.barrier()
    elapsed = time.perf_counter() - t0
    # the energy counter is read after the clock stops: an amdsmi call is not
    # part of the timed steps (its cost would weigh on a 2 ms N = 8 step)
    joules = meter.stop() if meter else None
    elapsed_max = dist.max_over_ranks(elapsed)
    if nsub:
        t_grid = sum(e[0].elapsed_time(e[1]) for e in bounds) / steps / 1e3
        t_degrid = sum(e[1].elapsed_time(e[2]) for e in bounds) / steps / 1e3
    else:
        t_grid = t_degrid = 0.0
    return (elapsed_max, dist.max_over_ranks(t_grid),
            dist.max_over_ranks(t_degrid), joules, elapsed,
            (grid_out, degrid_out))


def time_pipeline(w, dev, sub_out, stream, steps, world, dist):
    """Gridder output -> FFT -> adder -> grid-sum over ranks and splitter ->
    FFT: the IDG steps either side of the path (not in `value`).  Returns
    (timings dict, the summed grid of the last pass)."""
    import torch
    import idg_amd
    G, S = w["grid_size"], w["subgrid_size"]
    nw = w.get("w_layers", 1)
    gridt = torch.zeros((nw, 4, G, G, 2), dtype=torch.float32, device="cuda")
    uvsub = torch.empty_like(sub_out)
    uvfused = torch.empty_like(sub_out)
    npipe = max(1, min(steps, 5))
    pev = [[torch.cuda.Event(enable_timing=True) for _ in range(7)]
           for _ in range(npipe)]
    has = sub_out.shape[0] > 0
    for it in range(npipe + 1):
        e = pev[it - 1] if it > 0 else None
        uvsub.copy_(sub_out)
        gridt.zero_()
        dist.barrier()
        if e:
            e[0].record(stream)
        if has:
            idg_amd.subgrid_fft_launch(uvsub, +1, 1.0, stream=stream)
        if e:
            e[1].record(stream)
        if has:
            idg_amd.adder_launch(G, dev["metadata"], uvsub, gridt,
                                 nr_w_layers=nw, stream=stream)
        if e:
            e[2].record(stream)
        dist.reduce_grid(gridt)
        if e:
            e[3].record(stream)
        if has:
            idg_amd.splitter_launch(G, dev["metadata"], gridt, uvsub,
                                    nr_w_layers=nw, stream=stream)
        if e:
            e[4].record(stream)
        if has:
            idg_amd.subgrid_fft_launch(uvsub, -1, 1.0 / (S * S),
                                       stream=stream)
        if e:
            e[5].record(stream)
        # the same two steps as one fused kernel (S = 32 / 64), into a
        # buffer of its own
        if has:
            idg_amd.splitter_fft_launch(G, dev["metadata"], gridt, uvfused,
                                        nr_w_layers=nw, stream=stream)
        if e:
            e[6].record(stream)
    torch.cuda.synchronize()
    # the gridder with the FFT in its epilogue (S = 32; other S: the two
    # launches) against the gridder followed by the FFT pass, the two
    # interleaved rep by rep after one untimed rep of each (the same clock
    # state for both), each into a buffer of its own
    gev = [[torch.cuda.Event(enable_timing=True) for _ in range(4)]
           for _ in range(npipe)]
    if has:
        nsub = sub_out.shape[0]
        p = (nsub, G, S, idg_amd.IMAGE_SIZE, w.get("w_step", idg_amd.W_STEP),
             w["nr_channels"], w["nr_stations"])
        ins = (dev["uvw"], dev["wavenumbers"], dev["visibilities"],
               dev["spheroidal"], dev["aterms"], dev["metadata"])
        for it in range(npipe + 1):
            e = gev[it - 1] if it > 0 else None
            if e:
                e[0].record(stream)
            idg_amd.gridder_launch(*p, *ins, uvsub, stream=stream)
            idg_amd.subgrid_fft_launch(uvsub, +1, 1.0, stream=stream)
            if e:
                e[1].record(stream)
                e[2].record(stream)
            idg_amd.gridder_fft_launch(*p, *ins, uvfused, stream=stream)
            if e:
                e[3].record(stream)
        torch.cuda.synchronize()
    gridder_then_fft_ms, gridder_fft_ms = (
        dist.max_over_ranks(sum(e[i].elapsed_time(e[i + 1]) for e in gev)
                            / npipe if has else 0.0) for i in (0, 2))
    # the whole cycle on the fused entries, timed as one: gridder with the
    # FFT in its epilogue -> adder -> grid-sum over ranks -> splitter +
    # inverse FFT -> degridder (idg_amd.grid_onto / degrid_from's launches)
    cev = [[torch.cuda.Event(enable_timing=True) for _ in range(2)]
           for _ in range(npipe)]
    vis_out = torch.empty_like(dev["visibilities"]) if has else None
    for it in range(npipe + 1):
        e = cev[it - 1] if it > 0 else None
        gridt.zero_()
        dist.barrier()
        if e:
            e[0].record(stream)
        if has:
            idg_amd.gridder_fft_launch(*p, *ins, uvfused, stream=stream)
            idg_amd.adder_launch(G, dev["metadata"], uvfused, gridt,
                                 nr_w_layers=nw, stream=stream)
        dist.reduce_grid(gridt)
        if has:
            idg_amd.splitter_fft_launch(G, dev["metadata"], gridt, uvsub,
                                        nr_w_layers=nw, stream=stream)
            idg_amd.degridder_launch(*p, dev["uvw"], dev["wavenumbers"],
                                     vis_out, dev["spheroidal"],
                                     dev["aterms"], dev["metadata"], uvsub,
                                     stream=stream)
        if e:
            e[1].record(stream)
    torch.cuda.synchronize()
    del vis_out
    fused_cycle_ms = dist.max_over_ranks(
        sum(e[0].elapsed_time(e[1]) for e in cev) / npipe)

    def avg(i, j):
        return dist.max_over_ranks(
            sum(e[i].elapsed_time(e[j]) for e in pev) / npipe)
    out = {
        "fft_ms": round(avg(0, 1), 4),
        "adder_ms": round(avg(1, 2), 4),
        "grid_reduce_ms": round(avg(2, 3), 4),
        "splitter_ms": round(avg(3, 4), 4),
        "ifft_ms": round(avg(4, 5), 4),
        "splitter_fft_ms": round(avg(5, 6), 4),
        "splitter_fft": ("splitter + inverse FFT fused "
                         "(idg_splitter_fft_launch), bit for bit "
                         "splitter_ms + ifft_ms's output"),
        "gridder_fft_ms": round(gridder_fft_ms, 4),
        "fused_cycle_ms": round(fused_cycle_ms, 4),
        "gridder_then_fft_ms": round(gridder_then_fft_ms, 4),
        "gridder_fft": ("gridder with the FFT in its epilogue "
                        "(idg_gridder_fft_launch) against the gridder "
                        "followed by the FFT pass (bit for bit the same "
                        "output), timed interleaved"),
        "grid": (f"[{nw}][4][{G}][{G}] complex64, "
                 f"{nw * G * G * 32 / 2**20:.0f} MiB"),
        "grid_reduce": (f"all_reduce(sum) of the ranks' partial grids, "
                        f"{dist.backend_name()}"
                        if world > 1 else "single rank: no collective"),
    }
    # HBM roofline of each step: algorithmic bytes (subgrids read/written
    # once, the grid once per pass) over the busiest rank's time
    sub_b = sub_out.numel() * 4
    grid_b = gridt.numel() * 4
    algo = {"fft_ms": 2 * sub_b, "adder_ms": sub_b + 2 * grid_b,
            "splitter_ms": sub_b + grid_b, "ifft_ms": 2 * sub_b,
            "splitter_fft_ms": sub_b + grid_b}
    roof = {}
    for k, nbytes in algo.items():
        t = out[k] / 1e3
        if t > 0:
            gbs = nbytes / t / 1e9
            roof[k[:-3]] = {"algorithmic_bytes": nbytes,
                            "achieved_gbs": round(gbs, 1),
                            "frac": round(gbs / HBM_PEAK_GBS, 4)}
    out["roofline_hbm"] = roof
    return out, gridt


def plan_line(args, w, a, world, dist):
    """The --plan-only line: the rendezvous and shard plan of a run, no
    device work (value null)."""
    counts = shard_counts(a, world, args.mode)
    T, C = w["nr_timesteps"], w["nr_channels"]
    ranks = dist.sum_over_ranks(1.0)  # a collective over every rank
    return {
        "metric": METRIC, "value": None, "unit": "Mvis/s", "n_gpus": world,
        "plan_only": True, "ranks_in_collective": int(ranks),
        "scaling": "weak" if args.mode == "replicated" else "strong",
        "config": {"workload": args.workload,
                   "nr_subgrids": int(a["metadata"].size),
                   "nr_subgrids_per_gpu": counts,
                   "visibilities_per_step": int(
                       a["metadata"].size * T * C *
                       (world if args.mode == "replicated" else 1)),
                   "backend": dist.backend_name()},
    }


def main(argv=None):
    t_run0 = time.perf_counter()
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # a plain `python bench.py --gpus N`: become the launcher
        raise SystemExit(launch_ranks(args, argv))
    import numpy as np
    import torch
    import idg_amd
    from idg_amd import dist

    if args.plan_only:
        rank, _, world = dist.init(
            backend=os.environ.get("IDG_DIST_BACKEND", "gloo"))
        w = workload(args.workload, args.timeslots)
        a = make_batch(w, nthreads=max(1, min(8, (os.cpu_count() or 8)
                                              // max(1, world))))
        line = plan_line(args, w, a, world, dist)
        if args.gpus != world:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but the world "
                             f"size is {world}")
        if rank == 0:
            print(json.dumps(line), flush=True)
        dist.finalize()
        return line

    rank, local_rank, world = dist.init()
    if args.gpus != world:
        raise SystemExit(
            f"bench.py: --gpus {args.gpus} but the world size is {world}")
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a HIP device (no CPU fallback)")
    torch.cuda.set_device(local_rank)
    w = workload(args.workload, args.timeslots)
    T, C, S = w["nr_timesteps"], w["nr_channels"], w["subgrid_size"]

    # ---- synthetic batch (reference generators), this rank's part in HBM --
    threads = max(1, min(16, (os.cpu_count() or 8) // max(1, world)))
    progress(f"generating the {args.workload} batch")
    a = make_batch(w, nthreads=threads)
    ns_total = a["metadata"].size
    idg_amd.validate_metadata(ns_total, S, C, w["nr_stations"], ns_total * T,
                              w["nr_timeslots"], a["metadata"])
    part = shard_batch(a, rank, world, args.mode)
    nsub = part["s1"] - part["s0"]
    idg_amd.validate_metadata(nsub, S, C, w["nr_stations"],
                              part["row1"] - part["row0"],
                              w["nr_timeslots"], part["metadata"])
    progress(f"uploading {nsub} subgrids")
    dev = upload(part)
    stream = torch.cuda.current_stream()
    progress("timing")

    from idg_amd.energy import EnergyMeter
    meter = EnergyMeter(local_rank)
    warm = {}
    elapsed_max, t_grid, t_degrid, joules, elapsed, outs = time_steps(
        w, dev, nsub, args.steps, args.warmup, stream, dist, meter,
        min_warmup_s=args.min_warmup_s, info=warm)
    sec_per_step = elapsed_max / args.steps
    # visibilities processed per step by all ranks together
    nvis_job = (ns_total * T * C * (world if args.mode == "replicated" else 1))
    nvis_rank = nsub * T * C
    nvis_max = dist.max_over_ranks(nvis_rank)  # the busiest rank's share
    nsub_max = int(nvis_max // (T * C))

    flops = idg_amd.flops_gridder(C, nsub_max * T, nsub_max, S)
    nbytes = idg_amd.bytes_gridder(C, nsub_max * T, nsub_max, S)
    kernels = {}
    for name, t in (("gridder", t_grid), ("degridder", t_degrid)):
        kname = idg_amd.kernel_name(name, S, C)
        pbits, pdesc = idg_amd.precision_options(name, S, C)
        kernels[name] = {
            "kernel": kname,
            "precision": {"bits": pbits, "options": pdesc},
            "ms": round(t * 1e3, 4),
            "mvis_s_per_gpu": round(nvis_max / t / 1e6, 2),
            "tflops": round(flops / t / 1e12, 3),
            "hbm_gbs_model": round(nbytes / t / 1e9, 2),
        }
    dom = "gridder" if t_grid >= t_degrid else "degridder"
    t_dom = t_grid if dom == "gridder" else t_degrid
    entry = profile_entry(args.traffic_file, args.workload,
                          kernels[dom]["kernel"])
    roofline = roofline_for(entry, kernels[dom]["kernel"], flops, nvis_max,
                            t_dom, nsub_max, ns_total if entry else 0, w)
    if entry and entry.get("algorithmic_bytes"):
        roofline["algorithmic_bytes"] = int(
            entry["algorithmic_bytes"] * nsub_max / ns_total)
    roofline_hbm = {
        "bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK_GBS,
        "achieved": round(nbytes / t_dom / 1e9, 2),
        "frac": round(nbytes / t_dom / 1e9 / HBM_PEAK_GBS, 4),
        "note": ("reference byte model (common.cpp:131-159, "
                 f"{nbytes / max(1, nvis_max):.2f} B/vis) over the measured "
                 f"time; AI = {flops / max(1, nbytes):.0f} FLOP/B, so the "
                 "path is compute-bound: at this kernel time the HBM "
                 f"fraction is {nbytes / t_dom / 1e9 / HBM_PEAK_GBS:.3f}"),
    }
    if roofline.get("traffic"):
        roofline_hbm["counter_gbs"] = round(roofline["traffic"] / t_dom / 1e9,
                                            2)

    # ---- pipeline steps around the path (not in `value`) ----------------
    pipeline, grid_sum = None, None
    if not args.no_pipeline or args.dump:
        progress("pipeline steps")
        pipeline, grid_sum = time_pipeline(w, dev, outs[0], stream,
                                           args.steps, world, dist)
        extra = sum(pipeline[k] for k in ("fft_ms", "adder_ms",
                                          "grid_reduce_ms", "splitter_ms",
                                          "ifft_ms")) / 1e3
        pipeline["full_cycle_mvis_s"] = round(
            nvis_job / (sec_per_step + extra) / 1e6, 2)
        # the same cycle on the fused entries, timed end to end
        pipeline["full_cycle_fused_mvis_s"] = round(
            nvis_job / (pipeline["fused_cycle_ms"] / 1e3) / 1e6, 2)
        pipeline["note"] = ("gridder -> FFT -> adder -> grid-sum over ranks "
                            "and splitter -> FFT around the timed step; "
                            "reported beside `value`, not in it; "
                            "full_cycle_mvis_s: the timed step plus the "
                            "separately timed steps around it; "
                            "full_cycle_fused_mvis_s: the cycle on the fused "
                            "entries (gridder with the FFT in its epilogue, "
                            "adder, grid-sum, splitter + inverse FFT, "
                            "degridder) timed as one (fused_cycle_ms)")

    if args.dump:
        dump_outputs(args.dump, a, part, outs, grid_sum, rank, world,
                     args.mode, dist)

    # ---- energy over the timed region (amdsmi accumulated-energy counter;
    # the reference's PowerSensor report, app/HIP/util.cpp:134-159) --------
    energy = None
    if joules is not None and joules > 0:
        j_all = dist.sum_over_ranks(joules)
        energy = {
            "joules_per_step": round(j_all / args.steps, 4),
            "avg_power_w_per_gpu": round(j_all / world / elapsed, 1),
            "mvis_per_joule": round(nvis_job * args.steps / j_all / 1e6, 3),
            "source": "amdsmi_get_energy_count over the timed steps",
        }

    # ---- the other scaling mode, beside the headline ----------------------
    weak = None
    if world > 1 and args.mode == "sharded" and not args.no_weak:
        del dev, outs
        torch.cuda.empty_cache()
        full = upload(shard_batch(a, rank, world, "replicated"))
        wsteps = max(1, min(args.steps, 5))
        w_el, w_tg, w_td, _, _, _ = time_steps(
            w, full, ns_total, wsteps, 1, stream, dist,
            min_warmup_s=args.min_warmup_s)
        weak = {
            "value": round(world * ns_total * T * C * wsteps / w_el / 1e6, 2),
            "ms_per_step": round(w_el / wsteps * 1e3, 4),
            "nr_subgrids_per_gpu": ns_total,
            "gridder_ms": round(w_tg * 1e3, 4),
            "degridder_ms": round(w_td * 1e3, 4),
            "steps": wsteps,
            "note": "every rank processes the whole batch (replicated); "
                    "value = all ranks' visibilities / max over ranks",
        }

    # ---- the wterm batch and the sequential kernels, beside `value` -------
    side = None
    if (world == 1 and args.workload == "default" and not args.no_side and
            not args.dump):
        progress("side legs (wterm batch, sequential kernels, configs[2] "
                 "and configs[4])")
        side = time_side_legs(args, w, a, dev, nsub, stream, dist,
                              nvis_job / sec_per_step / 1e6)

    sharded = args.mode == "sharded" and world > 1
    result = {
        "metric": METRIC,
        "value": round(nvis_job / sec_per_step / 1e6, 2),
        "unit": "Mvis/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "warmup_steps_run": warm.get("warmup_steps_run", args.warmup),
        "ms_per_step": round(sec_per_step * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak" if args.mode == "replicated" else "strong",
        "vs_baseline": None,
        "dtype": dtype_label(kernels),
        "data": "synthetic (reference generators app/common/init.cpp, srand(0))",
        "config": {
            "workload": (f"{args.workload}: NR_STATIONS={w['nr_stations']} "
                         f"NR_TIMESLOTS={w['nr_timeslots']} "
                         f"NR_TIMESTEPS_SUBGRID={T} NR_CHANNELS={C} "
                         f"SUBGRID_SIZE={S} GRID_SIZE={w['grid_size']}"
                         + (f" W_STEP={w['w_step']} w~U(-{w['w_range']:g},"
                            f"{w['w_range']:g}) w-layers={w['w_layers']}"
                            if w.get("w_range") else "")),
            "baseline_config": (("configs[3] (configs[1] sharded)"
                                 if sharded else
                                 BASELINE_CONFIG[args.workload])
                                if args.workload == "default"
                                else BASELINE_CONFIG[args.workload]),
            "nr_subgrids": ns_total,
            "nr_subgrids_per_gpu": shard_counts(a, world, args.mode),
            "visibilities_per_step": nvis_job,
            "step": "gridder + degridder over the batch",
            "parallelism": (f"subgrid-sharded x{world} (contiguous equal-cost "
                            "ranges, idg_amd.shard), no data-path collective"
                            if args.mode == "sharded" else
                            f"replicated x{world} (each rank the whole "
                            "batch), no data-path collective"),
        },
        "gridder_mvis_s": round(nvis_job / t_grid / 1e6, 2),
        "degridder_mvis_s": round(nvis_job / t_degrid / 1e6, 2),
        "kernels": kernels,
        "roofline": roofline,
        "roofline_hbm": roofline_hbm,
        "weak_scaling": weak,
        "pipeline": pipeline,
        "energy": energy,
        "reference_hip_mi355x": (reference_hip_for(
            args.workload, sec_per_step, t_grid, t_degrid)
            if world == 1 else None),
        "wterm": side["wterm"] if side else None,
        "sequential": side["sequential"] if side else None,
        "configs2": side.get("configs2") if side else None,
        "configs4": side.get("configs4") if side else None,
        "cpu_baseline": None,
    }
    t_cpu = 0.0
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        progress("cpu baseline")
        t_c0 = time.perf_counter()
        result["cpu_baseline"] = cpu_baseline(w, a, args.cpu_sample_subgrids)
        t_cpu = time.perf_counter() - t_c0
    t_run = time.perf_counter() - t_run0
    result["run_time_share"] = {
        "run_s": round(t_run, 2),
        "timed_region_s": round(elapsed, 4),
        "cpu_baseline_s": round(t_cpu, 2),
        "timed_frac": round(elapsed / t_run, 4),
        "cpu_baseline_frac": round(t_cpu / t_run, 4),
        "note": "wall time of this process (from argument parsing): the timed "
                "steps behind `value` are timed_region_s of it; the rest is "
                "batch generation, upload, warm-up, side legs and the CPU "
                "baseline"}
    if rank == 0:
        print(json.dumps(result), flush=True)
    dist.finalize()
    return result


def dump_outputs(path, a, part, outs, grid_sum, rank, world, mode, dist):
    """Gather the ranks' gridder subgrids and degridded visibility rows in
    rank order (they are disjoint) and write them with the summed uv grid
    from rank 0 (tests/test_gpu_dist.py compares N ranks with one)."""
    import numpy as np
    counts = shard_counts(a, world, mode)
    T = a["uvw"].shape[1]
    cpu = not dist.collectives_on_device()
    sub = outs[0].cpu() if cpu else outs[0]
    vis = outs[1].reshape(-1, T, *outs[1].shape[1:])
    vis = vis.cpu() if cpu else vis
    if mode == "replicated":
        counts = [counts[0]] + [0] * (world - 1)
        if rank:
            sub, vis = sub[:0], vis[:0]
    all_sub = dist.gather_shards(sub, counts)
    all_vis = dist.gather_shards(vis, counts)
    if rank == 0:
        os.makedirs(path, exist_ok=True)
        np.save(os.path.join(path, "subgrids.npy"), all_sub.cpu().numpy())
        np.save(os.path.join(path, "visibilities.npy"),
                all_vis.cpu().numpy())
        if grid_sum is not None:
            np.save(os.path.join(path, "grid.npy"), grid_sum.cpu().numpy())
        with open(os.path.join(path, "meta.json"), "w") as f:
            json.dump({"world": world, "mode": mode, "counts": counts}, f)


def reference_hip_for(workload_name, sec_per_step, t_grid, t_degrid):
    """The reference's own HIP kernels measured on MI355X at configs[1]
    (profiles/reference_hip.json, made by tools/debug/ref_hip.sh): this
    run's per-GPU rates over theirs, for the fastest reference kernels and
    for the fastest that pass the reference's own -c check."""
    if workload_name != "default":
        return None
    try:
        with open(os.path.join(REPO, "profiles", "reference_hip.json")) as f:
            ref = json.load(f)
    except Exception:
        return None
    out = {"source": "profiles/reference_hip.json "
                     "(profiles/r06/reference_hip/SUMMARY.txt)"}
    for tag in ("fastest", "fastest_passing"):
        r = ref[tag]
        step = (r["gridder_ms"] + r["degridder_ms"]) / 1e3
        out[tag] = {
            "kernels": f"{r['gridder']} ({r['gridder_c']} -c) + "
                       f"{r['degridder']} ({r['degridder_c']} -c)",
            "mvis_s_per_gpu": round(ref["mvis_per_step"] / step, 2),
            "speedup_step": round(step / sec_per_step, 2),
            "speedup_gridder": round(r["gridder_ms"] / 1e3 / t_grid, 2),
            "speedup_degridder": round(r["degridder_ms"] / 1e3 / t_degrid, 2),
        }
    return out


if __name__ == "__main__":
    main()
