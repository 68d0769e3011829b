#!/usr/bin/env python3
"""bench.py -- IDG gridder + degridder throughput on MI355X (BASELINE.json metric).

One step = one gridder pass + one degridder pass over one batch of the
workload, both kernels on the same HIP stream, inputs resident in HBM.  At
N=1 the batch is BASELINE.json configs[1], the reference's perf defaults
(app/HIP/util.cpp:181-187): NR_STATIONS=50, NR_TIMESLOTS=20,
NR_TIMESTEPS_SUBGRID=128, NR_CHANNELS=16, SUBGRID_SIZE=32, GRID_SIZE=1024
-> 24,500 subgrids, 50.176 M visibilities, with the reference's own synthetic
generators (srand(0)).  With N GPUs (one process per GPU, torchrun) every
rank processes its own batch of that size -- weak scaling, subgrid-sharded,
no collective on the data path; value = all ranks' visibilities / the max
over ranks of the timed region.

`value` counts a visibility once per step (it is gridded AND degridded);
per-kernel Mvis/s are reported alongside.  The roofline object is for the
dominant (slower) kernel: achieved = the reference work model's FLOPs per
launch (app/common/common.cpp:100-129; 35,459 FLOP/vis at this config) /
that kernel's mean duration from HIP events on its stream; peak = MI355X FP32
(157.3 TFLOP/s -- vector and f32-MFMA peaks are equal on gfx950).  The path is
compute-bound; its HBM roofline fraction is reported too.  cpu_baseline times
the reference's own CPU path (oracle/_ref) on a bounded sample of the same
batch: on 16 host threads (`value`, disjoint subgrid ranges) and on 1 thread
as the reference builds it (`single_thread`).

    python bench.py [--gpus N --steps K --warmup W] [--workload default]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "ska-sdp-idg-bench_amd"))

METRIC = "Mvisibilities/s (gridder & degridder) at 1/2/4/8 GPUs; % HBM roofline"
FP32_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 vector = FP32 matrix
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec

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


def apply_wterms(w, a):
    """w-terms of the 'wterm' workload, in place (seeded, numpy)."""
    import numpy as np
    if not w.get("w_range"):
        return
    rng = np.random.default_rng(7)
    a["uvw"][..., 2] = rng.uniform(-w["w_range"], w["w_range"],
                                   a["uvw"].shape[:2])
    a["metadata"]["z"] = rng.integers(0, w["w_layers"], a["metadata"].size)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="default", choices=sorted(WORKLOADS))
    ap.add_argument("--timeslots", type=int, default=None,
                    help="override NR_TIMESLOTS (batch size)")
    ap.add_argument("--cpu-sample-subgrids", type=int, default=128)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="skip timing the FFT / adder / grid-sum / splitter")
    ap.add_argument("--traffic-file", default=os.path.join(
        REPO, "profiles", "traffic.json"))
    return ap.parse_args()


def cpu_baseline(w, a, nsample):
    """Time the reference CPU path (oracle/_ref, else the oracle port) on the
    first `nsample` subgrids of the batch.  Test infrastructure only: the
    baseline the GPU number is reported beside, never the measured path."""
    import numpy as np
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as orc
    n = min(nsample, a["metadata"].size)
    md = a["metadata"][:n]
    T, C, S = w["nr_timesteps"], w["nr_channels"], w["subgrid_size"]
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
    multi = cpu_baseline_threads(w, a, impl, kind, args, nsample, extra)
    out = dict(multi or single)
    out.update({"unit": "Mvis/s", "kind": kind})
    if multi:
        out["single_thread"] = single
    return out


def cpu_baseline_threads(w, a, impl, kind, args, nsample, extra):
    """The same CPU path on `cores` host threads (the GPU box's CPU share),
    each thread running the reference's own kernel on its own contiguous
    range of `nsample` subgrids (ctypes drops the GIL during the call).  The
    ranges write disjoint subgrids / visibility rows.  Only valid when every
    subgrid has the same baseline_offset (the kernels rebase row indices on
    metadata[0].baseline_offset, gridder_reference.cpp:16-25) -- true for the
    synthetic batch; otherwise None."""
    import numpy as np
    from concurrent.futures import ThreadPoolExecutor
    md_all = a["metadata"]
    cores = int(os.environ.get("IDG_CPU_BASELINE_THREADS", "16"))
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


def traffic_for(path, workload, kernel):
    try:
        with open(path) as f:
            t = json.load(f)
        return t[workload][kernel]["hbm_bytes_per_launch"]
    except Exception:
        return None


def reference_hip_for(workload, sec_per_step, t_grid, t_degrid):
    """The reference's own HIP kernels measured on MI355X at configs[1]
    (profiles/reference_hip.json, made by tests/debug/ref_hip.sh): this
    run's per-GPU rates over theirs, for the fastest reference kernels and
    for the fastest that pass the reference's own -c check."""
    if workload != "default":
        return None
    try:
        with open(os.path.join(REPO, "profiles", "reference_hip.json")) as f:
            ref = json.load(f)
    except Exception:
        return None
    out = {"source": "profiles/reference_hip.json "
                     "(profiles/r01/reference_hip/SUMMARY.md)"}
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


def issue_for(path, workload, kernel):
    """VALU-issue utilisation of a kernel from its committed PMC summary."""
    try:
        with open(path) as f:
            t = json.load(f)
        return t[workload][kernel].get("issue_bound")
    except Exception:
        return None


def main():
    args = parse()
    import numpy as np
    import torch
    import idg_amd
    from idg_amd import dist

    rank, local_rank, world = dist.init()
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a HIP device (no CPU fallback)")
    torch.cuda.set_device(local_rank)
    w = dict(WORKLOADS[args.workload])
    if args.timeslots:
        w["nr_timeslots"] = args.timeslots
    st, ts, T, C, G, S = (w["nr_stations"], w["nr_timeslots"],
                          w["nr_timesteps"], w["nr_channels"], w["grid_size"],
                          w["subgrid_size"])
    ns = idg_amd.nr_subgrids_for(st, ts)
    nvis = ns * T * C

    # ---- synthetic batch (reference generators), resident in HBM ----------
    threads = max(1, min(16, (os.cpu_count() or 8) // max(1, world)))
    a = idg_amd.generate(st, ts, T, C, G, S, nthreads=threads)
    apply_wterms(w, a)
    idg_amd.validate_metadata(ns, S, C, st, ns * T, ts, a["metadata"])
    dev = {k: torch.from_numpy(a[k]).cuda() for k in
           ("uvw", "wavenumbers", "visibilities", "spheroidal", "aterms",
            "subgrids")}
    dev["metadata"] = torch.from_numpy(
        a["metadata"].view(np.int32).reshape(-1, 9).copy()).cuda()
    grid_out = torch.empty_like(dev["subgrids"])
    degrid_out = torch.empty_like(dev["visibilities"])
    p = (ns, G, S, idg_amd.IMAGE_SIZE, w.get("w_step", idg_amd.W_STEP), C,
         st)
    stream = torch.cuda.current_stream()

    def step(ev=None):
        if ev:
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

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    events = [[torch.cuda.Event(enable_timing=True) for _ in range(3)]
              for _ in range(args.steps)]
    from idg_amd.energy import EnergyMeter
    meter = EnergyMeter(local_rank)
    dist.barrier()
    torch.cuda.synchronize()
    meter.start()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(events[k])
    torch.cuda.synchronize()
    joules = meter.stop()
    dist.barrier()
    elapsed = time.perf_counter() - t0
    elapsed_max = dist.max_over_ranks(elapsed)

    t_grid = sum(e[0].elapsed_time(e[1]) for e in events) / args.steps / 1e3
    t_degrid = sum(e[1].elapsed_time(e[2]) for e in events) / args.steps / 1e3
    t_grid = dist.max_over_ranks(t_grid)
    t_degrid = dist.max_over_ranks(t_degrid)
    sec_per_step = elapsed_max / args.steps

    flops = idg_amd.flops_gridder(C, ns * T, ns, S)
    nbytes = idg_amd.bytes_gridder(C, ns * T, ns, S)
    kernels = {}
    for name, t in (("gridder", t_grid), ("degridder", t_degrid)):
        kname = idg_amd.kernel_name(name, S, C)
        kernels[name] = {
            "kernel": kname,
            "ms": round(t * 1e3, 4),
            "mvis_s_per_gpu": round(nvis / t / 1e6, 2),
            "tflops": round(flops / t / 1e12, 3),
            "fp32_frac": round(flops / t / 1e12 / FP32_PEAK_TFLOPS, 4),
            "hbm_gbs_model": round(nbytes / t / 1e9, 2),
        }
    dom = "gridder" if t_grid >= t_degrid else "degridder"
    t_dom = t_grid if dom == "gridder" else t_degrid
    achieved = flops / t_dom / 1e12
    roofline = {
        "bound": "mfma",
        "achieved": round(achieved, 3),
        "peak": FP32_PEAK_TFLOPS,
        "unit": "TFLOP/s",
        "frac": round(achieved / FP32_PEAK_TFLOPS, 4),
        "traffic": traffic_for(args.traffic_file, args.workload,
                               kernels[dom]["kernel"]),
        "kernel": kernels[dom]["kernel"],
        "note": ("achieved = reference work model FLOPs per launch "
                 f"({flops / nvis:.0f} FLOP/vis x {nvis} vis) / mean "
                 "kernel duration (HIP events on the launch stream); peak = "
                 "gfx950 FP32 peak (vector = f32 MFMA = 157.3 TF), the "
                 "ceiling of the work model as the reference computes it. "
                 "frac > 1 is possible: the complex MAC (32 of the model's "
                 "~35 FLOP per pixel-visibility) runs on the f16 matrix "
                 "core with a two-term f16 split at f32 accuracy, so the "
                 "binding resource is VALU issue (exact phase, v_sin/v_cos, "
                 "split), see issue_bound"),
    }
    issue = issue_for(args.traffic_file, args.workload,
                      kernels[dom]["kernel"])
    if issue is not None:
        roofline["issue_bound"] = issue
    roofline_hbm = {
        "bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK_GBS,
        "achieved": round(nbytes / t_dom / 1e9, 2),
        "frac": round(nbytes / t_dom / 1e9 / HBM_PEAK_GBS, 4),
        "note": ("reference byte model (common.cpp:131-159, "
                 f"{nbytes / nvis:.2f} B/vis); AI = {flops / nbytes:.0f} "
                 "FLOP/B, so <= ~5.5% by construction"),
    }

    # ---- pipeline steps around the path (not in `value`): subgrid FFT,
    # adder onto the uv grid, the multi-GPU grid-sum over RCCL (the one
    # exchange step, BASELINE configs[3]), splitter, inverse FFT ----------
    pipeline = None
    if not args.no_pipeline:
        nw = w.get("w_layers", 1)
        gridt = torch.zeros((nw, 4, G, G, 2), dtype=torch.float32,
                            device="cuda")
        uvsub = torch.empty_like(grid_out)
        npipe = max(1, min(args.steps, 5))
        pev = [[torch.cuda.Event(enable_timing=True) for _ in range(6)]
               for _ in range(npipe)]
        for it in range(npipe + 1):
            e = pev[it - 1] if it > 0 else None
            uvsub.copy_(grid_out)
            gridt.zero_()
            dist.barrier()
            if e:
                e[0].record(stream)
            idg_amd.subgrid_fft_launch(uvsub, +1, 1.0, stream=stream)
            if e:
                e[1].record(stream)
            idg_amd.adder_launch(G, dev["metadata"], uvsub, gridt,
                                 nr_w_layers=nw, stream=stream)
            if e:
                e[2].record(stream)
            dist.reduce_grid(gridt)
            if e:
                e[3].record(stream)
            idg_amd.splitter_launch(G, dev["metadata"], gridt, uvsub,
                                    nr_w_layers=nw, stream=stream)
            if e:
                e[4].record(stream)
            idg_amd.subgrid_fft_launch(uvsub, -1, 1.0 / (S * S),
                                       stream=stream)
            if e:
                e[5].record(stream)
        torch.cuda.synchronize()

        def avg(i, j):
            return dist.max_over_ranks(
                sum(e[i].elapsed_time(e[j]) for e in pev) / npipe)
        pipeline = {
            "fft_ms": round(avg(0, 1), 4),
            "adder_ms": round(avg(1, 2), 4),
            "grid_reduce_ms": round(avg(2, 3), 4),
            "splitter_ms": round(avg(3, 4), 4),
            "ifft_ms": round(avg(4, 5), 4),
            "grid": (f"[{nw}][4][{G}][{G}] complex64, "
                     f"{nw * G * G * 32 / 2**20:.0f} MiB"),
            "grid_reduce": (f"all_reduce(sum), {dist.backend_name()}"
                            if world > 1 else "single rank: no collective"),
        }
        extra = sum(pipeline[k] for k in ("fft_ms", "adder_ms",
                                          "grid_reduce_ms", "splitter_ms",
                                          "ifft_ms")) / 1e3
        pipeline["full_cycle_mvis_s"] = round(
            world * nvis / (sec_per_step + extra) / 1e6, 2)
        pipeline["note"] = ("gridder -> FFT -> adder -> grid-sum and "
                            "splitter -> FFT -> degridder around the timed "
                            "step; reported beside `value`, not in it")

    # ---- energy over the timed region (amdsmi accumulated-energy counter;
    # the reference's PowerSensor report, app/HIP/util.cpp:134-159) --------
    energy = None
    if joules is not None and joules > 0:
        j_all = dist.sum_over_ranks(joules)
        energy = {
            "joules_per_step": round(j_all / args.steps, 4),
            "avg_power_w_per_gpu": round(j_all / world / elapsed, 1),
            "mvis_per_joule": round(world * nvis * args.steps / j_all / 1e6,
                                    3),
            "source": "amdsmi_get_energy_count over the timed steps",
        }

    result = {
        "metric": METRIC,
        "value": round(world * nvis / sec_per_step / 1e6, 2),
        "unit": "Mvis/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(sec_per_step * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (reference generators app/common/init.cpp, srand(0))",
        "config": {
            "workload": (f"{args.workload}: NR_STATIONS={st} "
                         f"NR_TIMESLOTS={ts} NR_TIMESTEPS_SUBGRID={T} "
                         f"NR_CHANNELS={C} SUBGRID_SIZE={S} GRID_SIZE={G}"
                         + (f" W_STEP={w['w_step']} w~U(-{w['w_range']:g},"
                            f"{w['w_range']:g}) w-layers={w['w_layers']}"
                            if w.get("w_range") else "")),
            "baseline_config": ("configs[1]" if args.workload == "default"
                                else {"c256": "configs[2]",
                                      "s64": "configs[4]",
                                      "wterm": "SURVEY.md §8f row 4"}[
                                          args.workload]),
            "nr_subgrids_per_gpu": ns,
            "visibilities_per_gpu_per_step": nvis,
            "step": "gridder + degridder over the batch",
            "parallelism": f"subgrid-sharded x{world}, no data-path collective",
        },
        "gridder_mvis_s": round(world * nvis / t_grid / 1e6, 2),
        "degridder_mvis_s": round(world * nvis / t_degrid / 1e6, 2),
        "kernels": kernels,
        "roofline": roofline,
        "roofline_hbm": roofline_hbm,
        "pipeline": pipeline,
        "energy": energy,
        "reference_hip_mi355x": reference_hip_for(
            args.workload, sec_per_step, t_grid, t_degrid),
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(w, a, args.cpu_sample_subgrids)
    if rank == 0:
        print(json.dumps(result), flush=True)
    dist.finalize()


if __name__ == "__main__":
    main()
