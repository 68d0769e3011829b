"""Per-workgroup timeline of the combined kernels at a shard-size launch
(debug build: make BUILD=build_tl LIB=../ab/tl.so EXTRA=-DIDG_WG_TIMELINE=1,
run with IDG_MI355X_LIB=ab/tl.so IDG_KERNEL_FORM=combined):

    python tools/debug/wg_timeline.py [--counts 3063,24500] [--steps 3]

For the last gridder and degridder launch of `--steps` bench steps over the
first n subgrids of configs[1] it prints, from the workgroups' own
s_memrealtime stamps (10 ns): the launch window, the dispatch ramp (spread of
the first round's starts), mean workgroup duration in the first round, the
middle and the last round, and the drain (from the last workgroup start to
the last end, and how much of the window the slots sit idle at the end,
against the half workgroup duration a steady stagger leaves anyway), and
each XCD's last end."""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "ska-sdp-idg-bench_amd"))

STAMP = np.dtype([("t0", "<u8"), ("t1", "<u8"), ("hw", "<u4"),
                  ("xcc", "<u4")])


def analyse(st, name):
    t0 = st["t0"].astype(np.int64)
    t1 = st["t1"].astype(np.int64)
    start, end = t0.min(), t1.max()
    t0 = (t0 - start) * 10 / 1e3   # us
    t1 = (t1 - start) * 10 / 1e3
    dur = t1 - t0
    order = np.argsort(t0)
    slots = 0
    # concurrent workgroups right after the ramp = the resident slots
    first = t0[order[0]]
    for k in range(len(t0)):
        if t0[order[k]] > first + 5.0:
            break
        slots = k + 1
    rnd = order[:slots], order[len(order) // 2:len(order) // 2 + slots], \
        order[-slots:]
    busy_end = np.sort(t1)
    # idle slot-time at the end: each of the `slots` slots is idle from its
    # last workgroup's end to the window's end; approximate by the last
    # `slots` ends
    tail_ends = busy_end[-slots:]
    idle = float(np.sum(tail_ends[-1] - tail_ends)) / slots
    out = {
        "kernel": name, "workgroups": int(len(t0)), "slots": int(slots),
        "window_us": round(float(t1.max()), 2),
        "ramp_us (first-round start spread)": round(
            float(t0[rnd[0]].max() - t0[rnd[0]].min()), 2),
        "mean_us first/middle/last round": [
            round(float(dur[r].mean()), 2) for r in rnd],
        "last_start_to_end_us": round(float(t1.max() - t0.max()), 2),
        "mean_idle_us_per_slot_at_end": round(idle, 2),
        # what a steady state of staggered workgroups leaves anyway: the
        # last round's ends spread over one workgroup duration
        "uniform_end_idle_us": round(float(dur.mean()) / 2, 2),
        "sum_dur/slots_us": round(float(dur.sum()) / slots, 2),
    }
    # per-XCD end times
    xcc = st["xcc"] & 0xF
    out["xcc_last_end_us"] = [round(float(t1[xcc == x].max()), 1)
                              for x in np.unique(xcc)]
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--counts", default="3063")
    ap.add_argument("--steps", type=int, default=3)
    args = ap.parse_args()
    import torch
    import bench
    from idg_amd import dist, shard
    import idg_amd
    lib = idg_amd._lib.lib
    dist.init()
    w = bench.workload("default")
    a = bench.make_batch(w, nthreads=16)
    stream = torch.cuda.current_stream()
    C = a["wavenumbers"].size
    for n in [int(x) for x in args.counts.split(",")]:
        sub, r0, r1 = shard.shard(a["metadata"], 0, n)
        part = dict(a, metadata=sub, s0=0, s1=n,
                    uvw=a["uvw"].reshape(-1, 3)[r0:r1].copy(),
                    visibilities=a["visibilities"].reshape(
                        -1, C, 4, 2)[r0:r1].copy(),
                    subgrids=a["subgrids"][:n].copy())
        dev = bench.upload(part)
        bench.time_steps(w, dev, n, args.steps, 1, stream, dist)
        torch.cuda.synchronize()
        for name in ("gridder", "degridder"):
            buf = np.zeros(min(n, 32768), STAMP)
            fn = getattr(lib, f"idg_debug_timeline_{name}_copy")
            rc = fn(ctypes.c_void_p(buf.ctypes.data), ctypes.c_int(buf.size))
            assert rc == 0, rc
            print(f"n={n}", end=" ")
            analyse(buf, name)
        del dev
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
