"""What the per-kernel timing events cost the wall clock of a timed step.
Times the gridder + degridder step on one shard (default: rank 7 of an
N = 8 bench run, 3,062 subgrids) with 0, 2 (shared step-boundary events)
and 3 events per step, interleaved, same process:
    python tools/debug/event_cost.py [--world 8] [--steps 50] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "ska-sdp-idg-bench_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch
    import bench
    import idg_amd
    w = bench.workload("default")
    a = bench.make_batch(w, nthreads=16)
    part = bench.shard_batch(a, args.world - 1, args.world)
    nsub = part["s1"] - part["s0"]
    dev = bench.upload(part)
    stream = torch.cuda.current_stream()
    S, C, G = w["subgrid_size"], w["nr_channels"], w["grid_size"]
    p = (nsub, G, S, idg_amd.IMAGE_SIZE, w.get("w_step", idg_amd.W_STEP), C,
         w["nr_stations"])
    gout = torch.empty_like(dev["subgrids"])
    dout = torch.empty_like(dev["visibilities"])

    def grid():
        idg_amd.gridder_launch(*p, dev["uvw"], dev["wavenumbers"],
                               dev["visibilities"], dev["spheroidal"],
                               dev["aterms"], dev["metadata"], gout,
                               stream=stream)

    def degrid():
        idg_amd.degridder_launch(*p, dev["uvw"], dev["wavenumbers"], dout,
                                 dev["spheroidal"], dev["aterms"],
                                 dev["metadata"], dev["subgrids"],
                                 stream=stream)

    def run(mode, steps):
        ev = [torch.cuda.Event(enable_timing=True)
              for _ in range(2 * steps + 1 if mode == 2 else 3 * steps)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(steps):
            if mode == 3:
                ev[3 * k].record(stream)
            elif mode == 2 and k == 0:
                ev[0].record(stream)
            grid()
            if mode == 3:
                ev[3 * k + 1].record(stream)
            elif mode == 2:
                ev[2 * k + 1].record(stream)
            degrid()
            if mode == 3:
                ev[3 * k + 2].record(stream)
            elif mode == 2:
                ev[2 * k + 2].record(stream)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps * 1e3

    # warm-up: about 2 s of steps (the clock ramp, bench.py time_steps)
    t = time.perf_counter()
    while time.perf_counter() - t < 2.0:
        run(0, 20)
    for rep in range(args.reps):
        for mode in (0, 2, 3):
            print(json.dumps({"rep": rep, "events_per_step": mode,
                              "nr_subgrids": nsub,
                              "wall_ms_per_step": round(run(mode, args.steps), 4)}),
                  flush=True)


if __name__ == "__main__":
    main()
