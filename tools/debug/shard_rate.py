"""Strong-scaling rehearsal on ONE GPU: time the gridder + degridder on the
subgrid shard that rank r of an N-rank bench.py run would own (first and last
rank of N = 1, 2, 4, 8; bench.shard_batch, identical code path), and print the
per-GPU efficiency those shard times predict for the sharded bench line:
    eff(N) = t_step(N = 1) / (N * max over the timed ranks of t_step(N)).
It measures only the kernels' tail / launch behaviour at 3,062 subgrids per
GPU (configs[3] at N = 8); RCCL and the host are not in it.

    python tools/debug/shard_rate.py [--steps 10] [--workload default]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "ska-sdp-idg-bench_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="default")
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--counts", default=None,
                    help="instead of shards: time the first n subgrids for "
                         "each n of this comma list (fixed cost per launch)")
    ap.add_argument("--min-warmup-s", type=float, default=1.0,
                    help="as bench.py (0: exactly --warmup steps)")
    ap.add_argument("--gap-ms", type=float, default=0.0,
                    help="host sleep in the barrier before/after timing "
                         "(an idle GPU between warm-up and timed steps)")
    args = ap.parse_args()
    import time
    import torch
    import bench
    from idg_amd import dist
    dist.init()
    if args.gap_ms:
        dist.barrier = lambda: time.sleep(args.gap_ms / 1e3)
    assert torch.cuda.is_available(), "needs a HIP device"
    w = bench.workload(args.workload)
    a = bench.make_batch(w, nthreads=16)
    stream = torch.cuda.current_stream()
    if args.counts:
        from idg_amd import shard
        C = a["wavenumbers"].size
        for n in [int(x) for x in args.counts.split(",")]:
            sub, r0, r1 = shard.shard(a["metadata"], 0, n)
            part = dict(a, metadata=sub, s0=0, s1=n,
                        uvw=a["uvw"].reshape(-1, 3)[r0:r1].copy(),
                        visibilities=a["visibilities"].reshape(
                            -1, C, 4, 2)[r0:r1].copy(),
                        subgrids=a["subgrids"][:n].copy())
            dev = bench.upload(part)
            el, tg, td, _, _, _ = bench.time_steps(
                w, dev, n, args.steps, args.warmup, stream, dist,
                min_warmup_s=args.min_warmup_s)
            del dev
            torch.cuda.empty_cache()
            print(json.dumps({"nr_subgrids": n,
                              "gridder_ms": round(tg * 1e3, 4),
                              "degridder_ms": round(td * 1e3, 4),
                              "wall_ms_per_step": round(
                                  el / args.steps * 1e3, 4)}),
                  flush=True)
        return
    rows, base = [], None
    for world in [int(x) for x in args.worlds.split(",")]:
        ranks = sorted({0, world - 1})
        worst = 0.0
        for rank in ranks:
            part = bench.shard_batch(a, rank, world)
            nsub = part["s1"] - part["s0"]
            dev = bench.upload(part)
            el, tg, td, _, _, _ = bench.time_steps(
                w, dev, nsub, args.steps, args.warmup, stream, dist,
                min_warmup_s=args.min_warmup_s)
            del dev
            torch.cuda.empty_cache()
            step = tg + td
            worst = max(worst, step)
            rows.append({"world": world, "rank": rank, "nr_subgrids": nsub,
                         "gridder_ms": round(tg * 1e3, 4),
                         "degridder_ms": round(td * 1e3, 4),
                         "step_ms": round(step * 1e3, 4),
                         "wall_ms_per_step": round(
                             el / args.steps * 1e3, 4)})
            print(json.dumps(rows[-1]), flush=True)
        if base is None:
            base = worst
        eff = base / (world * worst)
        print(json.dumps({"world": world, "predicted_step_ms": round(
            worst * 1e3, 4), "predicted_efficiency": round(eff, 4)}),
            flush=True)


if __name__ == "__main__":
    main()
