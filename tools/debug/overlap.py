"""Serial vs overlapped steps on ONE GPU: K steps of (gridder; degridder) on
one stream, against the gridder's K launches on one stream and the
degridder's K launches on a second stream, both streams running at once (the
two directions read and write disjoint buffers).  Wall clock of the K steps
after >= 1 s of warm-up in the same form; full batch and the N = 2/4/8 shard
sizes (first n subgrids).

    python tools/debug/overlap.py [--steps 20] [--counts 24500,6125,3063]
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
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--counts", default="24500,12250,6125,3063")
    ap.add_argument("--workload", default="default")
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()
    import torch
    import bench
    import idg_amd
    from idg_amd import shard
    assert torch.cuda.is_available(), "needs a HIP device"
    w = bench.workload(args.workload)
    a = bench.make_batch(w, nthreads=16)
    C = a["wavenumbers"].size
    s_main = torch.cuda.current_stream()
    s_b = torch.cuda.Stream()
    for n in [int(x) for x in args.counts.split(",")]:
        sub, r0, r1 = shard.shard(a["metadata"], 0, n)
        part = dict(a, metadata=sub, s0=0, s1=n,
                    uvw=a["uvw"].reshape(-1, 3)[r0:r1].copy(),
                    visibilities=a["visibilities"].reshape(
                        -1, C, 4, 2)[r0:r1].copy(),
                    subgrids=a["subgrids"][:n].copy())
        dev = bench.upload(part)
        p = (n, w["grid_size"], w["subgrid_size"], idg_amd.IMAGE_SIZE,
             w.get("w_step", idg_amd.W_STEP), C, w["nr_stations"])
        gout = torch.empty_like(dev["subgrids"])
        dout = torch.empty_like(dev["visibilities"])

        def grid(st):
            idg_amd.gridder_launch(*p, dev["uvw"], dev["wavenumbers"],
                                   dev["visibilities"], dev["spheroidal"],
                                   dev["aterms"], dev["metadata"], gout,
                                   stream=st)

        def degrid(st):
            idg_amd.degridder_launch(*p, dev["uvw"], dev["wavenumbers"], dout,
                                     dev["spheroidal"], dev["aterms"],
                                     dev["metadata"], dev["subgrids"],
                                     stream=st)

        def serial(k):
            for _ in range(k):
                grid(s_main)
                degrid(s_main)

        def overlapped(k):
            s_b.wait_stream(s_main)
            for _ in range(k):
                grid(s_main)
                degrid(s_b)
            s_main.wait_stream(s_b)

        def timed(fn, k):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn(k)
            torch.cuda.synchronize()
            return time.perf_counter() - t0

        for rep in range(args.reps):
            for name, fn in (("serial", serial), ("overlapped", overlapped)):
                t1 = timed(fn, 1)
                timed(fn, max(1, int(1.0 / t1)))
                el = timed(fn, args.steps)
                ms = el / args.steps * 1e3
                print(json.dumps({"nr_subgrids": n, "form": name, "rep": rep,
                                  "ms_per_step": round(ms, 4),
                                  "mvis_s": round(n * 128 * C / ms / 1e3, 1)}),
                      flush=True)
        # outputs of the overlapped form equal the serial ones bit for bit
        serial(1)
        torch.cuda.synchronize()
        g1, d1 = gout.clone(), dout.clone()
        gout.zero_()
        dout.zero_()
        overlapped(1)
        torch.cuda.synchronize()
        print(json.dumps({"nr_subgrids": n, "bitwise_equal":
                          bool(torch.equal(g1, gout) and torch.equal(d1, dout))}),
              flush=True)
        del dev, gout, dout, g1, d1
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
