"""The adder (home sort + kernel_adder) on subgrid layouts of increasing
concentration around the grid centre: the configs[1] batch's own corners,
then the same 24,500 subgrids with corners drawn from a Gaussian of shrinking
width, so the densest tile's overlap count crosses the LDS list's cap
(kAddListCap = 1,536: above it a tile falls back to an ordered scan of all
the metadata).  Prints, per layout, the densest tile's overlap count, the
tiles over the cap and the adder's mean time (HIP events, 10 launches).

    python tools/debug/adder_crowded.py [--sigmas 200,100,75,60,40,15]
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "ska-sdp-idg-bench_amd"))

CAP = 1536  # pipeline_mi355x.hip.cpp kAddListCap
TILE = 16   # IDG_ADD_TW / IDG_ADD_TH


def tile_overlaps(x, y, G, S):
    nt = (G + TILE - 1) // TILE
    cnt = np.zeros((nt, nt), np.int64)
    for dx in range(S // TILE + 1):
        for dy in range(S // TILE + 1):
            tx, ty = x // TILE + dx, y // TILE + dy
            ok = (tx * TILE < x + S) & (ty * TILE < y + S) & (tx < nt) & (ty < nt)
            np.add.at(cnt, (ty[ok], tx[ok]), 1)
    return cnt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sigmas", default="200,100,75,60,40,15")
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    import torch
    import bench
    import idg_amd
    assert torch.cuda.is_available(), "needs a HIP device"
    w = bench.workload("default")
    a = bench.make_batch(w, nthreads=16)
    G, S = w["grid_size"], w["subgrid_size"]
    md0 = a["metadata"]
    n = md0.size
    sub = torch.randn((n, 4, S, S, 2), dtype=torch.float32, device="cuda")
    grid = torch.zeros((1, 4, G, G, 2), dtype=torch.float32, device="cuda")
    stream = torch.cuda.current_stream()
    rng = np.random.default_rng(5)
    layouts = [("configs[1]", None)] + [
        (f"gauss sigma={s}", float(s)) for s in args.sigmas.split(",")]
    for name, sigma in layouts:
        md = md0.copy()
        if sigma is not None:
            c = (G - S) / 2
            md["x"] = np.clip(np.rint(rng.normal(c, sigma, n)), 0, G - S)
            md["y"] = np.clip(np.rint(rng.normal(c, sigma, n)), 0, G - S)
        cnt = tile_overlaps(md["x"].astype(np.int64), md["y"].astype(np.int64),
                            G, S)
        dmd = torch.from_numpy(md.view(np.int32).reshape(-1, 9).copy()).cuda()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        idg_amd.adder_launch(G, dmd, sub, grid, stream=stream)  # warm-up
        torch.cuda.synchronize()
        ev[0].record(stream)
        for _ in range(args.reps):
            idg_amd.adder_launch(G, dmd, sub, grid, stream=stream)
        ev[1].record(stream)
        torch.cuda.synchronize()
        print(json.dumps({"layout": name, "max_overlaps": int(cnt.max()),
                          "tiles_over_cap": int((cnt > CAP).sum()),
                          "adder_ms": round(ev[0].elapsed_time(ev[1]) /
                                            args.reps, 4)}), flush=True)


if __name__ == "__main__":
    main()
