"""The adder's tile order over the 8 XCDs: each XCD's share of the subgrid
pixels the adder gathers (configs[1] batch, or --workload), for the
XCD-contiguous order alone (device.hpp xcd_subgrid) and with the rows dealt
by r % 8 first (adder_tile, tried in round 6 and not kept: the adder
kernel ran as before and the splitter after it lost the grid band its XCD
had just written, 0.18 -> 0.205 ms, profiles/r06/adder/); and a check that
adder_tile is a bijection for every tile-grid shape up to 64 x 64.
    python tools/debug/adder_balance.py [--workload default]
"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__))))
sys.path.insert(0, REPO)


def xcd_subgrid(b, n):
    q, r, x = n // 8, n % 8, b % 8
    return (x * (q + 1) if x < r else r * (q + 1) + (x - r) * q) + b // 8


def adder_tile(p, ntx, nty):
    rp, col = divmod(p, ntx)
    x, before = 0, 0
    while x < 7:
        nx = (nty - x + 7) // 8
        if rp < before + nx:
            break
        before += nx
        x += 1
    return (x + 8 * (rp - before)) * ntx + col


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="default")
    args = ap.parse_args()
    for ntx in range(1, 65):
        for nty in range(1, 65):
            n = ntx * nty
            assert sorted(adder_tile(p, ntx, nty) for p in range(n)) == \
                list(range(n)), (ntx, nty)
    print("adder_tile: a bijection for every ntx, nty <= 64")
    import bench
    w = bench.workload(args.workload)
    md = bench.make_batch(w, nthreads=8)["metadata"]
    G, S, T = w["grid_size"], w["subgrid_size"], 16
    ntx = nty = (G + T - 1) // T
    pix = np.zeros((nty, ntx))
    for cx, cy in zip(md["x"], md["y"]):
        if cx < 0 or cy < 0 or cx + S > G or cy + S > G:
            continue
        for ty in range(cy // T, min(nty, (cy + S - 1) // T + 1)):
            oy = min(cy + S, (ty + 1) * T) - max(cy, ty * T)
            for tx in range(cx // T, min(ntx, (cx + S - 1) // T + 1)):
                ox = min(cx + S, (tx + 1) * T) - max(cx, tx * T)
                if ox > 0 and oy > 0:
                    pix[ty, tx] += ox * oy
    work = pix.ravel()
    n = ntx * nty
    for name, tile in (("xcd_subgrid", lambda p: p),
                       ("xcd_subgrid + adder_tile",
                        lambda p: adder_tile(p, ntx, nty))):
        share = np.zeros(8)
        for b in range(n):
            share[b % 8] += work[tile(xcd_subgrid(b, n))]
        print(f"{name:26s} XCD shares of the mean: "
              + " ".join(f"{v:.3f}" for v in share / share.mean()))


if __name__ == "__main__":
    main()
