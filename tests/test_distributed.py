"""World-size-2 gloo rehearsal of the multi-GPU path (CPU only).

The subgrid shard plan + rebasing (idg_amd.shard) and the driver's
collectives (idg_amd.dist: barrier, max-over-ranks, gather of shard outputs)
run on two CPU processes; the per-shard compute is the CPU oracle standing in
for the GPU kernel (the oracle is the checker here, not the thing shipped).
The gathered result must equal a single-process run bit for bit.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import ORACLE, PKG


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, result_path):
    import sys
    for p in (PKG, ORACLE):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      RANK=str(rank), LOCAL_RANK=str(rank),
                      WORLD_SIZE=str(world))
    import idg_amd
    from idg_amd import dist, shard
    import oracle as orc
    r, _, w = dist.init(backend="gloo")
    st, ts, T, C, G, S = 4, 3, 6, 3, 256, 16
    a = idg_amd.generate(st, ts, T, C, G, S)
    md = a["metadata"]
    plan = shard.plan_shards(md, w)
    s0, s1 = plan[r]
    sub, r0, r1 = shard.shard(md, s0, s1)
    out = np.zeros((s1 - s0, 4, S, S, 2), np.float32)
    uvw = np.ascontiguousarray(a["uvw"].reshape(-1, 3)[r0:r1])
    vis = np.ascontiguousarray(a["visibilities"].reshape(-1, C, 4, 2)[r0:r1])
    orc.Oracle().gridder(s1 - s0, G, S, idg_amd.IMAGE_SIZE, 0.0, C, st, uvw,
                         a["wavenumbers"], vis, a["spheroidal"], a["aterms"],
                         sub, out)
    counts = [b - a_ for a_, b in plan]
    full = dist.gather_shards(torch.from_numpy(out), counts)
    dist.barrier()
    tmax = dist.max_over_ranks(float(r + 1))
    tsum = dist.sum_over_ranks(1.0)
    if r == 0:
        np.save(result_path, full.numpy())
        with open(result_path + ".txt", "w") as f:
            f.write(f"{tmax} {tsum}")
    dist.finalize()


@pytest.mark.timeout(300)
def test_gloo_world2_sharded_gridder_equals_single_process(tmp_path,
                                                           oracle_lib):
    import idg_amd
    port = _free_port()
    path = str(tmp_path / "full.npy")
    mp.start_processes(_worker, args=(2, port, path), nprocs=2, join=True,
                       start_method="spawn")
    got = np.load(path)
    st, ts, T, C, G, S = 4, 3, 6, 3, 256, 16
    a = idg_amd.generate(st, ts, T, C, G, S)
    ns = a["metadata"].size
    ref = np.zeros((ns, 4, S, S, 2), np.float32)
    oracle_lib.gridder(ns, G, S, idg_amd.IMAGE_SIZE, 0.0, C, st, a["uvw"],
                       a["wavenumbers"], a["visibilities"], a["spheroidal"],
                       a["aterms"], a["metadata"], ref)
    assert np.array_equal(got, ref)
    tmax, tsum = open(path + ".txt").read().split()
    assert float(tmax) == 2.0 and float(tsum) == 2.0


def _grid_worker(rank, world, port, result_path):
    """Each rank grids its shard (oracle gridder + numpy FFT/adder standing
    in for the GPU steps) onto a partial uv grid; reduce_grid sums them."""
    import sys
    for p in (PKG, ORACLE):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      RANK=str(rank), LOCAL_RANK=str(rank),
                      WORLD_SIZE=str(world))
    import idg_amd
    from idg_amd import dist, shard
    import oracle as orc
    import pipeline_oracle as pl
    r, _, w = dist.init(backend="gloo")
    st, ts, T, C, G, S = 4, 3, 6, 3, 256, 16
    a = idg_amd.generate(st, ts, T, C, G, S)
    md = a["metadata"]
    s0, s1 = shard.plan_shards(md, w)[r]
    sub, r0, r1 = shard.shard(md, s0, s1)
    out = np.zeros((s1 - s0, 4, S, S, 2), np.float32)
    uvw = np.ascontiguousarray(a["uvw"].reshape(-1, 3)[r0:r1])
    vis = np.ascontiguousarray(a["visibilities"].reshape(-1, C, 4, 2)[r0:r1])
    orc.Oracle().gridder(s1 - s0, G, S, idg_amd.IMAGE_SIZE, 0.0, C, st, uvw,
                         a["wavenumbers"], vis, a["spheroidal"], a["aterms"],
                         sub, out)
    part = pl.adder(np.zeros((1, 4, G, G), complex), sub,
                    pl.subgrid_fft(pl.to_complex(out), +1))
    grid = torch.from_numpy(np.ascontiguousarray(pl.to_pairs(part)))
    dist.reduce_grid(grid)
    if r == 0:
        np.save(result_path, grid.numpy())
    dist.finalize()


@pytest.mark.timeout(300)
def test_gloo_world2_grid_reduce_equals_single_process(tmp_path, oracle_lib):
    """The pipeline's one exchange step (SURVEY.md §8e final grid-sum): the
    sum of the ranks' partial grids equals gridding every subgrid at once."""
    import idg_amd
    import pipeline_oracle as pl
    port = _free_port()
    path = str(tmp_path / "grid.npy")
    mp.start_processes(_grid_worker, args=(2, port, path), nprocs=2,
                       join=True, start_method="spawn")
    got = pl.to_complex(np.load(path))
    st, ts, T, C, G, S = 4, 3, 6, 3, 256, 16
    a = idg_amd.generate(st, ts, T, C, G, S)
    ns = a["metadata"].size
    sg = np.zeros((ns, 4, S, S, 2), np.float32)
    oracle_lib.gridder(ns, G, S, idg_amd.IMAGE_SIZE, 0.0, C, st, a["uvw"],
                       a["wavenumbers"], a["visibilities"], a["spheroidal"],
                       a["aterms"], a["metadata"], sg)
    ref = pl.adder(np.zeros((1, 4, G, G), complex), a["metadata"],
                   pl.subgrid_fft(pl.to_complex(sg), +1))
    assert np.abs(got - ref).max() <= 1e-5 * np.abs(ref).max()


# ---------------------------------------------------------------------------
# bench.py's own sharded path (BASELINE configs[3]) at world size 2
# ---------------------------------------------------------------------------
SMALL = dict(nr_stations=5, nr_timeslots=3, nr_timesteps=8, nr_channels=3,
             grid_size=256, subgrid_size=16)


def _bench_worker(rank, world, port, out_dir, mode):
    """One rank of bench.py's sharded run with the oracle standing in for the
    HIP kernels: bench.make_batch -> bench.shard_batch (this rank's
    subgrids, rebased metadata, only the rows they read) -> grid + degrid
    -> subgrid FFT + adder onto a partial grid -> dist.reduce_grid ->
    bench.dump_outputs (gather in rank order, write on rank 0)."""
    import sys
    for p in (PKG, ORACLE, os.path.dirname(PKG)):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      RANK=str(rank), LOCAL_RANK=str(rank),
                      WORLD_SIZE=str(world))
    import bench
    import idg_amd
    from idg_amd import dist
    import oracle as orc
    import pipeline_oracle as pl
    r, _, w_ = dist.init(backend="gloo")
    w = dict(SMALL)
    a = bench.make_batch(w, nthreads=1)
    part = bench.shard_batch(a, r, w_, mode)
    n = part["s1"] - part["s0"]
    S, C, G = w["subgrid_size"], w["nr_channels"], w["grid_size"]
    p = (n, G, S, idg_amd.IMAGE_SIZE, 0.0, C, w["nr_stations"])
    o = orc.Oracle()
    sg = np.zeros((n, 4, S, S, 2), np.float32)
    o.gridder(*p, part["uvw"], part["wavenumbers"], part["visibilities"],
              part["spheroidal"], part["aterms"], part["metadata"], sg)
    vis = np.zeros_like(part["visibilities"])
    o.degridder(*p, part["uvw"], part["wavenumbers"], vis,
                part["spheroidal"], part["aterms"], part["metadata"],
                part["subgrids"])
    grid = pl.adder(np.zeros((1, 4, G, G), complex), part["metadata"],
                    pl.subgrid_fft(pl.to_complex(sg), +1))
    grid = torch.from_numpy(np.ascontiguousarray(pl.to_pairs(grid)))
    dist.reduce_grid(grid)
    bench.dump_outputs(out_dir, a, part,
                       (torch.from_numpy(sg), torch.from_numpy(vis)), grid,
                       r, w_, mode, dist)
    dist.finalize()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("mode", ["sharded", "replicated"])
def test_gloo_world2_bench_sharded_path_equals_single_rank(tmp_path, mode):
    """bench.py --gpus 2: the ranks' gathered subgrids and degridded
    visibilities equal one rank's bit for bit (disjoint shards, the same
    per-subgrid arithmetic), and the all-reduced grid equals one rank's grid
    up to float summation order (two partial sums instead of one running
    sum)."""
    import pipeline_oracle as pl
    outs = {}
    for world in (1, 2):
        d = str(tmp_path / f"w{world}")
        mp.start_processes(_bench_worker, args=(world, _free_port(), d, mode),
                           nprocs=world, join=True, start_method="spawn")
        outs[world] = {k: np.load(os.path.join(d, k + ".npy"))
                       for k in ("subgrids", "visibilities", "grid")}
    one, two = outs[1], outs[2]
    ns = SMALL["nr_stations"] * (SMALL["nr_stations"] - 1) // 2 * \
        SMALL["nr_timeslots"]
    assert one["subgrids"].shape[0] == ns == two["subgrids"].shape[0]
    assert np.array_equal(one["subgrids"], two["subgrids"])
    assert np.array_equal(one["visibilities"], two["visibilities"])
    g1, g2 = pl.to_complex(one["grid"]), pl.to_complex(two["grid"])
    scale = 2.0 if mode == "replicated" else 1.0  # every rank adds it all
    assert np.abs(g2 - scale * g1).max() <= 1e-6 * np.abs(g1).max()


def test_bench_shard_batch_uploads_only_its_rows():
    import bench
    a = bench.make_batch(dict(SMALL), nthreads=1)
    T, C = SMALL["nr_timesteps"], SMALL["nr_channels"]
    parts = [bench.shard_batch(a, r, 3) for r in range(3)]
    assert [p["s1"] - p["s0"] for p in parts] == bench.shard_counts(a, 3)
    assert sum(p["s1"] - p["s0"] for p in parts) == a["metadata"].size
    for p in parts:
        n = p["s1"] - p["s0"]
        assert p["visibilities"].shape == (n * T, C, 4, 2)
        assert p["uvw"].shape == (n * T, 3)
        assert p["metadata"]["time_offset"][0] == 0
        assert np.array_equal(
            p["visibilities"].reshape(n, T, C, 4, 2),
            a["visibilities"][p["s0"]:p["s1"]])


# ---------------------------------------------------------------------------
# bench.py's warm-up: every rank runs the same untimed step count
# ---------------------------------------------------------------------------
def _warmup_worker(rank, world, port, out_dir):
    """Ranks price their step differently (rank r: (2 + r) ms); the count
    bench.time_steps runs is the max over ranks of extra_warmup_steps."""
    import sys
    for p in (PKG, os.path.dirname(PKG)):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      RANK=str(rank), LOCAL_RANK=str(rank),
                      WORLD_SIZE=str(world))
    import bench
    from idg_amd import dist
    r, _, _ = dist.init(backend="gloo")
    mine = bench.extra_warmup_steps((2 + r) * 1e-3, 1.0)
    agreed = int(dist.max_over_ranks(mine))
    np.save(os.path.join(out_dir, f"r{r}.npy"), np.array([mine, agreed]))
    dist.finalize()


def test_dtype_label_follows_the_selected_kernels():
    import bench
    mf = {"kernel": "gridder_mi355x_s32"}
    va = {"kernel": "gridder_mi355x_s32_valu"}
    assert bench.dtype_label({"gridder": mf, "degridder": mf}).startswith(
        "f32 phase/accumulate, f16x2-split")
    assert bench.dtype_label({"gridder": va, "degridder": va}) == "f32"
    mixed = bench.dtype_label({"gridder": va, "degridder": mf})
    assert mixed.startswith("gridder: f32; degridder: f32 phase")


def test_extra_warmup_steps():
    import bench
    assert bench.extra_warmup_steps(0.015, 1.0) == 67   # configs[1], N = 1
    assert bench.extra_warmup_steps(0.002, 1.0) == 501  # N = 8 shard
    assert bench.extra_warmup_steps(0.0, 1.0) == 10001  # bounded
    assert bench.extra_warmup_steps(5.0, 1.0) == 1      # the pricing step
    assert bench.extra_warmup_steps(0.002, 0.0) == 0    # exactly W steps


@pytest.mark.timeout(120)
def test_gloo_world2_warmup_count_agreed(tmp_path):
    mp.start_processes(_warmup_worker, args=(2, _free_port(), str(tmp_path)),
                       nprocs=2, join=True, start_method="spawn")
    got = [np.load(str(tmp_path / f"r{r}.npy")) for r in range(2)]
    assert got[0][0] == 501 and got[1][0] == 334
    assert got[0][1] == got[1][1] == 501


@pytest.mark.parametrize("n,counts", [(2, [1225, 1225]),
                                      (4, [613, 612, 613, 612])])
def test_bench_plain_command_launches_its_own_ranks(n, counts):
    """`python bench.py --gpus N` without torchrun: the process
    starts torch.distributed.run on itself as a child, the ranks rendezvous
    on 127.0.0.1 and shard the batch, and rank 0's line is the command's
    output.  --plan-only stops after the plan (no device on this host)."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(ORACLE)
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["IDG_DIST_BACKEND"] = "gloo"
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"),
                        "--gpus", str(n), "--timeslots", "2", "--plan-only"],
                       env=env, capture_output=True, text=True, timeout=300,
                       cwd="/tmp")
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = [json.loads(l) for l in r.stdout.splitlines()
             if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = lines[0]
    assert line["n_gpus"] == n and line["ranks_in_collective"] == n
    assert line["config"]["nr_subgrids_per_gpu"] == counts
    assert sum(counts) == line["config"]["nr_subgrids"] == 2450


def test_bench_plain_command_propagates_a_rank_failure():
    # a batch the generator rejects (negative timeslots) fails inside every
    # rank, after the launch: the launcher's exit code must say so
    import subprocess
    import sys
    repo = os.path.dirname(ORACLE)
    env = {k: v for k, v in os.environ.items() if k != "WORLD_SIZE"}
    env["IDG_DIST_BACKEND"] = "gloo"
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"),
                        "--gpus", "2", "--timeslots", "-1", "--plan-only"],
                       env=env, capture_output=True, text=True, timeout=300,
                       cwd="/tmp")
    assert r.returncode != 0
    assert "torch.distributed" in r.stderr or "Error" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
