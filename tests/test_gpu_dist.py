"""bench.py's multi-GPU path on the HIP kernels (run on the GPU box: -m gpu).

`bench.py --gpus 2` (as a plain command, and under torchrun), with
IDG_DIST_BACKEND=gloo so that both
ranks can share the box's one device (RCCL refuses two ranks on one GPU),
shards BASELINE configs[1]'s subgrids over the ranks exactly as the 8-GPU run
does (BASELINE configs[3]).  Its gathered gridder subgrids and degridded
visibilities must equal a one-rank run bit for bit, and its all-reduced uv
grid must equal the one-rank grid up to float summation order.  Reduced batch
(NR_TIMESLOTS=2, 2,450 subgrids) so the two runs take seconds.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(cmd, env, timeout=240):
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True,
                       text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    return json.loads(lines[-1])


@pytest.mark.timeout(600)
@pytest.mark.parametrize("launcher", ["plain", "torchrun"])
def test_bench_two_ranks_sharded_equals_one_rank(tmp_path, launcher):
    """launcher "plain": `python bench.py --gpus 2` with no WORLD_SIZE starts
    its own ranks (bench.launch_ranks); "torchrun": the driver's form."""
    common = ["--steps", "2", "--warmup", "1", "--timeslots", "2",
              "--no-cpu-baseline", "--no-weak"]
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    one = _run([sys.executable, "bench.py", "--gpus", "1", "--dump",
                str(tmp_path / "one")] + common, env)
    env2 = dict(env, IDG_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    if launcher == "plain":
        cmd = [sys.executable, "bench.py"]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
               "--master-port", str(_port()), "bench.py"]
    two = _run(cmd + ["--gpus", "2", "--dump", str(tmp_path / "two")] +
               common, env2)
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert two["scaling"] == "strong"
    assert two["config"]["nr_subgrids_per_gpu"] == [1225, 1225]
    assert two["config"]["visibilities_per_step"] == \
        one["config"]["visibilities_per_step"]
    got = {}
    for tag in ("one", "two"):
        d = tmp_path / tag
        got[tag] = {k: np.load(d / (k + ".npy"))
                    for k in ("subgrids", "visibilities", "grid")}
    assert got["one"]["subgrids"].shape[0] == 2450
    assert np.array_equal(got["one"]["subgrids"], got["two"]["subgrids"])
    assert np.array_equal(got["one"]["visibilities"],
                          got["two"]["visibilities"])
    g1, g2 = got["one"]["grid"], got["two"]["grid"]
    assert np.abs(g2 - g1).max() <= 1e-6 * np.abs(g1).max()


@pytest.mark.timeout(600)
def test_bench_collectives_over_rccl_single_rank(tmp_path):
    """The RCCL side of the same path on the box's one device: bench.py runs
    inside an "nccl" (RCCL) process group of world size 1, so its barrier
    (device_ids), max/sum over ranks on device tensors, the uv-grid
    all-reduce and the output gathers all go through RCCL.  Outputs must equal
    the run without a process group bit for bit (a one-rank all-reduce is the
    identity).  The 8-GPU run differs only in the world size."""
    common = ["--gpus", "1", "--steps", "2", "--warmup", "1", "--timeslots",
              "2", "--no-cpu-baseline"]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    plain = _run([sys.executable, "bench.py", "--dump", str(tmp_path / "plain")]
                 + common, env)
    code = ("import sys, torch, torch.distributed as d\n"
            "torch.cuda.set_device(0)\n"
            f"d.init_process_group('nccl', init_method='tcp://127.0.0.1:{_port()}',"
            " rank=0, world_size=1, device_id=torch.device('cuda', 0))\n"
            "assert d.get_backend() == 'nccl'\n"
            "sys.path.insert(0, '.')\n"
            "import bench\n"
            "bench.main(sys.argv[1:])\n")
    rccl = _run([sys.executable, "-c", code, "--dump", str(tmp_path / "rccl")]
                + common, env)
    assert rccl["n_gpus"] == 1 and rccl["value"] > 0
    for k in ("subgrids", "visibilities", "grid"):
        a = np.load(tmp_path / "plain" / (k + ".npy"))
        b = np.load(tmp_path / "rccl" / (k + ".npy"))
        assert np.array_equal(a, b), k
