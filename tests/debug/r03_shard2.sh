#!/bin/bash
# Round 3: combined kernels below 8,192 subgrids -- mixed-batch and
# two-kernel tests, then the one-GPU shard rehearsal.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r03shard2
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -m gpu -q --timeout 300 --timeout-method thread -k "mixed or two_kernel or empty or small" > $out/pytest_gpu.txt 2>&1 || { echo "pytest rc=$?"; tail -30 $out/pytest_gpu.txt; exit 1; }
tail -1 $out/pytest_gpu.txt
timeout -k 10 400 python -u tests/debug/shard_rate.py --steps 10 > $out/shard_rate.txt 2>&1 || { tail -20 $out/shard_rate.txt; exit 1; }
grep predicted $out/shard_rate.txt
grep '"world": 8, "rank"' $out/shard_rate.txt
echo done
