#!/bin/bash
# Round 3: full GPU suite on the home-sort pipeline build, then the one-GPU
# shard rehearsal (N = 1, 2, 4, 8 first/last rank shards).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r03shard
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $out/pytest_gpu.txt 2>&1 || { echo "pytest rc=$?"; tail -30 $out/pytest_gpu.txt; exit 1; }
tail -1 $out/pytest_gpu.txt
timeout -k 10 400 python -u tests/debug/shard_rate.py --steps 10 > $out/shard_rate.txt 2>&1 || { tail -20 $out/shard_rate.txt; exit 1; }
grep -v "^W2026\|^I2026" $out/shard_rate.txt | tail -20
echo done
