#!/bin/bash
# One-GPU strong-scaling rehearsal of the final tree (tests/debug/shard_rate.py).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03h
timeout -k 10 600 python -u tests/debug/shard_rate.py --steps 20 > gpurun_out/r03h/shard_rate.txt 2>&1 || { tail -20 gpurun_out/r03h/shard_rate.txt; exit 1; }
cat gpurun_out/r03h/shard_rate.txt
