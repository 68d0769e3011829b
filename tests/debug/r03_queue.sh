#!/bin/bash
# Two-kernel form with the general queue: GPU parity subset, then A/B against
# the combined kernel on the wterm and default workloads.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/queue
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/queue/pytest.txt 2>&1 || { tail -30 gpurun_out/queue/pytest.txt; exit 1; }
tail -1 gpurun_out/queue/pytest.txt
BENCH_ARGS="--workload wterm" STEPS=10 bash tests/debug/ab.sh ab/new.so ab/nosplit.so
bash tests/debug/ab.sh ab/new.so ab/nosplit.so
echo done
