#!/bin/bash
# Round 3: the LDS home sort up to 36,864 keys (w-layer batches) --
# pipeline tests, then the wterm pipeline A/B against the previous build.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pp.txt 2>&1 || { tail -30 gpurun_out/pp.txt; exit 1; }
tail -1 gpurun_out/pp.txt
BENCH_ARGS="--workload wterm" bash tests/debug/ab_pipe.sh ab/old.so ab/new.so
bash tests/debug/ab_pipe.sh ab/old.so ab/new.so
echo done
