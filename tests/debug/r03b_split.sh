#!/bin/bash
# Fused splitter + FFT variants: the bitwise pipeline tests on the shipped
# build, then A/B of the persistent kernel with and without the window
# prefetch (pipeline timings of bench.py).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03b
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r03b/pytest_pipe.txt 2>&1 || { echo "pytest rc=$?"; grep -E "FAIL|Error" gpurun_out/r03b/pytest_pipe.txt | tail -20; exit 1; }
grep -E "passed|failed" gpurun_out/r03b/pytest_pipe.txt | tail -1
bash tests/debug/ab_pipe.sh ab/pf.so ab/nopf.so
