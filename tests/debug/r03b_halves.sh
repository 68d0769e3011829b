#!/bin/bash
# The 256-thread splitter + FFT (kernel_splitter_fft32_halves, each
# transform split over two threads; measured slower and removed, DESIGN.md
# §8 item 5): pipeline GPU tests on the build that had it
# (that kernel), then pipeline A/B against the persistent 128-thread kernel
# (IDG_SPLIT_FFT_HALVES=0).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r03k
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest_halves.txt 2>&1 || { echo "pytest rc=$?"; grep -E "FAIL|Error|assert" $out/pytest_halves.txt | tail -20; exit 1; }
grep -E "passed|failed" $out/pytest_halves.txt | tail -1
STEPS=10 bash tests/debug/ab_pipe.sh ab/halves.so ab/pers.so
echo all done
