#!/bin/bash
# Paired 16-byte FFT output stores (fft.hpp store_columns; measured no
# faster, removed): the FFT /
# pipeline / gridder-FFT GPU tests on the shipped build, then pipeline A/B
# against one 8-byte store per value (IDG_FFT_PAIR_STORE=0).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r03j
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_gpu_pipeline.py -m gpu -x -v --timeout 300 --timeout-method thread -k "fft or splitter or pipeline or adder" > $out/pytest_pair.txt 2>&1 || { echo "pytest rc=$?"; grep -E "FAIL|Error|assert" $out/pytest_pair.txt | tail -20; exit 1; }
grep -E "passed|failed" $out/pytest_pair.txt | tail -1
STEPS=10 bash tests/debug/ab_pipe.sh ab/pair.so ab/nopair.so
echo all done
