#!/bin/bash
# The lean splitter + FFT (kernel_splitter_fft32_lean: 32 KB LDS, 5 units
# per CU; measured no faster and removed): bitwise
# pipeline tests on that build (ab/lean.so), then pipeline A/B against the
# shipped (persistent) kernel.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r03i
mkdir -p $out
IDG_MI355X_LIB=$PWD/ab/lean.so timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest_lean.txt 2>&1 || { echo "pytest rc=$?"; grep -E "FAIL|Error|assert" $out/pytest_lean.txt | tail -20; exit 1; }
grep -E "passed|failed" $out/pytest_lean.txt | tail -1
STEPS=10 bash tests/debug/ab_pipe.sh ab/lean.so ab/shipped.so
echo all done
