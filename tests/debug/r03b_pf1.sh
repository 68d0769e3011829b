#!/bin/bash
# The persistent splitter + FFT with the next unit's window loaded behind
# the current transform, at one wave per SIMD (IDG_SPLIT_FFT_PREFETCH=1):
# pipeline GPU tests on that build, then pipeline A/B against the shipped one
# (measured slower and removed).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r03l
mkdir -p $out
IDG_MI355X_LIB=$PWD/ab/pf1.so timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -m gpu -x -v --timeout 120 --timeout-method thread -k "splitter or pipeline" > $out/pytest_pf1.txt 2>&1 || { echo "pytest rc=$?"; grep -E "FAIL|Error|assert" $out/pytest_pf1.txt | tail -20; exit 1; }
grep -E "passed|failed" $out/pytest_pf1.txt | tail -1
STEPS=10 bash tests/debug/ab_pipe.sh ab/pf1.so ab/shipped.so
echo all done
