#!/bin/bash
# The band adder (kernel_adder_band32, measured 3.2x slower and removed;
# DESIGN.md §11): pipeline GPU tests on the band build (ab/band.so, built
# from that kernel), then pipeline timings of it against the shipped one.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r03g
mkdir -p $out
IDG_MI355X_LIB=$PWD/ab/band.so timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest_band.txt 2>&1 || { echo "pytest rc=$?"; grep -E "FAIL|Error|assert" $out/pytest_band.txt | tail -20; exit 1; }
grep -E "passed|failed" $out/pytest_band.txt | tail -1
cp ska-sdp-idg-bench_amd/libidg_mi355x.so ab/shipped.so
STEPS=10 bash tests/debug/ab_pipe.sh ab/band.so ab/shipped.so
echo all done
