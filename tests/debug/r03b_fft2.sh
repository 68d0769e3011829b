#!/bin/bash
# Split FFT transforms (fft.hpp fft2_planes_lds_parts): bitwise tests of the
# shipped build, then A/B: base (gridder epilogue 4 threads per transform),
# gp1 (1 thread per transform), st512 (splitter + FFT on 512-thread groups).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r03d
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_gpu_pipeline.py -m gpu -x -v --timeout 300 --timeout-method thread -k "fft or splitter or pipeline" > $out/pytest_fft.txt 2>&1 || { echo "pytest rc=$?"; grep -E "FAIL|Error" $out/pytest_fft.txt | tail -20; exit 1; }
grep -E "passed|failed" $out/pytest_fft.txt | tail -1
IDG_MI355X_LIB=$PWD/ab/st512.so timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -m gpu -x -q --timeout 120 --timeout-method thread -k "splitter_fft" > $out/pytest_st512.txt 2>&1 || { echo "st512 pytest rc=$?"; tail -20 $out/pytest_st512.txt; exit 1; }
grep -E "passed|failed" $out/pytest_st512.txt | tail -1
bash tests/debug/ab_pipe.sh ab/base.so ab/gp1.so ab/st512.so
echo all done
