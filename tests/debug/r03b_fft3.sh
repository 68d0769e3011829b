#!/bin/bash
# The simplified FFT kernels: bitwise FFT / pipeline tests, then the
# pipeline timings twice (interleaved gridder + FFT vs gridder_fft).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r03e
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_gpu_pipeline.py -m gpu -x -v --timeout 300 --timeout-method thread -k "fft or splitter or pipeline" > $out/pytest_fft.txt 2>&1 || { echo "pytest rc=$?"; grep -E "FAIL|Error" $out/pytest_fft.txt | tail -20; exit 1; }
grep -E "passed|failed" $out/pytest_fft.txt | tail -1
STEPS=10 bash tests/debug/ab_pipe.sh ab/base.so
echo all done
