#!/bin/bash
# Round 5: the added parity cases (baseline offsets, image sizes, large grids).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05_newtests
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu.py tests/test_gpu_sequential.py -k "baseline_offsets or image_size or large_grid or non_finite or sweep or s64_degridder" \
  > gpurun_out/r05_newtests/tests.txt 2>&1
echo rc=$?
