#!/bin/bash
# Tuning round: MFMA-vs-VALU parity of the current library (w = 0, w-terms),
# the GPU suite, then A/B timing of the given library variants.
#   bash tests/debug/check_ab.sh ab/old.so ab/new.so
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 python tests/debug/diff_impl.py 2>&1 | grep -v "^  s" || exit 1
DIFF_W=1 timeout -k 10 200 python tests/debug/diff_impl.py 2>&1 | grep -v "^  s" || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1 || { tail -30 gpurun_out/pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/pytest_gpu.txt
[ $# -gt 0 ] && bash tests/debug/ab.sh "$@"
