#!/bin/bash
# Round 3: pipeline tests, then A/B: previous build, new (home sort, 16-byte
# splitter loads), 8-byte splitter loads, plain (not non-temporal) stores.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pp.txt 2>&1 || { tail -30 gpurun_out/pp.txt; exit 1; }
tail -1 gpurun_out/pp.txt
bash tests/debug/ab_pipe.sh ab/pold.so ab/p16.so ab/sx2.so ab/nt0.so
echo done
