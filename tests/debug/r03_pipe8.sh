#!/bin/bash
# Round 3: adder loads predicated on the lane being inside the entry's
# subgrid -- pipeline tests, then the pipeline A/B (masked vs unmasked).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pp.txt 2>&1 || { tail -30 gpurun_out/pp.txt; exit 1; }
tail -1 gpurun_out/pp.txt
bash tests/debug/ab_pipe.sh ab/nomask.so ab/mask.so
echo done
