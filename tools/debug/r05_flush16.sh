#!/bin/bash
# Round 5: the 16-fill flush default, validated: the accuracy suite, the
# configs[2] full batch and sampled large configs, then configs[2]'s
# (NR_TIMESLOTS = 4) kernel trace and HBM counters.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_flush16; mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
  tests/test_gpu_accuracy.py tests/test_gpu.py -k "accuracy or configs2 or large_configs or fill_scale or c256 or closer" \
  > $out/tests.txt 2>&1
BENCH_ARGS="--workload c256 --timeslots 4" timeout -k 10 400 bash tools/probes/profile_round.sh r05_c256f16 > $out/prof_c256.log 2>&1
echo done
