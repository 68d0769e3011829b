#!/bin/bash
# Round 5: configs[4] on the closing kernels: the bench line, then the
# kernel trace and HBM counters (profiles/r05/kernels_s64, traffic.json).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_s64f; mkdir -p $out
timeout -k 10 400 python bench.py --workload s64 --steps 5 --no-cpu-baseline --no-side > $out/s64.json 2> $out/s64.err
BENCH_ARGS="--workload s64" timeout -k 10 400 bash tools/probes/profile_round.sh r05_s64cs > $out/prof.log 2>&1
echo done
