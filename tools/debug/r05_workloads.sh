#!/bin/bash
# Round 5: the configs[2] (C = 256) and configs[4] (S = 64) bench lines on the
# closing kernels (profiles/r05/workloads/).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_workloads; mkdir -p $out
timeout -k 10 500 python bench.py --workload c256 --steps 5 --no-cpu-baseline --no-side > $out/c256.json 2> $out/c256.err
timeout -k 10 400 python bench.py --workload s64 --steps 5 --no-cpu-baseline --no-side > $out/s64.json 2> $out/s64.err
echo done
