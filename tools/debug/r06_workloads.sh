#!/bin/bash
# Round 6: full-size configs[2] (C = 256, 24,500 subgrids) on this round's
# kernels -- the default pair and the sequential gridder with the default
# degridder (the pair that passes the reference's metric there) -- and the
# configs[4] line (profiles/r06/workloads/).  Every GPU step has its own
# limit; the first failure ends the call.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r06_workloads; mkdir -p $out
timeout -k 10 500 python bench.py --workload c256 --steps 5 --no-cpu-baseline \
  --no-side > $out/c256.json 2> $out/c256.err
IDG_GRIDDER_IMPL=sequential timeout -k 10 500 python bench.py --workload c256 \
  --steps 2 --warmup 1 --min-warmup-s 0 --no-cpu-baseline --no-side \
  --no-pipeline --no-weak > $out/c256_seq_gridder.json 2> $out/c256_seq_gridder.err
timeout -k 10 400 python bench.py --workload s64 --steps 5 --no-cpu-baseline \
  --no-side > $out/s64.json 2> $out/s64.err
echo "r06_workloads done"
