#!/bin/bash
# L2 (TCC) hit / miss counts per kernel of one bench step (pipeline kernels
# included): one PMC pass, two TCC counters.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
out=$GRAFT_REPO_ROOT/gpurun_out/pmc_tcc
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$out/p1" -o run -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --steps 1 --warmup 1 --min-warmup-s 0 --no-cpu-baseline > /dev/null 2> "$out/p1.err"
echo done
