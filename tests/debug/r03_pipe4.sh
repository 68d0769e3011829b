#!/bin/bash
# Round 3: kernel traces of the pipeline steps, previous build against the
# home-sort build (bench.py, 3 timed steps each).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for lib in pold p16; do
  IDG_MI355X_LIB=$PWD/ab/$lib.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_$lib -o run -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/kt_$lib.log 2>&1 || { tail -20 gpurun_out/kt_$lib.log; exit 1; }
  echo "$lib ok"
done
echo done
