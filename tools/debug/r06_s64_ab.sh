#!/bin/bash
# Round 6: the S = 64 single-chunk mirror degridder (16 waves, 2,048 pairs
# in 160 KB of LDS) against the two-chunk form, same box:
#   bash tools/debug/r06_s64_ab.sh NEW_LIB BASE_LIB
# 1. the S = 64 GPU tests on NEW_LIB; 2. configs[4] bench, both libraries,
# two interleaved reps; 3. kernel trace + FETCH/WRITE passes of NEW_LIB.
# Output under gpurun_out/r06_s64/.  Every GPU step has its own limit; the
# first failure ends the call.
set -eo pipefail
new=${1:?new lib}
base=${2:?base lib}
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r06_s64
mkdir -p $out
IDG_MI355X_LIB=$PWD/$new timeout -k 10 900 python -u -m pytest tests -m gpu \
  -k "s64 or S64 or configs4 or 64" -x -v --timeout 600 --timeout-method thread \
  > $out/tests.log 2>&1
for rep in 1 2; do
  for lib in $base $new; do
    n=$(basename $lib .so)_$rep
    IDG_MI355X_LIB=$PWD/$lib timeout -k 10 300 python bench.py --workload s64 \
      --no-cpu-baseline --no-pipeline --no-side --no-weak --steps 10 \
      > $out/ab_$n.json 2> $out/ab_$n.err
    python -c "
import json; d=json.load(open('$out/ab_$n.json')); k=d['kernels']
print('$n', d['value'], k['gridder']['ms'], k['degridder']['ms'])" | tee -a $out/ab.txt
  done
done
IDG_MI355X_LIB=$PWD/$new BENCH_ARGS="--workload s64" timeout -k 10 600 \
  bash tools/probes/profile_round.sh r06_s64_single > $out/prof.log 2>&1
echo "r06_s64 done"
