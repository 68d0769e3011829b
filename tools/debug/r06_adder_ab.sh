#!/bin/bash
# Round 6: the adder with the crowded-tile pass folded into the home sort's
# place kernel and the tile rows dealt over the XCDs by r % 8, against the
# round-6 base, same box:
#   bash tools/debug/r06_adder_ab.sh BASE_LIB NEW_LIB
# 1. the pipeline GPU tests on NEW_LIB; 2. pipeline step times, both
# libraries, two interleaved reps (tools/debug/ab_pipe.sh); 3. the crowded
# layouts (tools/debug/adder_crowded.py), both libraries.
# Output under gpurun_out/r06_adder/.  Every GPU step has its own limit; the
# first failure ends the call.
set -eo pipefail
base=${1:?base lib}
new=${2:?new lib}
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r06_adder
mkdir -p $out
IDG_MI355X_LIB=$PWD/$new timeout -k 10 600 python -u -m pytest \
  tests/test_gpu_pipeline.py -x -v --timeout 300 --timeout-method thread \
  > $out/tests.log 2>&1
tail -1 $out/tests.log
timeout -k 10 900 bash tools/debug/ab_pipe.sh $base $new | tee $out/ab_pipe.txt
for lib in $base $new; do
  n=$(basename $lib .so)
  IDG_MI355X_LIB=$PWD/$lib timeout -k 10 300 python tools/debug/adder_crowded.py \
    > $out/crowded_$n.txt 2> $out/crowded_$n.err
  sed "s/^/$n /" $out/crowded_$n.txt
done
echo "r06_adder done"
