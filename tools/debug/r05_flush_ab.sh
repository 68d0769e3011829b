#!/bin/bash
# Round 5: the blocked summation's flush interval (IDG_FLUSH_FILLS 8, the
# default, against 16 and 32): accuracy against the exact sum
# (tools/debug/flush_ab.py), the c256 gridder's time (configs[2] at
# NR_TIMESLOTS=4, interleaved, two reps) and its HBM counters.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_flush; mkdir -p $out
for lib in flush8 flush16 flush32; do
  IDG_MI355X_LIB=$PWD/ab/$lib.so timeout -k 10 300 python tools/debug/flush_ab.py $lib >> $out/accuracy.txt 2> $out/acc_$lib.err
done
BENCH_ARGS="--workload c256 --timeslots 4" STEPS=5 bash tools/debug/ab.sh ab/flush8.so ab/flush16.so ab/flush32.so > $out/ab_c256.txt
cd /tmp && export TMPDIR=/tmp
for lib in flush8 flush16 flush32; do
  for c in FETCH_SIZE WRITE_SIZE; do
    IDG_MI355X_LIB=$GRAFT_REPO_ROOT/ab/$lib.so timeout -s KILL 200 rocprofv3 --pmc $c -d $GRAFT_REPO_ROOT/$out/${lib}_$c -o run -- \
      python3 $GRAFT_REPO_ROOT/bench.py --workload c256 --timeslots 4 --steps 2 --warmup 1 --min-warmup-s 0 \
      --no-cpu-baseline --no-side --no-pipeline > /dev/null 2> $GRAFT_REPO_ROOT/$out/${lib}_$c.err
  done
done
echo done
