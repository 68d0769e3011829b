#!/bin/bash
# Round 5: configs[4] (S = 64) A/B of the round-4 forms (ab/s64base.so:
# IDG_GRID_SPLIT64=0, IDG_DEGRID_KP64=512) against the round-5 defaults
# (ab/s64new.so: the gridder's four passes on four workgroups, the
# degridder's mirror kernel on 8 waves with 1,024-pair chunks).  Timing
# interleaved, two reps (tools/debug/ab.sh), then FETCH_SIZE / WRITE_SIZE of
# each in separate passes.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_s64ab; mkdir -p $out
BENCH_ARGS="--workload s64" STEPS=10 bash tools/debug/ab.sh ab/s64base.so ab/s64new.so > $out/ab_s64.txt
cd /tmp && export TMPDIR=/tmp
for lib in s64base s64new; do
  for c in FETCH_SIZE WRITE_SIZE; do
    IDG_MI355X_LIB=$GRAFT_REPO_ROOT/ab/$lib.so timeout -s KILL 200 rocprofv3 --pmc $c -d $GRAFT_REPO_ROOT/$out/${lib}_$c -o run -- \
      python3 $GRAFT_REPO_ROOT/bench.py --workload s64 --steps 2 --warmup 1 --min-warmup-s 0 \
      --no-cpu-baseline --no-side --no-pipeline > /dev/null 2> $GRAFT_REPO_ROOT/$out/${lib}_$c.err
  done
done
echo done
