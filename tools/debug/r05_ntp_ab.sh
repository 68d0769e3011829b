#!/bin/bash
# Round 5: non-temporal L2 prefetch DMA (IDG_GRID_NT_PREFETCH), alone and with
# the non-temporal fill loads (IDG_GRID_NT_FILL), A/B.  Timing of both
# libraries on the default batch and on configs[2] at NR_TIMESLOTS=4 (same
# box, interleaved, two reps: tools/debug/ab.sh), then the HBM counters
# (FETCH_SIZE, WRITE_SIZE in separate passes) of the c256 gridder under each.
# (IDG_GRID_NT_PREFETCH was removed after this A/B, profiles/r05/nt/ntp_*.)
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_ntp; mkdir -p $out
bash tools/debug/ab.sh ab/ntp0.so ab/ntp1.so ab/ntfp1.so > $out/ab_default.txt
BENCH_ARGS="--workload c256 --timeslots 4" STEPS=5 bash tools/debug/ab.sh ab/ntp0.so ab/ntp1.so ab/ntfp1.so > $out/ab_c256.txt
cd /tmp && export TMPDIR=/tmp
for lib in ntp0 ntp1 ntfp1; do
  for c in FETCH_SIZE WRITE_SIZE; do
    IDG_MI355X_LIB=$GRAFT_REPO_ROOT/ab/$lib.so timeout -s KILL 200 rocprofv3 --pmc $c -d $GRAFT_REPO_ROOT/$out/${lib}_$c -o run -- \
      python3 $GRAFT_REPO_ROOT/bench.py --workload c256 --timeslots 4 --steps 2 --warmup 1 --min-warmup-s 0 \
      --no-cpu-baseline --no-side --no-pipeline > /dev/null 2> $GRAFT_REPO_ROOT/$out/${lib}_$c.err
  done
done
echo done
