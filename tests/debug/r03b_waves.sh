#!/bin/bash
# Gridder launch bound A/B: IDG_GRID_WAVES 4 (shipped; the combined kernel
# spills 92 B/lane), 3 and 2 (no spills, one 512-lane workgroup per CU), on
# the all-general wterm batch and a 3,675-subgrid default batch (both take
# the combined kernel).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
BENCH_ARGS="--workload wterm" STEPS=10 bash tests/debug/ab.sh ab/base.so ab/w3.so ab/w2.so
BENCH_ARGS="--timeslots 3" STEPS=50 bash tests/debug/ab.sh ab/base.so ab/w3.so ab/w2.so
echo all done
