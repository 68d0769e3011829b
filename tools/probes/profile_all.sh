#!/bin/bash
# One GPU call's worth of profiling for a round (output under gpurun_out/):
# the default bench workload (kernel trace + FETCH/WRITE + SQ passes), the
# wterm workload (the same), and the traffic-probe calibration passes.
#   bash tools/probes/profile_all.sh TAG
set -eo pipefail
tag=${1:-r02}
cd "$GRAFT_REPO_ROOT"
bash tools/probes/profile_round.sh "$tag"
bash tools/probes/pmc_sq.sh "$tag"
BENCH_ARGS="--workload wterm" bash tools/probes/profile_round.sh "${tag}_wterm"
BENCH_ARGS="--workload wterm" bash tools/probes/pmc_sq.sh "${tag}_wterm"
out=$GRAFT_REPO_ROOT/gpurun_out/calib_$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d "$out/$c" -o run -- \
    "$GRAFT_REPO_ROOT/tools/probes/traffic_probe" > "$out/$c.log" 2>&1
done
echo profile_all done
