#!/bin/bash
# Profiles the default bench workload on the GPU box: kernel trace + stats,
# then FETCH_SIZE and WRITE_SIZE in separate PMC passes (never combined with
# trace domains).  Output under gpurun_out/prof_<tag>/.
set -eo pipefail
tag=${1:-r01}
out=$GRAFT_REPO_ROOT/gpurun_out/prof_$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/ktrace" -o run -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" ${BENCH_ARGS:-} --steps 10 --warmup 3 --no-cpu-baseline --no-side > "$out/bench_ktrace.json"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$out/fetch" -o run -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" ${BENCH_ARGS:-} --steps 2 --warmup 1 --min-warmup-s 0 --no-cpu-baseline --no-side > /dev/null
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$out/write" -o run -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" ${BENCH_ARGS:-} --steps 2 --warmup 1 --min-warmup-s 0 --no-cpu-baseline --no-side > /dev/null
echo done
