#!/bin/bash
# Round 5 closing GPU calls (output under gpurun_out/r05_final/):
#   part 1: the whole GPU suite, smoke, the default bench line;
#   part 2: the default workload's kernel trace, FETCH/WRITE and SQ passes
#           (profiles/traffic.json), configs[4]'s and configs[2]'s kernel
#           traces and HBM counters, and the one-GPU shard rehearsal.
# Every GPU step has its own limit; the first failure ends the call.
set -eo pipefail
part=${1:-1}
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_final
mkdir -p $out
if [ "$part" = 1 ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 \
    --timeout-method thread > $out/pytest_gpu.txt 2>&1
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1
  timeout -k 10 400 python bench.py > $out/bench.json 2> $out/bench.err
else
  timeout -k 10 400 bash tools/probes/profile_round.sh r05 > $out/prof.log 2>&1
  timeout -k 10 500 bash tools/probes/pmc_sq.sh r05 > $out/pmc.log 2>&1
  BENCH_ARGS="--workload s64" timeout -k 10 400 bash tools/probes/profile_round.sh r05_s64 > $out/prof_s64.log 2>&1
  BENCH_ARGS="--workload c256 --timeslots 4" timeout -k 10 400 bash tools/probes/profile_round.sh r05_c256 > $out/prof_c256.log 2>&1
  timeout -k 10 300 python tools/debug/shard_rate.py > $out/shard_default.txt 2> $out/shard.err
fi
echo "r05_final part $part done"
