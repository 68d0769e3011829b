#!/bin/bash
# Round 4: the s64 workload profiled like configs[1]:
# kernel trace + FETCH/WRITE passes + SQ passes (profile_round.sh,
# pmc_sq.sh), then one bench line with its cpu_baseline.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r04wl_s64
mkdir -p $out
bash tests/debug/session.sh $out/p profile=r04s64,--workload,s64 || exit 1
timeout -k 10 900 python bench.py --workload s64 --steps 3 > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$out/bench.json')); k=d['kernels']; print('s64', d['value'], k['gridder']['ms'], k['degridder']['ms'], d.get('cpu_baseline'))"
