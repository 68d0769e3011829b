#!/bin/bash
# Round 4: the c256 workload profiled like configs[1]:
# kernel trace + FETCH/WRITE passes + SQ passes (profile_round.sh,
# pmc_sq.sh), then one bench line with its cpu_baseline.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r04wl_c256
mkdir -p $out
bash tests/debug/session.sh $out/p profile=r04c256,--workload,c256 || exit 1
timeout -k 10 900 python bench.py --workload c256 --steps 3 > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$out/bench.json')); k=d['kernels']; print('c256', d['value'], k['gridder']['ms'], k['degridder']['ms'], d.get('cpu_baseline'))"
