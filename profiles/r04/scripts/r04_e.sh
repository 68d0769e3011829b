#!/bin/bash
# Round 4: the precision defaults (gridder: tail on one channel per quad,
# blocked summation above 16 channels; degridder: no tail) -- GPU suite,
# smoke, the default bench line, and the default workload's kernel trace +
# FETCH/WRITE + SQ passes (profiles/traffic.json for the bench's roofline).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r04e
mkdir -p $out
bash tests/debug/session.sh $out/s suite smoke  # a failing test does not end the call
timeout -k 10 600 python bench.py > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$out/bench.json')); k=d['kernels']; print('default', d['value'], k['gridder']['ms'], k['degridder']['ms'], d['roofline'].get('frac'), (d.get('cpu_baseline') or {}).get('value'))"
bash tests/debug/session.sh $out/p profile=r04default
