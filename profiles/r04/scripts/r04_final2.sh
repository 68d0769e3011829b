#!/bin/bash
# Round 4 closing call (re-run after the staged-fill experiment was removed): GPU suite, smoke, the default bench line (cpu
# baseline, pipeline), and the default workload's kernel trace + FETCH/WRITE
# + SQ passes (profiles/traffic.json for the bench's roofline).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r04final2
mkdir -p $out
bash tests/debug/session.sh $out/s suite smoke  # a failing test does not end the call
timeout -k 10 600 python bench.py > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$out/bench.json')); k=d['kernels']; r=d['roofline']
print('default', d['value'], k['gridder']['ms'], k['degridder']['ms'], r.get('frac'), r.get('issue_efficiency',{}).get('frac'), (d.get('cpu_baseline') or {}).get('value'), d['pipeline']['full_cycle_fused_mvis_s'])"
bash tests/debug/session.sh $out/p profile=r04final2
timeout -k 10 400 python -u tests/debug/shard_rate.py --steps 10 > $out/shard_default.txt 2> $out/shard.err || { tail -5 $out/shard.err; exit 1; }
grep predicted $out/shard_default.txt
