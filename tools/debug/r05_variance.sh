#!/bin/bash
# Round 5: run-to-run spread of the default line on one box (five runs of
# the timed step, no side legs), for reading same-box A/Bs against noise.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_var; mkdir -p $out
for i in 1 2 3 4 5; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-side --no-pipeline --steps 20 > $out/run_$i.json 2> $out/run_$i.err
  python -c "import json; d=json.load(open('$out/run_$i.json')); print($i, d['value'], d['kernels']['gridder']['ms'], d['kernels']['degridder']['ms'], d.get('energy',{}).get('joules_per_step'))" >> $out/summary.txt
done
echo done
