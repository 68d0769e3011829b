#!/bin/bash
# Round 6: the default bench line after 1 s and after 5 s of untimed
# warm-up steps (--min-warmup-s), interleaved, two reps, same box.
# Output under gpurun_out/r06_warmup/.  Every GPU step has its own limit; the
# first failure ends the call.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r06_warmup
mkdir -p $out
for rep in 1 2; do
  for wu in 1 5; do
    timeout -k 10 300 python bench.py --steps 20 --min-warmup-s $wu --no-cpu-baseline \
      --no-pipeline --no-side --no-weak > $out/w${wu}_$rep.json 2> $out/w${wu}_$rep.err
    python -c "
import json; d=json.load(open('$out/w${wu}_$rep.json')); k=d['kernels']
print('warmup_s $wu rep $rep', d['value'], k['gridder']['ms'], k['degridder']['ms'], d.get('warmup_steps_run'))"
  done
done
echo "r06_warmup done"
