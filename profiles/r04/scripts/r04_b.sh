#!/bin/bash
# Round 4, second GPU call: suite on this tree; the gridder's distance to
# exact accumulation per precision option (IDG_PREC 0 / 1 / 3 / 4 / 5 / 6:
# none, tail, tail + flush, alternating tail, alternating gridder tail +
# degridder tail, alternating + flush) and the default-workload timing of
# 0 / 1 / 4 / 5 (interleaved, two reps); the one-GPU shard rehearsal in the default, split and combined
# launch forms (the combined gridder is spill-free since the general path's
# geometry moved to LDS); the wterm workload's kernel trace + counters.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r04b
mkdir -p $out
bash tests/debug/session.sh $out/s suite  # a failing test does not end the call
for pr in 0 1 3 4 5 6; do
  IDG_PREC=$pr timeout -k 10 300 python -u tests/debug/accuracy_ab.py >> $out/accuracy.jsonl 2>> $out/accuracy.err || { tail -5 $out/accuracy.err; exit 1; }
done
cat $out/accuracy.jsonl
for rep in 1 2; do
for pr in 0 1 4 5; do
  IDG_PREC=$pr timeout -k 10 240 python bench.py --no-cpu-baseline --no-pipeline --steps 20 > $out/d_$pr.$rep.json 2> $out/d_$pr.$rep.err || { tail -5 $out/d_$pr.$rep.err; exit 1; }
  python -c "
import json; d=json.load(open('$out/d_$pr.$rep.json')); k=d['kernels']; print('default IDG_PREC=$pr', d['value'], k['gridder']['ms'], k['degridder']['ms'])"
done
done
for form in default split combined; do
  e=(); [ $form != default ] && e=(IDG_KERNEL_FORM=$form)
  env "${e[@]}" timeout -k 10 600 python -u tests/debug/shard_rate.py --steps 10 > $out/shard_$form.txt 2>&1 || { tail -5 $out/shard_$form.txt; exit 1; }
  echo "shard $form"; grep -E "predicted|N=" $out/shard_$form.txt | tail -6
done
bash tests/debug/session.sh $out/p profile=r04wterm,--workload,wterm
