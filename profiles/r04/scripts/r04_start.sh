#!/bin/bash
# Round-4 opening call: MFMA accumulation probe, gridder accuracy split
# (MFMA and all-VALU bodies), and the round-2 tree against HEAD on one box
# (interleaved A B B A, each tree's own bench.py and library).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r04start
mkdir -p $out
timeout -k 10 120 tests/probes/mfma_acc_probe > $out/mfma_acc_probe.txt 2>&1 || exit 1
cat $out/mfma_acc_probe.txt
timeout -k 10 300 python -u tests/debug/accuracy_ab.py mfma > $out/accuracy.jsonl 2> $out/accuracy.err || { tail -5 $out/accuracy.err; exit 1; }
IDG_GRIDDER_IMPL=valu timeout -k 10 300 python -u tests/debug/accuracy_ab.py valu >> $out/accuracy.jsonl 2>> $out/accuracy.err || { tail -5 $out/accuracy.err; exit 1; }
cat $out/accuracy.jsonl
run() {  # run <tag> <tree>
  (cd $2 && timeout -k 10 240 python bench.py --no-cpu-baseline --no-pipeline --steps 20) > $out/ab_$1_$3.json 2> $out/ab_$1_$3.err || { tail -5 $out/ab_$1_$3.err; exit 1; }
  python -c "
import json; d=json.load(open('$out/ab_$1_$3.json')); k=d['kernels']; print('$1', '$3', d['value'], k['gridder']['ms'], k['degridder']['ms'])"
}
run r02 ab/r02tree 1 && run head . 1 && run head . 2 && run r02 ab/r02tree 2 &&
run r02 ab/r02tree 3 && run head . 3 && run head . 4 && run r02 ab/r02tree 4
