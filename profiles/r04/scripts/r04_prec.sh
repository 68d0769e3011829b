#!/bin/bash
# Precision options of the MFMA kernels (IDG_PREC, util.hpp precision_for):
# GPU suite on the new build, gridder/degridder accuracy per option at the
# -c defaults and C = 256, then configs[1] and c256 timing per option
# (interleaved, two reps).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r04prec
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.txt 2>&1 || { echo "pytest failed"; tail -30 $out/pytest_gpu.txt; exit 1; }
tail -1 $out/pytest_gpu.txt
for pr in 0 1 3; do
  IDG_PREC=$pr timeout -k 10 300 python -u tests/debug/accuracy_ab.py >> $out/accuracy.jsonl 2>> $out/accuracy.err || { tail -5 $out/accuracy.err; exit 1; }
done
cat $out/accuracy.jsonl
for rep in 1 2; do
for pr in 0 1 3; do
  IDG_PREC=$pr timeout -k 10 240 python bench.py --no-cpu-baseline --no-pipeline --steps 20 > $out/d_$pr.$rep.json 2> $out/d_$pr.$rep.err || { tail -5 $out/d_$pr.$rep.err; exit 1; }
  python -c "
import json; d=json.load(open('$out/d_$pr.$rep.json')); k=d['kernels']; print('default IDG_PREC=$pr', d['value'], k['gridder']['ms'], k['degridder']['ms'])"
done
done
for rep in 1 2; do
for pr in 1 3; do
  IDG_PREC=$pr timeout -k 10 400 python bench.py --workload c256 --no-cpu-baseline --no-pipeline --steps 3 > $out/c_$pr.$rep.json 2> $out/c_$pr.$rep.err || { tail -5 $out/c_$pr.$rep.err; exit 1; }
  python -c "
import json; d=json.load(open('$out/c_$pr.$rep.json')); k=d['kernels']; print('c256 IDG_PREC=$pr', d['value'], k['gridder']['ms'], k['degridder']['ms'])"
done
done
