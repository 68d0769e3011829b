#!/bin/bash
# Round 4: the C = 256 gridder's blocked summation priced -- bench c256 with
# flush every 4 fills (the default), 8 and 16 (ab/flushN.so builds) and with
# no flush (IDG_PREC=4), interleaved; accuracy of each; then the c256 bench
# line with its cpu_baseline.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r04c256b
mkdir -p $out
run() {  # tag lib prec
  local e=(IDG_MI355X_LIB=$PWD/$2); [ -n "$3" ] && e+=(IDG_PREC=$3)
  env "${e[@]}" timeout -k 10 400 python bench.py --workload c256 --no-cpu-baseline --no-pipeline --steps 3 > $out/$1.json 2> $out/$1.err || { tail -5 $out/$1.err; return 1; }
  python -c "
import json; d=json.load(open('$out/$1.json')); k=d['kernels']; print('$1', d['value'], k['gridder']['ms'], k['degridder']['ms'])"
}
run f4_1 ab/flush4.so && run f8_1 ab/flush8.so && run nf_1 ab/flush4.so 4 &&
  run f16_1 ab/flush16.so && run f4_2 ab/flush4.so || exit 1
for l in flush4 flush8 flush16; do
  IDG_MI355X_LIB=$PWD/ab/$l.so timeout -k 10 300 python -u tests/debug/accuracy_ab.py $l >> $out/accuracy.jsonl 2>> $out/accuracy.err || { tail -5 $out/accuracy.err; exit 1; }
done
grep c256 $out/accuracy.jsonl | grep gridder
timeout -k 10 900 python bench.py --workload c256 --steps 3 > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$out/bench.json')); k=d['kernels']; print('c256', d['value'], k['gridder']['ms'], k['degridder']['ms'], d.get('cpu_baseline',{}).get('value'))"
