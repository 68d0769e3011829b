#!/bin/bash
# Round 4: the B operand's f16 scale raised high in the range (ab/bs13.so:
# gridder first-fill maximum below 2^12, degridder below 2^13, so the
# split's lo parts stay normal f16) against the shipped scale (ab/bs0.so):
# accuracy of each, then default-workload timing interleaved; then the s64
# workload (configs[4]) profiled and its bench line with the cpu_baseline.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r04f
mkdir -p $out
for l in bs0 bs13; do
  IDG_MI355X_LIB=$PWD/ab/$l.so timeout -k 10 300 python -u tests/debug/accuracy_ab.py $l >> $out/accuracy.jsonl 2>> $out/accuracy.err || { tail -5 $out/accuracy.err; exit 1; }
done
cat $out/accuracy.jsonl | cut -c1-220
bash tests/debug/session.sh $out/ab ab=ab/bs0.so,ab/bs13.so 'suite@ab/bs13.so=gridder or degridder' || exit 1
bash profiles/r04/scripts/r04_wl_s64.sh
