#!/bin/bash
# The degridder's subgrid pulled into L2 beside the eligibility check's uvw
# loads (deg) against HEAD (base): degridder tests on it, timing at 24,500
# subgrids (bench) and 512 / 3,063 / 6,125 (shard_rate --counts), interleaved.
# Then the closing steps on the in-tree library (= deg): GPU suite, smoke,
# bench line, default counters, shard rehearsal (r04_final2.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r04m
bash tests/debug/session.sh $out \
  'suite@ab/deg.so=degridder and not harness and not perf_mode' \
  ab=ab/base.so,ab/deg.so || exit 1
for rep in 1 2; do
  for lib in base deg; do
    IDG_MI355X_LIB=$PWD/ab/$lib.so timeout -k 10 300 python -u tests/debug/shard_rate.py \
      --steps 20 --counts 512,3063,6125 > $out/counts_${lib}_$rep.txt 2>&1 || exit 1
    echo "$lib $rep"; grep nr_subgrids $out/counts_${lib}_$rep.txt
  done
done
bash profiles/r04/scripts/r04_final2.sh
