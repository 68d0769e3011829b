#!/bin/bash
# The gridder's prologue merged (the mirror check's uvw loads and the first
# fill's max-|V| scan in one pass, one barrier): gridder tests on it, then
# timing against HEAD at 24,500 subgrids (bench) and at 512 / 3,063 / 6,125
# (shard_rate --counts: the combined kernel of the N >= 4 shards), interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r04l
bash tests/debug/session.sh $out \
  'suite@ab/pro.so=gridder and not harness and not perf_mode' \
  ab=ab/base.so,ab/pro.so || exit 1
for rep in 1 2; do
  for lib in base pro; do
    IDG_MI355X_LIB=$PWD/ab/$lib.so timeout -k 10 300 python -u tests/debug/shard_rate.py \
      --steps 20 --counts 512,3063,6125 > $out/counts_${lib}_$rep.txt 2>&1 || exit 1
    echo "$lib $rep"; grep nr_subgrids $out/counts_${lib}_$rep.txt
  done
done
