#!/bin/bash
# Round 6: the N = 8 fixed cost.  The shard rehearsal (first and last rank of
# N = 1, 2, 4, 8) and the per-launch times at 3,062 .. 24,500 subgrids in the
# combined and the two-kernel form, same box:
#   bash tools/debug/r06_n8.sh TAG [LIB...]
# Output under gpurun_out/r06_n8_TAG/.  Every GPU step has its own limit; the
# first failure ends the call.
set -eo pipefail
tag=${1:-a}
shift || true
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r06_n8_$tag
mkdir -p $out
libs=${*:-ska-sdp-idg-bench_amd/libidg_mi355x.so}
for lib in $libs; do
  n=$(basename $lib .so)
  IDG_MI355X_LIB=$PWD/$lib timeout -k 10 300 python tools/debug/shard_rate.py \
    > $out/shard_$n.txt 2> $out/shard_$n.err
  for form in combined split; do
    IDG_MI355X_LIB=$PWD/$lib IDG_KERNEL_FORM=$form timeout -k 10 300 \
      python tools/debug/shard_rate.py --counts 1531,3062,6125,12250,24500 \
      > $out/counts_${n}_$form.txt 2> $out/counts_${n}_$form.err
  done
done
echo "r06_n8 $tag done"
