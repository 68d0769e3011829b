#!/bin/bash
# Round 6: the persistent S = 32 mirror gridder (-DIDG_GRID_PERSIST=1)
# against the one-workgroup-per-subgrid mirror kernel, both in the
# two-kernel form (IDG_KERNEL_FORM=split), same box:
#   bash tools/debug/r06_persist_ab.sh BASE_LIB PERSIST_LIB
# 1. outputs of both on the lib_outputs batches, compared bit for bit;
# 2. per-launch times at 3,062 (an N = 8 shard) .. 24,500 subgrids, two
#    interleaved reps.  Output under gpurun_out/r06_persist/.  Every GPU
# step has its own limit; the first failure ends the call.
set -eo pipefail
base=${1:?base lib}
new=${2:?persistent lib}
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r06_persist
mkdir -p $out
for lib in $base $new; do
  n=$(basename $lib .so)
  IDG_MI355X_LIB=$PWD/$lib IDG_KERNEL_FORM=split timeout -k 10 300 \
    python tools/debug/lib_outputs.py $out/out_$n.npz > $out/out_$n.log 2>&1
done
python tools/debug/lib_outputs.py --compare $out/out_$(basename $base .so).npz \
  $out/out_$(basename $new .so).npz | tee $out/compare.txt
for rep in 1 2; do
  for lib in $base $new; do
    n=$(basename $lib .so)
    IDG_MI355X_LIB=$PWD/$lib IDG_KERNEL_FORM=split timeout -k 10 300 \
      python tools/debug/shard_rate.py --counts 3062,6125,24500 \
      > $out/counts_${n}_$rep.txt 2> $out/counts_${n}_$rep.err
    sed "s/^/$n rep$rep /" $out/counts_${n}_$rep.txt
  done
done
echo "r06_persist done"
