#!/bin/bash
# Round 5: the degridder (and the other TUs) scheduled with
# -amdgpu-sched-strategy=max-ilp (ab/dg_ilp.so; the gridder has it already)
# against the shipped build (ab/base.so): outputs bit for bit, then the
# default timing, interleaved, two reps.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_sched; mkdir -p $out
for lib in base dg_ilp; do
  IDG_MI355X_LIB=$PWD/ab/$lib.so timeout -k 10 300 python tools/debug/lib_outputs.py $out/$lib.npz > $out/out_$lib.txt 2>&1
done
python tools/debug/lib_outputs.py --compare $out/base.npz $out/dg_ilp.npz > $out/compare.txt 2>&1 || true
rm -f $out/*.npz
bash tools/debug/ab.sh ab/base.so ab/dg_ilp.so > $out/ab_default.txt
echo done
