#!/bin/bash
# Round 5: the gridder's full fills by LDS-DMA (IDG_GRID_DMA_FILL=1, ab/dma1.so)
# against the per-K-step loads (ab/dma0.so): outputs bit for bit, then the
# default and configs[2] (NR_TIMESLOTS=4) timings, interleaved, two reps.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_dma; mkdir -p $out
for lib in dma0 dma1; do
  IDG_MI355X_LIB=$PWD/ab/$lib.so timeout -k 10 300 python tools/debug/lib_outputs.py $out/$lib.npz > $out/out_$lib.txt 2>&1
done
python tools/debug/lib_outputs.py --compare $out/dma0.npz $out/dma1.npz > $out/compare.txt 2>&1 || true
rm -f $out/*.npz
bash tools/debug/ab.sh ab/dma0.so ab/dma1.so > $out/ab_default.txt
BENCH_ARGS="--workload c256 --timeslots 4" STEPS=5 bash tools/debug/ab.sh ab/dma0.so ab/dma1.so > $out/ab_c256.txt
echo done
