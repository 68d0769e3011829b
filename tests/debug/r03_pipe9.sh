#!/bin/bash
# Round 3: the 4- vs 8-wave degridder bitwise test; masked adder loads with
# other tile shapes / batch sizes.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -q --timeout 120 --timeout-method thread -k "4_and_8_wave or ragged" > gpurun_out/pw.txt 2>&1 || { tail -30 gpurun_out/pw.txt; exit 1; }
tail -1 gpurun_out/pw.txt
for v in t32x8u4 t32x16u4 t64x4u4; do
  IDG_MI355X_LIB=$PWD/ab/$v.so timeout -k 10 200 python -u -m pytest tests/test_gpu_pipeline.py -m gpu -q --timeout 120 --timeout-method thread -k "adder or home_sort" > gpurun_out/pp_$v.txt 2>&1 || { echo "$v FAIL"; tail -20 gpurun_out/pp_$v.txt; exit 1; }
done
echo tests ok
bash tests/debug/ab_pipe.sh ab/mask.so ab/t32x8u4.so ab/t32x16u4.so ab/t16x16u8.so ab/t64x4u4.so
echo done
