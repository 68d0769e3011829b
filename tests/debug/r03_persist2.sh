#!/bin/bash
# Round 3: persistent mirror kernels taking subgrids from per-XCD work
# ranges with stealing -- two-kernel/mixed/full-size tests, then A/B against
# the one-workgroup-per-subgrid mirror kernels (default and N = 2 shard).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r03persist2
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu.py -m gpu -q --timeout 300 --timeout-method thread -k "two_kernel or mixed or full_size or deterministic" > $out/pytest_gpu.txt 2>&1 || { echo "pytest rc=$?"; grep -E "FAIL|Error" $out/pytest_gpu.txt | tail -20; exit 1; }
tail -1 $out/pytest_gpu.txt
bash tests/debug/ab.sh ab/old.so ab/new.so
for lib in old new; do
  IDG_MI355X_LIB=$PWD/ab/$lib.so timeout -k 10 300 python -u tests/debug/shard_rate.py --steps 10 --counts 12250 > $out/shard_$lib.txt 2>&1 || { tail -5 $out/shard_$lib.txt; exit 1; }
  echo "$lib: $(grep nr_subgrids $out/shard_$lib.txt)"
done
echo done
