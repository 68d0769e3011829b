#!/bin/bash
# Round 5: the degridder's per-chunk f16 scale (IDG_DEGRID_CHUNK_SCALE=1,
# ab/cs.so) against the per-subgrid scale pass (ab/base.so): which outputs
# change (multi-chunk subgrids only), the parity tests on the new library,
# configs[4] timing (interleaved, two reps) and its HBM counters.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_cs; mkdir -p $out
for lib in base cs; do
  IDG_MI355X_LIB=$PWD/ab/$lib.so timeout -k 10 300 python tools/debug/lib_outputs.py $out/$lib.npz > $out/out_$lib.txt 2>&1
done
python tools/debug/lib_outputs.py --compare $out/base.npz $out/cs.npz > $out/compare.txt 2>&1 || true
rm -f $out/*.npz
IDG_MI355X_LIB=$PWD/ab/cs.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu.py -k "sweep or w_terms or mixed or ragged or large_configs or image_size or large_grid or baseline_offsets or two_kernel or 4_and_8_wave or golden or oracle" \
  > $out/tests.txt 2>&1
BENCH_ARGS="--workload s64" STEPS=10 bash tools/debug/ab.sh ab/base.so ab/cs.so > $out/ab_s64.txt
cd /tmp && export TMPDIR=/tmp
for lib in base cs; do
  for c in FETCH_SIZE WRITE_SIZE; do
    IDG_MI355X_LIB=$GRAFT_REPO_ROOT/ab/$lib.so timeout -s KILL 200 rocprofv3 --pmc $c -d $GRAFT_REPO_ROOT/$out/${lib}_$c -o run -- \
      python3 $GRAFT_REPO_ROOT/bench.py --workload s64 --steps 2 --warmup 1 --min-warmup-s 0 \
      --no-cpu-baseline --no-side --no-pipeline > /dev/null 2> $GRAFT_REPO_ROOT/$out/${lib}_$c.err
  done
done
echo done
