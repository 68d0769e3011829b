#!/bin/bash
# Round 6: the bit-exact ("sequential") kernels, before / after.
#   bash tools/debug/r06_seq_ab.sh TAG NEW_LIB [BASE_LIB]
# 1. the instruction-rate probe of the kinds they spend their time in;
# 2. tests/test_gpu_sequential.py on NEW_LIB (bit-exactness, both sincosf
#    forms on the GPU against glibc);
# 3. same-box A/B of BASE_LIB and NEW_LIB, sequential kernels, configs[1],
#    two interleaved reps;
# 4. kernel trace + SQ class passes of NEW_LIB (tools/debug/r06_seq_prof.sh),
#    and of BASE_LIB with SQ_BASE=1.
# Output under gpurun_out/r06_seq_ab_TAG/.  Every GPU step has its own limit;
# the first failure ends the call.
set -eo pipefail
tag=${1:?tag}
new=${2:?new lib}
base=${3:-}
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r06_seq_ab_$tag
mkdir -p $out
timeout -k 10 120 tools/probes/seq_rates_probe > $out/seq_rates.txt
IDG_MI355X_LIB=$PWD/$new timeout -k 10 600 python -u -m pytest \
  tests/test_gpu_sequential.py -x -v --timeout 300 --timeout-method thread \
  > $out/seq_tests.log 2>&1
export IDG_GRIDDER_IMPL=sequential IDG_DEGRIDDER_IMPL=sequential
for rep in 1 2; do
  for lib in $base $new; do
    n=$(basename $lib .so)_$rep
    IDG_MI355X_LIB=$PWD/$lib timeout -k 10 300 python bench.py \
      --no-cpu-baseline --no-pipeline --no-side --no-weak --steps 3 \
      --warmup 1 --min-warmup-s 0 ${BENCH_ARGS:-} > $out/ab_$n.json 2> $out/ab_$n.err
    python -c "
import json; d=json.load(open('$out/ab_$n.json')); k=d['kernels']
print('$n', d['value'], k['gridder']['ms'], k['degridder']['ms'])" | tee -a $out/ab.txt
  done
done
unset IDG_GRIDDER_IMPL IDG_DEGRIDDER_IMPL
# optional: the default (MFMA) kernels of BASE_LIB and NEW_LIB, same box
if [ -n "${ABDEF:-}" ] && [ -n "$base" ]; then
  for rep in 1 2; do
    for lib in $base $new; do
      n=def_$(basename $lib .so)_$rep
      IDG_MI355X_LIB=$PWD/$lib timeout -k 10 300 python bench.py \
        --no-cpu-baseline --no-pipeline --no-side --no-weak --steps 20 \
        > $out/ab_$n.json 2> $out/ab_$n.err
      python -c "
import json; d=json.load(open('$out/ab_$n.json')); k=d['kernels']
print('$n', d['value'], k['gridder']['ms'], k['degridder']['ms'])" | tee -a $out/ab.txt
    done
  done
fi
# optional: extra GPU tests on NEW_LIB (pytest -k expression)
if [ -n "${TESTS_K:-}" ]; then
  IDG_MI355X_LIB=$PWD/$new timeout -k 10 900 python -u -m pytest tests -m gpu \
    -k "$TESTS_K" -x -v -s --timeout 600 --timeout-method thread \
    > $out/extra_tests.log 2>&1
fi
IDG_MI355X_LIB=$PWD/$new timeout -k 10 900 bash tools/debug/r06_seq_prof.sh ${tag}_new ${BENCH_ARGS:-}
if [ -n "${SQ_BASE:-}" ] && [ -n "$base" ]; then
  IDG_MI355X_LIB=$PWD/$base timeout -k 10 900 bash tools/debug/r06_seq_prof.sh ${tag}_base ${BENCH_ARGS:-}
fi
echo "r06_seq_ab $tag done"
