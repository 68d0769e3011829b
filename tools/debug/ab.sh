#!/bin/bash
# A/B timing of library variants: ab.sh lib1.so lib2.so ...  (per-kernel ms,
# default workload unless BENCH_ARGS says otherwise), each run twice, interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
for rep in 1 2; do
for lib in "$@"; do
  n=$(basename $lib .so)
  IDG_MI355X_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-pipeline --no-side --steps ${STEPS:-20} ${BENCH_ARGS:-} > gpurun_out/ab/$n.json 2> gpurun_out/ab/$n.err || { tail -5 gpurun_out/ab/$n.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/ab/$n.json')); k=d['kernels']; print('$n', d['value'], k['gridder']['ms'], k['degridder']['ms'])"
done
done
