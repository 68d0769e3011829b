#!/bin/bash
# A/B of library variants on the pipeline steps (FFT, adder, splitter ms).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/abp
for rep in 1 2; do
for lib in "$@"; do
  n=$(basename $lib .so)
  IDG_MI355X_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 ${BENCH_ARGS:-} > gpurun_out/abp/$n.json 2> gpurun_out/abp/$n.err || { tail -5 gpurun_out/abp/$n.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/abp/$n.json')); p=d['pipeline']; print('$n', p['fft_ms'], p['adder_ms'], p['splitter_ms'], p['ifft_ms'], p.get('splitter_fft_ms'), p.get('gridder_fft_ms'), p.get('gridder_then_fft_ms'), p.get('full_cycle_mvis_s'), p.get('full_cycle_fused_mvis_s'))"
done
done
