#!/bin/bash
# Bench line per workload (s64, c256, wterm) into gpurun_out/wl/, plus the
# all-VALU A/B reference on wterm.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/wl
for w in ${WORKLOADS:-s64 wterm c256}; do
  steps=5; [ $w = c256 ] && steps=3
  timeout -k 10 400 python bench.py --no-cpu-baseline --workload $w --steps $steps > gpurun_out/wl/$w.json 2> gpurun_out/wl/$w.err || { tail -5 gpurun_out/wl/$w.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/wl/$w.json')); k=d['kernels']; print('$w', d['value'], k['gridder']['ms'], k['degridder']['ms'])"
done
IDG_GRIDDER_IMPL=valu IDG_DEGRIDDER_IMPL=valu timeout -k 10 300 python bench.py --no-cpu-baseline --no-pipeline --workload wterm --steps 5 > gpurun_out/wl/wterm_valu.json 2> gpurun_out/wl/wterm_valu.err || exit 1
python -c "
import json; d=json.load(open('gpurun_out/wl/wterm_valu.json')); k=d['kernels']; print('wterm_valu', d['value'], k['gridder']['ms'], k['degridder']['ms'])"
