#!/bin/bash
# Round 4: the workload bench lines on the closing kernels, with the
# committed traffic.json entries (roofline.traffic) and cpu_baselines:
# wterm, s64, c256; then launch cost against launch size (shard_rate.py
# --counts) for the N = 8 analysis.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r04h
mkdir -p $out
for w in wterm s64 c256; do
  steps=5; [ $w = c256 ] && steps=3
  timeout -k 10 900 python bench.py --workload $w --steps $steps > $out/$w.json 2> $out/$w.err || { tail -5 $out/$w.err; exit 1; }
  python -c "
import json; d=json.load(open('$out/$w.json')); k=d['kernels']; r=d['roofline']
print('$w', d['value'], k['gridder']['ms'], k['degridder']['ms'], r.get('frac'), r.get('traffic'), (d.get('cpu_baseline') or {}).get('value'))"
done
timeout -k 10 600 python -u tests/debug/shard_rate.py --counts 512,1024,2048,3063,4096,6125,12250 --steps 10 > $out/counts.txt 2>&1 || { tail -5 $out/counts.txt; exit 1; }
grep -v amdgpu.ids $out/counts.txt
