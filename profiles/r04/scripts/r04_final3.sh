#!/bin/bash
# Round 4 closing call after the segmented adder: GPU suite, smoke and the
# default bench line (kernels unchanged since r04_final2; the pipeline's
# adder is the segmented one).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r04final3
mkdir -p $out
bash tests/debug/session.sh $out/s suite smoke || exit 1
timeout -k 10 600 python bench.py > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$out/bench.json')); k=d['kernels']; r=d['roofline']; p=d['pipeline']
print('default', d['value'], k['gridder']['ms'], k['degridder']['ms'], r.get('frac'), p['adder_ms'], p['roofline_hbm']['adder']['frac'], p['full_cycle_fused_mvis_s'])"
