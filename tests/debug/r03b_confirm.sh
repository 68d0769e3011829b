#!/bin/bash
# Closing confirmation of the committed tree: the GPU suite, smoke() and the
# default bench line.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r03confirm
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $out/pytest_gpu.txt 2>&1 || { echo "pytest rc=$?"; grep -E "FAIL|Error" $out/pytest_gpu.txt | tail -20; exit 1; }
grep -E "passed|failed" $out/pytest_gpu.txt | tail -1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 || { tail -20 $out/smoke.txt; exit 1; }
echo smoke ok
timeout -k 10 300 python bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python -c "
import json
d = json.load(open('$out/bench.json')); k = d['kernels']
print(d['value'], k['gridder']['ms'], k['degridder']['ms'], d['roofline']['frac'], d['pipeline']['full_cycle_fused_mvis_s'])
"
echo all done
