#!/bin/bash
# Round 3 final (second session): the GPU suite, smoke(), the bench lines
# (default, wterm) and the profiles (kernel traces, FETCH / WRITE and SQ
# passes, traffic calibration).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r03final2
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $out/pytest_gpu.txt 2>&1 || { echo "pytest rc=$?"; grep -E "FAIL|Error" $out/pytest_gpu.txt | tail -20; exit 1; }
grep -E "passed|failed" $out/pytest_gpu.txt | tail -1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 || { tail -20 $out/smoke.txt; exit 1; }
echo smoke ok
timeout -k 10 300 python bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
timeout -k 10 300 python bench.py --workload wterm --no-cpu-baseline > $out/bench_wterm.json 2> $out/bench_wterm.err || { tail -20 $out/bench_wterm.err; exit 1; }
python -c "
import json
for f in ('bench', 'bench_wterm'):
    d = json.load(open('$out/' + f + '.json')); k = d['kernels']; p = d.get('pipeline', {})
    print(f, d['value'], k['gridder']['ms'], k['degridder']['ms'], d['roofline']['frac'], {x: p.get(x) for x in ('fft_ms', 'adder_ms', 'splitter_ms', 'ifft_ms', 'splitter_fft_ms', 'gridder_fft_ms', 'gridder_then_fft_ms', 'full_cycle_mvis_s', 'full_cycle_fused_mvis_s')})
"
bash tests/probes/profile_all.sh r03f2
echo all done
