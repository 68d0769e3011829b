#!/bin/bash
# The gridder's FFT epilogue and the persistent fused splitter + FFT: their
# bitwise GPU tests, then the bench line (pipeline.gridder_fft_ms,
# splitter_fft_ms) and a kernel trace of it.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r03c
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_gpu_pipeline.py -m gpu -x -v --timeout 300 --timeout-method thread -k "fft or splitter or adder or pipeline" > $out/pytest_fft.txt 2>&1 || { echo "pytest rc=$?"; grep -E "FAIL|Error" $out/pytest_fft.txt | tail -20; exit 1; }
grep -E "passed|failed" $out/pytest_fft.txt | tail -1
timeout -k 10 300 python bench.py --no-cpu-baseline > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python -c "
import json
d = json.load(open('$out/bench.json')); k = d['kernels']; p = d['pipeline']
print(d['value'], k['gridder']['ms'], k['degridder']['ms'])
print({x: p.get(x) for x in ('fft_ms', 'adder_ms', 'splitter_ms', 'ifft_ms', 'splitter_fft_ms', 'gridder_fft_ms', 'full_cycle_mvis_s', 'full_cycle_fused_mvis_s')})
"
bash tests/probes/profile_round.sh r03c
echo all done
