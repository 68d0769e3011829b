#!/bin/bash
# Tuning round: MFMA-vs-VALU parity (w = 0 and w-terms), the GPU suite, and
# the bench per workload (value, gridder ms, degridder ms).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python tests/debug/diff_impl.py 2>&1 | grep -v "^  s"
DIFF_W=1 timeout -k 10 200 python tests/debug/diff_impl.py 2>&1 | grep -v "^  s"
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.txt 2>&1 || { tail -30 gpurun_out/pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/pytest_gpu.txt
for w in ${WORKLOADS:-default wterm s64}; do
timeout -k 10 300 python bench.py --no-cpu-baseline --workload $w > gpurun_out/b_$w.json 2> gpurun_out/b_$w.err
python -c "
import json; d=json.load(open('gpurun_out/b_$w.json')); print('$w', d['value'], d['kernels']['gridder']['ms'], d['kernels']['degridder']['ms'], d.get('pipeline',{}).get('adder_ms'))"
done
