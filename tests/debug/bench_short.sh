#!/bin/bash
# Bench without the CPU baseline; prints value, kernel times and pipeline.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 250 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/b.json 2> gpurun_out/b.err
python - <<'PY'
import json
d = json.load(open("gpurun_out/b.json"))
print("value", d["value"], "gridder", d["kernels"]["gridder"]["ms"], "degridder", d["kernels"]["degridder"]["ms"])
print("pipeline", d.get("pipeline"))
PY
