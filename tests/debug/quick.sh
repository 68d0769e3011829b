#!/bin/bash
# Quick GPU check used while tuning: MFMA-vs-VALU parity on every subgrid of
# the full config, then the bench line's per-kernel times.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python tests/debug/diff_impl.py 2>&1 | grep -v "^  s"
timeout -k 10 200 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/b.json 2> gpurun_out/b.err
python - <<'PY'
import json
d = json.load(open("gpurun_out/b.json"))
print("value", d["value"], "gridder ms", d["kernels"]["gridder"]["ms"], "degridder ms", d["kernels"]["degridder"]["ms"])
PY
