#!/bin/bash
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r03start
mkdir -p $out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.txt 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1
timeout -k 10 300 python bench.py > $out/bench.json 2> $out/bench.err
echo done
