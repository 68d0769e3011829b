#!/bin/bash
# Round 6: the whole GPU suite, smoke() and the default bench line (with its
# side legs) on this tree.  Output under gpurun_out/r06_suite_TAG/.  Every
# GPU step has its own limit; the first failure ends the call.
#   bash tools/debug/r06_suite.sh TAG [skip-tests]
set -eo pipefail
tag=${1:-a}
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r06_suite_$tag
mkdir -p $out
if [ "${2:-}" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 \
    --timeout-method thread > $out/pytest_gpu.txt 2>&1
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1
fi
timeout -k 10 600 python bench.py > $out/bench.json 2> $out/bench.err
echo "r06_suite $tag done"
