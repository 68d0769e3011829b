#!/bin/bash
# Round 6: the GPU suite on this tree, then the event-cost probe
# (tools/debug/event_cost.py).  Output under gpurun_out/r06_check_TAG/.
# Every GPU step has its own limit; the first failure ends the call.
#   bash tools/debug/r06_check.sh TAG [skip-tests]
set -eo pipefail
tag=${1:-a}
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r06_check_$tag
mkdir -p $out
if [ "${2:-}" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 \
    --timeout-method thread > $out/pytest_gpu.txt 2>&1
  tail -1 $out/pytest_gpu.txt
fi
timeout -k 10 300 python tools/debug/event_cost.py > $out/event_cost.txt 2> $out/event_cost.err
cat $out/event_cost.txt
echo "r06_check $tag done"
