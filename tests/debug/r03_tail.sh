#!/bin/bash
# Round 3: tail-split small launches -- bitwise tests, small-batch tests,
# then the one-GPU shard rehearsal.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r03tail
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -m gpu -v --timeout 300 --timeout-method thread -k "tail or mixed or empty or ragged or golden" > $out/pytest_gpu.txt 2>&1 || { echo "pytest rc=$?"; grep -E "PASS|FAIL|Error|error" $out/pytest_gpu.txt | tail -30; exit 1; }
grep -E "passed|failed" $out/pytest_gpu.txt | tail -1
timeout -k 10 400 python -u tests/debug/shard_rate.py --steps 10 > $out/shard_rate.txt 2>&1 || { tail -20 $out/shard_rate.txt; exit 1; }
grep predicted $out/shard_rate.txt
grep '"world": 8, "rank"' $out/shard_rate.txt
echo done
