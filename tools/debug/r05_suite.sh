#!/bin/bash
# The whole GPU suite in one process, as the driver runs it at round end.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05_suite
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r05_suite/pytest_gpu.txt 2>&1
echo rc=$?
