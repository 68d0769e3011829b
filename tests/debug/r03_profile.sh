#!/bin/bash
# Round 3 profiles: the default and wterm workloads (kernel trace + FETCH /
# WRITE + SQ passes, pipeline kernels included) and the bench line.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03prof
timeout -k 10 300 python bench.py > gpurun_out/r03prof/bench.json 2> gpurun_out/r03prof/bench.err
bash tests/probes/profile_all.sh r03
echo all done
