#!/bin/bash
# Round 3: kernel trace of the N = 8 shard-size launches (plain combined
# kernels): GPU-side kernel durations against the event-timed ones.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
IDG_TAIL_SPLIT=0 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/kt_shard -o run -- python3 tests/debug/shard_rate.py --steps 20 --counts 3063 > gpurun_out/kt_shard.log 2>&1 || { tail -20 gpurun_out/kt_shard.log; exit 1; }
grep nr_subgrids gpurun_out/kt_shard.log
echo done
