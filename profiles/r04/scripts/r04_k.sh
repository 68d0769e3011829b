#!/bin/bash
# Round 4: the staged fill (IDG_GRID_STAGE: the next fill's raw rows copied
# into LDS by LDS-DMA during the current MFMA loop, 24 K-steps per fill;
# ab/st1.so) -- the gridder tests on it first, then timing against the
# shipped fill (ab/st0.so), default and c256 workloads, interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tests/debug/session.sh gpurun_out/r04k \
  'suite@ab/st1.so=gridder and not harness and not perf_mode' \
  ab=ab/st0.so,ab/st1.so || exit 1
BENCH_ARGS="--workload c256" STEPS=3 bash tests/debug/session.sh gpurun_out/r04k_c256 ab=ab/st0.so,ab/st1.so
