#!/bin/bash
# Round 4: the gridder's fill with the loads of 2 or 4 K-steps issued before
# the first is used (ab/p2.so, ab/p4.so; IDG_GRID_FILL_PIPE) against one
# K-step at a time (ab/p1.so): default workload, interleaved, two reps, and
# the gridder tests on the 2-deep build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tests/debug/session.sh gpurun_out/r04j ab=ab/p1.so,ab/p2.so,ab/p4.so \
  'suite@ab/p2.so=gridder and not harness and not perf_mode and not fft'
