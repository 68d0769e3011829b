#!/bin/bash
# Round 4: what the gridder's B fills cost -- a timing-only build whose
# fills after the first reuse the first fill's B fragments (wrong output,
# ab/skipfill.so, IDG_DEBUG_SKIPFILL) against the shipped build, default
# workload, interleaved, two reps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tests/debug/session.sh gpurun_out/r04i ab=ab/base.so,ab/skipfill.so
