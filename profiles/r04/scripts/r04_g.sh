#!/bin/bash
# Round 4: the B operands high in the f16 range (gridder first-fill maximum
# below 2^12, degridder below 2^13) and blocked summation every 8 fills as
# defaults -- GPU suite + smoke on this tree, then the s64 workload profiled
# with its bench line + cpu_baseline, then the c256 workload re-profiled.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r04g
mkdir -p $out
bash tests/debug/session.sh $out/s suite smoke  # a failing test does not end the call
bash profiles/r04/scripts/r04_wl_s64.sh || exit 1
bash tests/debug/session.sh $out/c profile=r04c256f8,--workload,c256
