#!/bin/bash
# The round's closing GPU call: GPU suite, smoke, the default bench line and
# the profiles (tools/probes/profile_all.sh).  Output under gpurun_out/final
# and gpurun_out/{prof,pmc,calib}_TAG*; every GPU step has its own limit and
# the first failure ends the call.
set -eo pipefail
tag=${1:-r02}
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/final
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 \
  --timeout-method thread > $out/pytest_gpu.txt 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1
timeout -k 10 400 python bench.py > $out/bench.json 2> $out/bench.err
bash tools/probes/profile_all.sh "$tag"
echo final done
