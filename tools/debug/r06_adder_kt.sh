#!/bin/bash
# Round 6: kernel traces of the pipeline steps for two libraries (the adder
# A/B's splitter question), same box:
#   bash tools/debug/r06_adder_kt.sh LIB...
# Output under gpurun_out/r06_adder_kt/.  Every GPU step has its own limit;
# the first failure ends the call.
set -eo pipefail
out=$GRAFT_REPO_ROOT/gpurun_out/r06_adder_kt
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
for lib in "$@"; do
  n=$(basename $lib .so)
  IDG_MI355X_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 300 rocprofv3 --kernel-trace \
    --output-format csv -d "$out/kt_$n" -o run -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline \
    --no-side > "$out/bench_$n.json"
done
echo "r06_adder_kt done"
