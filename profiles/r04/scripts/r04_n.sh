#!/bin/bash
# The adder on increasingly centre-concentrated layouts of the configs[1]
# batch (ADVICE: the crowded-tile fallback's cost, never timed).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r04n
mkdir -p $out
timeout -k 10 400 python -u tests/debug/adder_crowded.py > $out/adder_crowded.txt 2> $out/adder_crowded.err || { tail -5 $out/adder_crowded.err; exit 1; }
cat $out/adder_crowded.txt
