#!/bin/bash
# Closing check after the adder's refused-slot guard: pipeline GPU tests,
# smoke, and the crowded-layout timing once.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r04p
mkdir -p $out
bash tests/debug/session.sh $out/s 'suite=pipeline or adder or dist' smoke || exit 1
timeout -k 10 400 python -u tests/debug/adder_crowded.py > $out/crowded.txt 2> $out/crowded.err || { tail -5 $out/crowded.err; exit 1; }
cat $out/crowded.txt
