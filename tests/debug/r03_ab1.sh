#!/bin/bash
# Round 3: GPU suite on the new default build, then A/B of the two-launch
# split, the k*phase_index tail correction and the general kernel's waves.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r03ab1
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $out/pytest_gpu.txt 2>&1 || echo "pytest rc=$?"
grep -E "passed|failed" $out/pytest_gpu.txt | tail -2
bash tests/debug/ab.sh ab/new.so ab/r02like.so ab/notail.so ab/nosplit.so ab/gw2.so
BENCH_ARGS="--workload wterm" STEPS=10 bash tests/debug/ab.sh ab/new.so ab/r02like.so ab/gw2.so
echo done
