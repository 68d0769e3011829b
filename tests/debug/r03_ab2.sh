#!/bin/bash
# Round 3: GPU suite on the two-launch (mirror-only + persistent general-only)
# build with the re-binned adder and the ordered splitter, then A/B against
# the combined kernel (nosplit), the round-2-like build and single-direction
# splits (default and wterm), and the pipeline steps.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r03ab2
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $out/pytest_gpu.txt 2>&1 || echo "pytest rc=$?"
grep -E "passed|failed" $out/pytest_gpu.txt | tail -2
bash tests/debug/ab.sh ab/new.so ab/nosplit.so ab/r02like.so ab/gsplit.so ab/dsplit.so
BENCH_ARGS="--workload wterm" STEPS=10 bash tests/debug/ab.sh ab/new.so ab/nosplit.so ab/r02like.so
bash tests/debug/ab_pipe.sh ab/new.so ab/r02like.so
echo done
