#!/bin/bash
# Segmented adder (crowded tiles split over several workgroups): the
# pipeline GPU tests, then the adder on the centre-concentrated layouts with
# the segments (IDG_ADD_SEG=1) and without (0), interleaved, two reps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r04o
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py -m gpu -x -v \
  --timeout 120 --timeout-method thread > $out/pipeline_tests.txt 2>&1
rc=$?; grep -E "passed|failed|error" $out/pipeline_tests.txt | tail -3; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  for seg in 0 1; do
    IDG_ADD_SEG=$seg timeout -k 10 400 python -u tests/debug/adder_crowded.py \
      > $out/crowded_seg${seg}_$rep.txt 2> $out/crowded_seg${seg}_$rep.err || { tail -5 $out/crowded_seg${seg}_$rep.err; exit 1; }
    echo "seg=$seg rep=$rep"; cat $out/crowded_seg${seg}_$rep.txt
  done
done
