#!/bin/bash
# Round 5: the fused splitter + inverse FFT, one plane per workgroup with
# rows across 2-4 lanes (default) against the four-plane form
# (IDG_SPLIT_FFT=rows): the bit-equality tests, then the bench's pipeline
# timings at configs[1] and configs[4], interleaved, two reps each, then a
# kernel trace of both.
# (The lanes kernel was removed after this A/B: profiles/r05/rejected/.  On
# today's tree IDG_SPLIT_FFT=1 and =rows both run the four-plane kernel.)
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_split; mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_pipeline.py -k "splitter_fft or splitter_matches or subgrid_fft" > $out/tests.txt 2>&1
for wl in default s64; do
  for rep in 1 2; do
    for form in 1 rows; do
      IDG_SPLIT_FFT=$form timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline --no-side \
        --steps 5 > $out/${wl}_${form}_$rep.json 2> $out/${wl}_${form}_$rep.err
      python -c "
import json; p=json.load(open('$out/${wl}_${form}_$rep.json'))['pipeline']
print('$wl', '$form', $rep, 'splitter_fft', p['splitter_fft_ms'], 'splitter', p['splitter_ms'], 'ifft', p['ifft_ms'], 'frac', p['roofline_hbm']['splitter_fft']['frac'], 'cycle', p['full_cycle_fused_mvis_s'])" >> $out/summary.txt
    done
  done
done
cd /tmp && export TMPDIR=/tmp
for wl in default s64; do
  for form in 1 rows; do
    IDG_SPLIT_FFT=$form timeout -s KILL 200 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/$out/kt_${wl}_$form -o run -- \
      python3 $GRAFT_REPO_ROOT/bench.py --workload $wl --no-cpu-baseline --no-side --steps 3 --warmup 1 \
      > /dev/null 2> $GRAFT_REPO_ROOT/$out/kt_${wl}_$form.err
  done
done
cd "$GRAFT_REPO_ROOT"
python tools/debug/kt_pipeline.py $out/kt_*/run_results.db >> $out/summary.txt
echo done
