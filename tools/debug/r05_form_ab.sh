#!/bin/bash
# Round 5: at the shard sizes of N = 2/4/8 (one GPU), the combined kernel
# (default below 8,192 subgrids) against the two-kernel form
# (IDG_KERNEL_FORM=split), now that the queue workspace is cached and the
# empty general launch returns before any atomic.  Same box, two reps.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_form; mkdir -p $out
for rep in 1 2; do
  timeout -k 10 300 python tools/debug/shard_rate.py --worlds 1,4,8 > $out/default_$rep.txt 2> $out/default_$rep.err
  IDG_KERNEL_FORM=split timeout -k 10 300 python tools/debug/shard_rate.py --worlds 1,4,8 > $out/split_$rep.txt 2> $out/split_$rep.err
done
grep -h predicted $out/*.txt
echo done
