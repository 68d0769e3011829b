#!/bin/bash
# Round 3: tail-split sweep at the N = 8 shard size (first n subgrids of
# configs[1]): plain combined kernels against tails of 128 / 256 / 512
# subgrids, and the size dependence of the plain form.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r03tail2
mkdir -p $out
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u tests/debug/shard_rate.py --steps 20 --counts 3063,6126 > $out/$name.txt 2>&1 || { tail -5 $out/$name.txt; exit 1; }
  echo "$name: $(grep nr_subgrids $out/$name.txt | tr '\n' ' ')"
}
run plain IDG_TAIL_SPLIT=0
run t256 IDG_TAIL_SPLIT=1
run t128 IDG_TAIL_SUBGRIDS=128
run t512 IDG_TAIL_SUBGRIDS=512
run plain2 IDG_TAIL_SPLIT=0
echo done
