#!/bin/bash
# Same-box bisection of the round-2 -> round-3 headline drop: each tree's
# own bench.py and library (git worktrees under ab/), in order and then in
# reverse order.  Prints value, gridder ms, degridder ms per run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r04bisect
mkdir -p $out
trees="ab/r02tree ab/t_eca6608 ab/t_ad86ffd ab/t_1688827 ab/t_c7a2166 ab/t_a05af18 ab/t_e827692 ab/t_4aac030 ."
rev=$(echo $trees | tr ' ' '\n' | tac | tr '\n' ' ')
i=0
for t in $trees $rev; do
  i=$((i+1))
  n=$(basename $t)
  [ "$t" = "." ] && n=head
  (cd $t && timeout -k 10 240 python bench.py --no-cpu-baseline --no-pipeline --steps 20) > $out/$i.$n.json 2> $out/$i.$n.err || { tail -5 $out/$i.$n.err; exit 1; }
  python -c "
import json; d=json.load(open('$out/$i.$n.json')); k=d['kernels']; print('$n', d['value'], k['gridder']['ms'], k['degridder']['ms'])"
done
echo "head, IDG_KERNEL_FORM=combined"
IDG_KERNEL_FORM=combined timeout -k 10 240 python bench.py --no-cpu-baseline --no-pipeline --steps 20 > $out/combined.json 2> $out/combined.err && python -c "
import json; d=json.load(open('$out/combined.json')); k=d['kernels']; print('head-combined', d['value'], k['gridder']['ms'], k['degridder']['ms'])"
