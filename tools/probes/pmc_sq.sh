#!/bin/bash
# SQ instruction-mix / busy counters for the bench workload, one pass per
# group (gfx950 block limits).  Output under gpurun_out/pmc_<tag>/.
set -eo pipefail
tag=${1:-sq}
out=$GRAFT_REPO_ROOT/gpurun_out/pmc_$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > "$out/avail.txt" 2>&1 || true
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES" \
           "SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU_MFMA_F16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY" \
           "SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d "$out/p$i" -o run -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" ${BENCH_ARGS:-} --steps 1 --warmup 1 --min-warmup-s 0 --no-cpu-baseline --no-side > /dev/null 2> "$out/p$i.err" || { echo "pass $i failed"; exit 1; }
done
# optional: the VALU instruction classes (for the issue model's prices);
# a counter this rocprofv3 does not know ends only this pass
for grp in "SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32" \
           "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FMA_F16 SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_VALU_INT64"; do
  i=$((i+1))
  miss=""
  for c in $grp; do grep -qw "$c" "$out/avail.txt" || miss="$miss $c"; done
  [ -n "$miss" ] && { echo "pass $i skipped (not listed:$miss)"; continue; }
  timeout -s KILL 120 rocprofv3 --pmc $grp -d "$out/p$i" -o run -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" ${BENCH_ARGS:-} --steps 1 --warmup 1 --min-warmup-s 0 --no-cpu-baseline --no-side > /dev/null 2> "$out/p$i.err" || echo "optional pass $i failed"
done
echo done
