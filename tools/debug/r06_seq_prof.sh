#!/bin/bash
# Round 6: the bit-exact ("sequential") kernels measured the way the default
# kernels are -- kernel trace + stats, then the SQ instruction-class passes
# (one rocprofv3 run per group, gfx950 block limits) -- and the issue cost of
# the instruction kinds they spend their time in (seq_rates_probe).
#   bash tools/debug/r06_seq_prof.sh TAG [bench args...]
# Output under gpurun_out/r06_seq_TAG/.  Every GPU step has its own limit;
# the first failure ends the call.
set -eo pipefail
tag=${1:-base}
shift || true
out=$GRAFT_REPO_ROOT/gpurun_out/r06_seq_$tag
mkdir -p "$out"
export IDG_GRIDDER_IMPL=sequential IDG_DEGRIDDER_IMPL=sequential
BA="$* --no-cpu-baseline --no-side --no-pipeline --no-weak"
if [ -n "${RATES:-}" ]; then
  timeout -k 10 120 "$GRAFT_REPO_ROOT/tools/probes/seq_rates_probe" > "$out/seq_rates.txt"
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/ktrace" -o run -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" $BA --steps 3 --warmup 1 --min-warmup-s 0 \
  > "$out/bench_ktrace.json" 2> "$out/bench_ktrace.err"
[ -n "${NO_PMC:-}" ] && { echo done; exit 0; }
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES" \
           "SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_CVT" \
           "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32" \
           "SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_LDS SQ_WAIT_INST_ANY" \
           "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_TRANS_F64 SQ_INST_CYCLES_VMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d "$out/p$i" -o run -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" $BA --steps 1 --warmup 0 --min-warmup-s 0 \
    > /dev/null 2> "$out/p$i.err" || { echo "pass $i failed"; exit 1; }
done
echo done
