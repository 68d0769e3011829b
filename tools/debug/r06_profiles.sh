#!/bin/bash
# Round 6: the profiles the bench line prices its rooflines from
# (profiles/traffic.json), every one on this round's kernels:
#   default (configs[1]), c256 at NR_TIMESLOTS=4 (configs[2]), s64
#   (configs[4]) and wterm: kernel trace + FETCH/WRITE passes
#   (tools/probes/profile_round.sh) and the SQ class passes
#   (tools/probes/pmc_sq.sh), MFMA kernels;
#   the order-preserving kernels at configs[1] and at configs[2] /
#   NR_TIMESLOTS=4 (tools/debug/r06_seq_prof.sh).
#   bash tools/debug/r06_profiles.sh [which...]   (default: all)
# Output under gpurun_out/.  Every GPU step has its own limit; the first
# failure ends the call.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r06_prof
mkdir -p $out
which=${*:-default c256 s64 wterm seq seq_c256}
for w in $which; do
  case $w in
    default) BA="" ;;
    c256) BA="--workload c256 --timeslots 4" ;;
    s64) BA="--workload s64" ;;
    wterm) BA="--workload wterm" ;;
    seq) timeout -k 10 900 bash tools/debug/r06_seq_prof.sh final > $out/seq.log 2>&1
         continue ;;
    seq_c256) timeout -k 10 900 bash tools/debug/r06_seq_prof.sh final_c256 \
                --workload c256 --timeslots 4 > $out/seq_c256.log 2>&1
              continue ;;
  esac
  BENCH_ARGS="$BA" timeout -k 10 600 bash tools/probes/profile_round.sh r06_$w > $out/prof_$w.log 2>&1
  BENCH_ARGS="$BA" timeout -k 10 900 bash tools/probes/pmc_sq.sh r06_$w > $out/pmc_$w.log 2>&1
  echo "$w done" | tee -a $out/progress.txt
done
echo "r06_profiles done"
