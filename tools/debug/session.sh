#!/bin/bash
# One GPU call built from steps (replaces the one-off per-experiment scripts
# of rounds 2-3).  Every step runs under its own time limit, the steps are
# chained, and the first failure ends the call.
#
#   bash tools/debug/session.sh OUTDIR STEP [STEP ...]
#
# STEP:
#   suite[=K]            GPU test suite (pytest -m gpu), optional -k filter K
#   suite@LIB[=K]        the same on another library build (IDG_MI355X_LIB)
#   smoke                __graft_entry__.smoke()
#   bench[=ARGS]         one bench.py line (ARGS with ',' for ' ')
#   ab=A.so,B.so,...     kernel A/B, interleaved, two reps (ab.sh; STEPS,
#                        BENCH_ARGS from the environment)
#   abpipe=A.so,B.so     pipeline-kernel A/B (ab_pipe.sh)
#   shard                one-GPU shard rehearsal (shard_rate.py)
#   profile=TAG[,ARGS]   kernel trace + FETCH/WRITE passes + SQ passes of a
#                        bench workload (profile_round.sh, pmc_sq.sh)
#   accuracy[@LIB]       gridder distance to exact accumulation
#                        (accuracy_ab.py)
#   probe=NAME           a built probe executable (tools/probes/NAME)
#
# Example (the round-3 "lean splitter" A/B):
#   bash tools/debug/session.sh gpurun_out/x 'suite@ab/lean.so=splitter' \
#        abpipe=ab/lean.so,ab/shipped.so
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
out=$1
shift
mkdir -p "$out"
n=0
for step in "$@"; do
  n=$((n + 1))
  name=${step%%=*}
  arg=${step#*=}
  [ "$arg" = "$step" ] && arg=""
  lib=""
  case $name in *@*) lib=${name#*@}; name=${name%%@*};; esac
  libenv=()
  [ -n "$lib" ] && libenv=(IDG_MI355X_LIB="$PWD/$lib")
  log=$out/$n.$name.txt
  echo "[$n] $step"
  case $name in
    suite)
      k=()
      [ -n "$arg" ] && k=(-k "$arg")
      env "${libenv[@]}" timeout -k 10 900 python -u -m pytest tests -m gpu -x -v \
        --timeout 300 --timeout-method thread "${k[@]}" > "$log" 2>&1
      rc=$?; grep -E "passed|failed|error" "$log" | tail -1 ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$log" 2>&1
      rc=$?; tail -2 "$log" ;;
    bench)
      env "${libenv[@]}" timeout -k 10 600 python bench.py ${arg//,/ } > "$log" 2> "$log.err"
      rc=$?; python -c "
import json; d = json.load(open('$log')); k = d['kernels']
print(d['value'], k['gridder']['ms'], k['degridder']['ms'])" ;;
    ab)
      timeout -k 10 1200 bash tools/debug/ab.sh ${arg//,/ } > "$log" 2>&1
      rc=$?; cat "$log" ;;
    abpipe)
      timeout -k 10 1200 bash tools/debug/ab_pipe.sh ${arg//,/ } > "$log" 2>&1
      rc=$?; cat "$log" ;;
    shard)
      timeout -k 10 600 python -u tools/debug/shard_rate.py --steps 10 > "$log" 2>&1
      rc=$?; grep predicted "$log" ;;
    profile)
      tag=${arg%%,*}
      bargs=""
      [ "$tag" != "$arg" ] && bargs=${arg#*,}
      BENCH_ARGS="${bargs//,/ }" timeout -k 10 900 bash tools/probes/profile_round.sh "$tag" > "$log" 2>&1 &&
      BENCH_ARGS="${bargs//,/ }" timeout -k 10 900 bash tools/probes/pmc_sq.sh "$tag" >> "$log" 2>&1
      rc=$?; tail -2 "$log" ;;
    accuracy)
      env "${libenv[@]}" timeout -k 10 600 python -u tools/debug/accuracy_ab.py "${lib:-head}" > "$log" 2>&1
      rc=$?; cat "$log" ;;
    probe)
      timeout -k 10 300 "tools/probes/$arg" > "$log" 2>&1
      rc=$?; cat "$log" ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
  if [ $rc -ne 0 ]; then
    echo "step $n ($step) failed: rc=$rc"
    tail -20 "$log"
    exit $rc
  fi
done
echo "session done"
