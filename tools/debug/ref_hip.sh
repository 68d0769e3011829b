#!/bin/bash
# The reference's own HIP kernels on this MI355X (oracle/_ref/hip/hip-*, built
# unmodified from /root/reference by `make -C oracle refhip`): `-c` parity at
# the reference's correctness defaults, then the reference's perf mode at
# BASELINE configs[1] (its env defaults: 50 stations, 20 timeslots, 128
# timesteps, 16 channels, S = 32).  The one-thread-per-subgrid *_reference
# kernels are timed at 2 timeslots (1,225 subgrids) only.  Output under
# gpurun_out/refhip/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/refhip
mkdir -p $out
export OUTPUT_PATH=$PWD/$out
for exe in oracle/_ref/hip/hip-*; do
  k=$(basename $exe)
  timeout -k 10 120 $exe -c > $out/$k.c.txt 2>&1 || { echo "$k -c exit $?"; tail -5 $out/$k.c.txt; exit 1; }
  res=$(grep -E "Result|error" $out/$k.c.txt | tr '\n' ' ')
  case $k in
    *reference) env="NR_TIMESLOTS=2 NR_WARM_UP_RUNS=0 NR_ITERATIONS=1" ;;
    *) env="" ;;
  esac
  env $env timeout -k 10 180 $exe > $out/$k.p.txt 2>&1 || { echo "$k perf exit $?"; tail -5 $out/$k.p.txt; exit 1; }
  perf=$(grep -iE "runtime|mvis" $out/$k.p.txt | tr -s ' ' | tr '\n' ' ')
  echo "$k | $res | $env | $perf"
done
