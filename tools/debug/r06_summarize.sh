#!/bin/bash
# Round 6: turn the profile calls of tools/debug/r06_profiles.sh (merged back
# under gpurun_out/) into profiles/r06/kernels_*/ and profiles/traffic.json,
# which bench.py prices its rooflines from.  CPU only.
set -eo pipefail
cd "$(dirname "$0")/../.."
declare -A NS=([default]=24500 [c256]=4900 [s64]=24500 [wterm]=24500)
declare -A NOTE=(
  [default]="configs[1]: 24,500 subgrids, 50.2 M visibilities"
  [c256]="configs[2] at NR_TIMESLOTS=4 (4,900 subgrids, 160.6 M visibilities)"
  [s64]="configs[4]: S = 64, 24,500 subgrids"
  [wterm]="the configs[1] batch with w-terms (bench.py apply_wterms)")
for w in default c256 s64 wterm; do
  [ -d gpurun_out/prof_r06_$w ] || continue
  python tools/probes/summarize_profiles.py --prof gpurun_out/prof_r06_$w \
    --pmc gpurun_out/pmc_r06_$w --out profiles/r06/kernels_$w --workload $w \
    --nr-subgrids ${NS[$w]} --note "${NOTE[$w]}"
done
if [ -d gpurun_out/r06_seq_final ]; then
  python tools/probes/summarize_seq.py gpurun_out/r06_seq_final \
    --out profiles/r06/sequential/sq_final.json --traffic profiles/traffic.json \
    --workload default --nr-subgrids 24500 --note "${NOTE[default]}" > /dev/null
fi
if [ -d gpurun_out/r06_seq_final_c256 ]; then
  python tools/probes/summarize_seq.py gpurun_out/r06_seq_final_c256 \
    --out profiles/r06/sequential/sq_final_c256.json --traffic profiles/traffic.json \
    --workload c256 --nr-subgrids 4900 --note "${NOTE[c256]}" > /dev/null
fi
echo summarized
