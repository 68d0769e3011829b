#!/bin/bash
# SQ counters of the gridder for library variants (A/B diagnosis):
#   bash tools/probes/pmc_ab.sh ab/a.so ab/b.so
# Output: gpurun_out/pmc_ab/<lib>/p<N>/..., summary printed per library.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
root=$GRAFT_REPO_ROOT/gpurun_out/pmc_ab
mkdir -p "$root"
for lib in "$@"; do
  n=$(basename $lib .so)
  mkdir -p "$root/$n"
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
             "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    (cd /tmp && export TMPDIR=/tmp && IDG_MI355X_LIB=$GRAFT_REPO_ROOT/$lib timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$root/$n/p$i" -o run -- \
      python3 "$GRAFT_REPO_ROOT/bench.py" --steps 1 --warmup 1 --min-warmup-s 0 --no-cpu-baseline --no-pipeline > /dev/null 2> "$root/$n/p$i.err") || { echo "pass $i failed for $n"; tail -3 "$root/$n/p$i.err"; exit 1; }
  done
  python3 - "$root/$n" <<'PY'
import csv, glob, sys
from collections import defaultdict
acc = defaultdict(list)
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")
        if "kernel_gridder_mi355x" not in k:
            continue
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(sys.argv[1].split("/")[-1], {c: "%.4g" % (sum(v) / len(v)) for c, v in sorted(acc.items())})
PY
done
