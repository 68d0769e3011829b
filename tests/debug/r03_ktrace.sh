#!/bin/bash
# Kernel trace of the wterm workload: per-kernel times of the two-kernel
# form (mirror launch that only queues, general launch) vs the combined one.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
out=$GRAFT_REPO_ROOT/gpurun_out/ktrace_wterm
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
for lib in new nosplit; do
  IDG_MI355X_LIB=$GRAFT_REPO_ROOT/ab/$lib.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/$lib" -o run -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --workload wterm --steps 5 --warmup 2 --min-warmup-s 0 --no-cpu-baseline --no-pipeline > "$out/$lib.json"
  python3 - "$out/$lib" <<'PY'
import csv, glob, sys
from collections import defaultdict
d = defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        d[r["Kernel_Name"][:70]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
for k, v in sorted(d.items(), key=lambda x: -sum(x[1])):
    if "mi355x" in k:
        print(sys.argv[1].split("/")[-1], f"{k:70s} n={len(v):3d} mean {sum(v)/len(v):.4f} ms min {min(v):.4f}")
PY
done
echo done
