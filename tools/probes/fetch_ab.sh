#!/bin/bash
# HBM-side bytes per launch (FETCH_SIZE x 2 + WRITE_SIZE, gfx950 correction)
# of the MFMA gridder/degridder for library variants:
#   bash tools/probes/fetch_ab.sh ab/a.so ab/b.so
set -o pipefail
cd "$GRAFT_REPO_ROOT"
root=$GRAFT_REPO_ROOT/gpurun_out/fetch_ab
for lib in "$@"; do
  n=$(basename $lib .so)
  mkdir -p "$root/$n"
  for c in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && export TMPDIR=/tmp && IDG_MI355X_LIB=$GRAFT_REPO_ROOT/$lib timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$root/$n/$c" -o run -- \
      python3 "$GRAFT_REPO_ROOT/bench.py" --steps 1 --warmup 1 --min-warmup-s 0 --no-cpu-baseline --no-pipeline > /dev/null 2> "$root/$n/$c.err") || { echo "$c failed for $n"; tail -3 "$root/$n/$c.err"; exit 1; }
  done
  python3 - "$root/$n" "$n" <<'PY'
import csv, glob, sys
from collections import defaultdict
acc = defaultdict(list)
for f in glob.glob(sys.argv[1] + "/*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")
        for d in ("degridder", "gridder"):
            if f"kernel_{d}_mi355x" in k:
                acc[(d, r["Counter_Name"])].append(float(r["Counter_Value"]))
                break
for d in ("gridder", "degridder"):
    f = sum(acc[(d, "FETCH_SIZE")]) / max(1, len(acc[(d, "FETCH_SIZE")]))
    w = sum(acc[(d, "WRITE_SIZE")]) / max(1, len(acc[(d, "WRITE_SIZE")]))
    print(sys.argv[2], d, "fetch GB x2 %.3f" % (2 * f * 1024 / 1e9), "write GB %.3f" % (w * 1024 / 1e9),
          "total %.3f" % ((2 * f + w) * 1024 / 1e9))
PY
done
