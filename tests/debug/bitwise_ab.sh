#!/bin/bash
# Bitwise A/B of two library builds on the bench batch (reduced to 2 time
# slots): gridder subgrids and degridded visibilities must be identical.
#   bash tests/debug/bitwise_ab.sh ab/old.so ab/new.so
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
for lib in "$1" "$2"; do
  n=$(basename $lib .so)
  IDG_MI355X_LIB=$PWD/$lib timeout -k 10 200 python bench.py --steps 1 --warmup 1 \
    --timeslots 2 --no-cpu-baseline --dump gpurun_out/bw/$n > /dev/null
done
python - "$(basename $1 .so)" "$(basename $2 .so)" <<'PY'
import sys, numpy as np
a, b = sys.argv[1:3]
for k in ("subgrids", "visibilities"):
    x = np.load(f"gpurun_out/bw/{a}/{k}.npy"); y = np.load(f"gpurun_out/bw/{b}/{k}.npy")
    print(k, "identical" if np.array_equal(x, y) else
          "DIFFER max rel %.3g" % (np.abs(x - y).max() / np.abs(x).max()))
PY
