#!/bin/bash
# Persistent general-only kernels (XCD-strided subgrids) on the wterm and
# default workloads against the combined kernel.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/persist
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "wterm or mixed or sweep or golden" > gpurun_out/persist/pytest.txt 2>&1 || { tail -20 gpurun_out/persist/pytest.txt; exit 1; }
tail -1 gpurun_out/persist/pytest.txt
for pc in auto 4; do
  if [ $pc = auto ]; then unset IDG_PERSISTENT_PER_CU; else export IDG_PERSISTENT_PER_CU=$pc; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-pipeline --steps 10 --workload wterm > gpurun_out/persist/$pc.json 2> gpurun_out/persist/$pc.err
  python -c "
import json; d=json.load(open('gpurun_out/persist/$pc.json')); k=d['kernels']; print('per_cu $pc', d['value'], k['gridder']['ms'], k['degridder']['ms'])"
done
unset IDG_PERSISTENT_PER_CU
BENCH_ARGS="--workload wterm" STEPS=10 bash tests/debug/ab.sh ab/new.so ab/nosplit.so
bash tests/debug/ab.sh ab/new.so ab/nosplit.so
echo done
