set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/v1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/v1/pytest_gpu.txt 2>&1 || { tail -30 gpurun_out/v1/pytest_gpu.txt; exit 1; }
tail -3 gpurun_out/v1/pytest_gpu.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/v1/smoke.txt 2>&1 || { cat gpurun_out/v1/smoke.txt; exit 1; }
cat gpurun_out/v1/smoke.txt
timeout -k 10 400 python bench.py > gpurun_out/v1/bench.json 2> gpurun_out/v1/bench.err || { tail gpurun_out/v1/bench.err; exit 1; }
cat gpurun_out/v1/bench.json
