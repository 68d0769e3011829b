set -eo pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/mall
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 $R/tools/probes/mall_probe > $R/gpurun_out/mall/plain.txt
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/mall/fetch -o run -- $R/tools/probes/mall_probe > $R/gpurun_out/mall/fetch.txt 2>&1
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum -d $R/gpurun_out/mall/dram -o run -- $R/tools/probes/mall_probe > $R/gpurun_out/mall/dram.txt 2>&1
timeout -s KILL 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $R/gpurun_out/mall/hit -o run -- $R/tools/probes/mall_probe > $R/gpurun_out/mall/hit.txt 2>&1
echo ok
