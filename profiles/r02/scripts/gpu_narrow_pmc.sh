# PMC traffic of the tiled 16-bit kernel (64 x 1e9 bf16), rocprofv3 counters in separate passes.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_narrow
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pmc_narrow/kt -o kt -- python $R/tools/bench_narrow.py --layout tiled --blocks-per-cu 2 --steps 3 > $R/gpurun_out/pmc_narrow/kt.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_narrow/fetch -o fetch -- python $R/tools/bench_narrow.py --layout tiled --blocks-per-cu 2 --steps 1 > $R/gpurun_out/pmc_narrow/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_narrow/write -o write -- python $R/tools/bench_narrow.py --layout tiled --blocks-per-cu 2 --steps 1 > $R/gpurun_out/pmc_narrow/write.log 2>&1
