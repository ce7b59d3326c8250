# GPU box script: PMC HBM traffic of the bench kernel on the current build, FETCH_SIZE and WRITE_SIZE in
# separate rocprofv3 passes (the program itself directly after --), each under its own hard time limit.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_bench
mkdir -p "$OUT"
cd /tmp
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o fetch -- python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --spot-check 0 > "$OUT/fetch.log" 2>&1
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o write -- python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --spot-check 0 > "$OUT/write.log" 2>&1
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch_adam" -o fetch -- python $R/bench.py --epilogue adam --steps 2 --warmup 1 --no-cpu-baseline --spot-check 0 > "$OUT/fetch_adam.log" 2>&1
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write_adam" -o write -- python $R/bench.py --epilogue adam --steps 2 --warmup 1 --no-cpu-baseline --spot-check 0 > "$OUT/write_adam.log" 2>&1
