# GPU session (round 4, final build: pairs from 4 plain clients on, sessions 5-17): full `pytest -m gpu`, smoke(), the default bench line (config 3 + configs 5, 4,
# 2h, 2s, 4x in `also`; CPU baseline at 16 threads and at the full affinity), config 2, the 1-3-client lines, rocprofv3
# kernel traces of config 3, config 5 and the 2-client line, and the PMC traffic passes (FETCH_SIZE, WRITE_SIZE) of
# the same three.  Every GPU step has its own time limit; the script stops at the first failure.
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04_final3
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
B="python -u $GRAFT_REPO_ROOT/bench.py"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1 || exit $?
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || exit $?
timeout -k 10 400 $B > "$OUT/bench.jsonl" 2> "$OUT/bench.err" || exit $?
timeout -k 10 300 $B --config 2 --steps 50 --also none --no-cpu-baseline > "$OUT/bench_config2.jsonl" 2> "$OUT/bench_config2.err" || exit $?
for K in 1 2 3; do
  timeout -k 10 300 $B --clients $K --params 1e9 --also none --no-cpu-baseline > "$OUT/bench_k$K.jsonl" 2> "$OUT/bench_k$K.err" || exit $?
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rocprof_bench" -o bench -- $B --also none --no-cpu-baseline > "$OUT/bench_prof.jsonl" 2> "$OUT/bench_prof.err" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rocprof_adam" -o adam -- $B --config 5 --also none --no-cpu-baseline > "$OUT/bench_adam_prof.jsonl" 2> "$OUT/bench_adam_prof.err" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rocprof_k2" -o k2 -- $B --clients 2 --params 1e9 --also none --no-cpu-baseline > "$OUT/bench_k2_prof.jsonl" 2> "$OUT/bench_k2_prof.err" || exit $?
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc/none_$C" -o pmc -- $B --also none --steps 2 --warmup 1 --no-cpu-baseline --spot-check 0 > "$OUT/pmc_none_$C.log" 2>&1 || exit $?
  timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc/adam_$C" -o pmc -- $B --config 5 --also none --steps 2 --warmup 1 --no-cpu-baseline --spot-check 0 > "$OUT/pmc_adam_$C.log" 2>&1 || exit $?
  timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc/k2_$C" -o pmc -- $B --clients 2 --params 1e9 --also none --steps 2 --warmup 1 --no-cpu-baseline --spot-check 0 > "$OUT/pmc_k2_$C.log" 2>&1 || exit $?
done
# the fused kernel's partial last client group without repeated loads (fedavg_arith.h tile_sum) and its constant
cd "$GRAFT_REPO_ROOT"
for K in 2 3; do
  timeout -k 10 300 $B --clients $K --params 1e9 --epilogue adam --also none --no-cpu-baseline --steps 10 > "$OUT/bench_adam_k$K.jsonl" 2> "$OUT/bench_adam_k$K.err" || exit $?
done
echo done
