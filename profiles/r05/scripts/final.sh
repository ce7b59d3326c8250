# GPU session: round-5 final tree (product library: routed forms only; few-client burst kernel for 1-2 reads; FIN_DIV
# with one rare-case branch per tile; fused burst epilogue kEmFast, fused per-tile kEmElem).  Full `pytest -m gpu`,
# smoke(), the default bench line (config 3 + configs 5, 4, 2h, 2s, 4x in `also`; CPU baseline at the cgroup quota),
# config 2, the 1-3-client plain lines, the 2-3-client fused Adam lines, config 5 at two blocks per CU against its
# default (one), rocprofv3 kernel stats of config 3, config 5 and the 1- and 2-client lines, and the PMC traffic passes
# (FETCH_SIZE, WRITE_SIZE) of configs 3 and 5.  Every GPU step has its own time limit; the script stops at the first
# failure (a test failure included).
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05_final
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
B="python -u $GRAFT_REPO_ROOT/bench.py"
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1 || exit $?
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || exit $?
timeout -k 10 600 $B > "$OUT/bench.jsonl" 2> "$OUT/bench.err" || exit $?
echo "bench done"
timeout -k 10 300 $B --config 2 --steps 50 --also none --no-cpu-baseline > "$OUT/bench_config2.jsonl" 2> "$OUT/bench_config2.err" || exit $?
for K in 1 2 3; do
  timeout -k 10 300 $B --clients $K --params 1e9 --also none --no-cpu-baseline > "$OUT/bench_k$K.jsonl" 2> "$OUT/bench_k$K.err" || exit $?
done
for K in 2 3; do
  timeout -k 10 300 $B --clients $K --params 1e9 --epilogue adam --also none --no-cpu-baseline --steps 10 > "$OUT/bench_adam_k$K.jsonl" 2> "$OUT/bench_adam_k$K.err" || exit $?
done
for R in 1 2; do
  timeout -k 10 300 $B --config 5 --also none --no-cpu-baseline >> "$OUT/c5_bpc1.jsonl" 2>> "$OUT/c5.err" || exit $?
  timeout -k 10 300 $B --config 5 --also none --no-cpu-baseline --blocks-per-cu 2 >> "$OUT/c5_bpc2.jsonl" 2>> "$OUT/c5.err" || exit $?
done
echo "lines done"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rocprof_bench" -o bench -- $B --also none --no-cpu-baseline > "$OUT/bench_prof.jsonl" 2> "$OUT/bench_prof.err" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rocprof_adam" -o adam -- $B --config 5 --also none --no-cpu-baseline > "$OUT/bench_adam_prof.jsonl" 2> "$OUT/bench_adam_prof.err" || exit $?
for K in 1 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rocprof_k$K" -o k$K -- $B --clients $K --params 1e9 --also none --no-cpu-baseline > "$OUT/bench_k${K}_prof.jsonl" 2> "$OUT/bench_k${K}_prof.err" || exit $?
done
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc/none_$C" -o pmc -- $B --also none --steps 2 --warmup 1 --no-cpu-baseline --spot-check 0 > "$OUT/pmc_none_$C.log" 2>&1 || exit $?
  timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc/adam_$C" -o pmc -- $B --config 5 --also none --steps 2 --warmup 1 --no-cpu-baseline --spot-check 0 > "$OUT/pmc_adam_$C.log" 2>&1 || exit $?
done
echo done
