# GPU session 12 (round 5): final tree with the 16-bit few-client kernel (fedavg_narrow.hip fedavg_tiles_narrow_few,
# packed arithmetic, defaults from sessions 10-11) and tile_sum16 back on its per-element form.  Full `pytest -m gpu`,
# smoke(), the default bench line, bf16 / fp16 lines at 1-3 clients and bf16 at 8 / 64 clients (the burst form, to
# confirm the revert), rocprofv3 kernel stats of the bf16 1- and 2-client lines, and the PMC traffic passes
# (FETCH_SIZE, WRITE_SIZE) of the bf16 1-client line.  Every GPU step has its own time limit; the script stops at
# the first failure (a test failure included).
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05_s12
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
N="python -u $GRAFT_REPO_ROOT/tools/bench_narrow.py --params 1e9 --steps 10"
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1 || exit $?
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > "$OUT/bench.jsonl" 2> "$OUT/bench.err" || exit $?
echo "bench done"
for K in 1 2 3; do
  timeout -k 10 300 $N --clients $K --fmt bfloat16 >> "$OUT/narrow.jsonl" 2>> "$OUT/err.log" || exit $?
  timeout -k 10 300 $N --clients $K --fmt float16 >> "$OUT/narrow.jsonl" 2>> "$OUT/err.log" || exit $?
  timeout -k 10 300 $N --clients $K --fmt float16 --mode numpy >> "$OUT/narrow.jsonl" 2>> "$OUT/err.log" || exit $?
done
timeout -k 10 300 $N --clients 8 --fmt bfloat16 >> "$OUT/narrow.jsonl" 2>> "$OUT/err.log" || exit $?
timeout -k 10 300 python -u tools/bench_narrow.py --clients 64 --params 2.5e8 --steps 10 --fmt bfloat16 >> "$OUT/narrow.jsonl" 2>> "$OUT/err.log" || exit $?
echo "lines done"
cd /tmp
for K in 1 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rocprof_bf16_k$K" -o k$K -- $N --clients $K --fmt bfloat16 > "$OUT/bf16_k${K}_prof.jsonl" 2> "$OUT/bf16_k${K}_prof.err" || exit $?
done
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc/bf16_k1_$C" -o pmc -- python -u $GRAFT_REPO_ROOT/tools/bench_narrow.py --params 1e9 --steps 2 --clients 1 --fmt bfloat16 > "$OUT/pmc_bf16_k1_$C.log" 2>&1 || exit $?
done
echo done
