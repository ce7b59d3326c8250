# GPU session 21 (round 5): final tree -- fp32 1-client few-client form on tile pairs (session 20), 16-bit on tile
# pairs at 1 and 3 reads (session 18), fused units split by optimizer kind.  Full `pytest -m gpu`, smoke(), the
# default bench line, fp32 1 / 2 / 3-client lines, bf16 1 / 2 / 3-client lines, rocprofv3 kernel stats and the PMC
# traffic passes of the fp32 1-client line.  Every GPU step has its own time limit; the script stops at the first
# failure (a test failure included).
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05_s21
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
B="python -u $GRAFT_REPO_ROOT/bench.py"
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1 || exit $?
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || exit $?
timeout -k 10 600 $B > "$OUT/bench.jsonl" 2> "$OUT/bench.err" || exit $?
echo "bench done"
for K in 1 2 3; do
  timeout -k 10 300 $B --clients $K --params 1e9 --also none --no-cpu-baseline > "$OUT/bench_k$K.jsonl" 2> "$OUT/bench_k$K.err" || exit $?
  timeout -k 10 300 python -u tools/bench_narrow.py --params 1e9 --steps 10 --clients $K --fmt bfloat16 >> "$OUT/narrow.jsonl" 2>> "$OUT/err.log" || exit $?
done
echo "lines done"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rocprof_k1" -o k1 -- $B --clients 1 --params 1e9 --also none --no-cpu-baseline > "$OUT/bench_k1_prof.jsonl" 2> "$OUT/bench_k1_prof.err" || exit $?
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc/k1_$C" -o pmc -- $B --clients 1 --params 1e9 --also none --steps 2 --warmup 1 --no-cpu-baseline --spot-check 0 > "$OUT/pmc_k1_$C.log" 2>&1 || exit $?
done
echo done
