# GPU session 15 (round 5): final tree with the fp64 few-client kernel (defaults from session 14).  Full
# `pytest -m gpu`, smoke(), the default bench line, fp64 lines at 1-3 clients (numpy mode; torch at 2), bf16 at 1-2
# clients, rocprofv3 kernel stats of the fp64 2-client line.  Every GPU step has its own time limit; the script stops
# at the first failure (a test failure included).
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05_s15
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
G="python -u $GRAFT_REPO_ROOT/tools/bench_generic.py --dtype float64 --layout tiled --params 5e8 --steps 10"
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1 || exit $?
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > "$OUT/bench.jsonl" 2> "$OUT/bench.err" || exit $?
echo "bench done"
for K in 1 2 3; do
  timeout -k 10 300 $G --clients $K >> "$OUT/f64.jsonl" 2>> "$OUT/err.log" || exit $?
done
timeout -k 10 300 $G --clients 2 --mode torch >> "$OUT/f64.jsonl" 2>> "$OUT/err.log" || exit $?
for K in 1 2; do
  timeout -k 10 300 python -u tools/bench_narrow.py --params 1e9 --steps 10 --clients $K --fmt bfloat16 >> "$OUT/narrow.jsonl" 2>> "$OUT/err.log" || exit $?
done
echo "lines done"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rocprof_f64_k2" -o k2 -- $G --clients 2 > "$OUT/f64_k2_prof.jsonl" 2> "$OUT/f64_k2_prof.err" || exit $?
echo done
