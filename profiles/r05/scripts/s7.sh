# GPU session 7 (round 5): the routing from session 6 (3 reads on the few-client kernel, 4 and 6 clients on the
# remainder forms, 5 built in): full pytest -m gpu and smoke() on the product library, then the 1-8-client plain
# bench lines x 1e9 (3 rounds) and the 3-client line under rocprofv3.
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05_s7
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
B="python -u $GRAFT_REPO_ROOT/bench.py --also none --no-cpu-baseline --params 1e9"
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1 || exit $?
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || exit $?
for R in 1 2 3; do
  for K in 1 2 3 4 5 6 7 8; do
    timeout -k 10 200 $B --clients $K >> "$OUT/bench_k$K.jsonl" 2>> "$OUT/err.log" || exit $?
  done
  echo "round $R done"
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rocprof_k3" -o k3 -- $B --clients 3 > "$OUT/bench_k3_prof.jsonl" 2>> "$OUT/err.log" || exit $?
echo done
