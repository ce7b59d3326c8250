# GPU session 19 (round 5): product library with the 16-bit few-client defaults on tile pairs at 1 and 3 reads
# (session 18).  The dtype GPU tests, smoke(), bf16 / fp16 lines at 1-3 clients (torch; fp16 numpy), rocprofv3 kernel
# stats and the PMC traffic passes of the bf16 1-client line.
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05_s19
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
N="python -u $GRAFT_REPO_ROOT/tools/bench_narrow.py --params 1e9 --steps 10"
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_dtypes.py > "$OUT/pytest_dtypes.log" 2>&1 || exit $?
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || exit $?
for K in 1 2 3; do
  timeout -k 10 300 $N --clients $K --fmt bfloat16 >> "$OUT/narrow.jsonl" 2>> "$OUT/err.log" || exit $?
  timeout -k 10 300 $N --clients $K --fmt float16 >> "$OUT/narrow.jsonl" 2>> "$OUT/err.log" || exit $?
  timeout -k 10 300 $N --clients $K --fmt float16 --mode numpy >> "$OUT/narrow.jsonl" 2>> "$OUT/err.log" || exit $?
done
echo "lines done"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rocprof_bf16_k1" -o k1 -- $N --clients 1 --fmt bfloat16 > "$OUT/bf16_k1_prof.jsonl" 2> "$OUT/bf16_k1_prof.err" || exit $?
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc/bf16_k1_$C" -o pmc -- python -u $GRAFT_REPO_ROOT/tools/bench_narrow.py --params 1e9 --steps 2 --clients 1 --fmt bfloat16 > "$OUT/pmc_bf16_k1_$C.log" 2>&1 || exit $?
done
echo done
