# GPU session 1 (round 5).  The stripped product library (routed forms only; few-client burst kernel for 1-2 reads;
# one rare-case branch per tile / column group in the finalisation and the fused epilogues) against the round-4 final
# sources (HEAD 60338f3, built by tools/build_rev_lib.py as nvflare_amd/lib/ab/head.so):
#   1. pytest -m gpu and smoke() on the product library;
#   2. alternating processes, 3 rounds: fused Adam at 2 / 3 clients (AMD-host sqrt), plain 1 / 2 /
#      3 clients (item 3), 5e8 params;
#   3. the default bench line on the product library.
# A test failure (pytest exit 1) does not stop the measurements; a crash, abort or time limit does.
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05_s1
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || exit $?
B="python -u $GRAFT_REPO_ROOT/bench.py --also none --no-cpu-baseline --params 5e8 --steps 20 --warmup 3"
for R in 1 2 3; do
  for L in head prod; do
    if [ $L = prod ]; then unset NVFLARE_AMD_FEDAVG_LIB; else export NVFLARE_AMD_FEDAVG_LIB=$GRAFT_REPO_ROOT/nvflare_amd/lib/ab/$L.so; fi
    for K in 2 3; do
      timeout -k 10 200 $B --clients $K --epilogue adam --sqrt torch_cpu_amd >> "$OUT/adam_k${K}_$L.jsonl" 2>> "$OUT/err.log" || exit $?
    done
    for K in 1 2 3; do
      timeout -k 10 200 $B --clients $K >> "$OUT/plain_k${K}_$L.jsonl" 2>> "$OUT/err.log" || exit $?
    done
    echo "round $R $L done"
  done
done
unset NVFLARE_AMD_FEDAVG_LIB
timeout -k 10 600 python -u bench.py > "$OUT/bench.jsonl" 2> "$OUT/bench.err" || exit $?
echo done
