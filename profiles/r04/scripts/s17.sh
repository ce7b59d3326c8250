# GPU session 17 (round 4): pairs as the default at 4 clients too; 3 clients as a pair then the third (variant 1024)
# against the three together; parity; 4-client default against four together (variant 2560).
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04_s17
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py > "$OUT/pytest_parity.log" 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab_variants.py --clients 3 --params 1e9 --variants 0,1024,8 --epilogues none --check --rounds 4 > "$OUT/split_k3.jsonl" 2> "$OUT/split_k3.err" || exit $?
timeout -k 10 300 python -u tools/ab_variants.py --clients 4 --params 1e9 --variants 0,2560 --epilogues none --check --rounds 4 > "$OUT/def_k4.jsonl" 2> "$OUT/def_k4.err" || exit $?
B="python -u bench.py --also none --no-cpu-baseline"
for K in 3 4; do
  timeout -k 10 300 $B --clients $K --params 1e9 > "$OUT/bench_k$K.jsonl" 2> "$OUT/bench_k$K.err" || exit $?
done
echo done
