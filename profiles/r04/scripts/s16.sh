# GPU session 16 (round 4): plain burst kernels with pairs from 5 clients on (the default now): parity, then in one
# process per count the default against four together (variant 2560 = shape 5) at 5-7 clients and pairs (variant
# 1024) against the default four together at 4 clients; config 3 and 2 lines as controls.
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04_s16
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py > "$OUT/pytest_parity.log" 2>&1 || exit $?
for K in 5 6 7; do
  timeout -k 10 300 python -u tools/ab_variants.py --clients $K --params 1e9 --variants 0,2560 --epilogues none --check --rounds 4 > "$OUT/def_k$K.jsonl" 2> "$OUT/def_k$K.err" || exit $?
done
timeout -k 10 300 python -u tools/ab_variants.py --clients 4 --params 1e9 --variants 0,1024 --epilogues none --check --rounds 4 > "$OUT/pairs_k4.jsonl" 2> "$OUT/pairs_k4.err" || exit $?
B="python -u bench.py --also none --no-cpu-baseline"
timeout -k 10 300 $B > "$OUT/c3.jsonl" 2> "$OUT/c3.err" || exit $?
timeout -k 10 300 $B --config 2 --steps 50 > "$OUT/c2.jsonl" 2> "$OUT/c2.err" || exit $?
for K in 5 6 7; do
  timeout -k 10 300 $B --clients $K --params 1e9 > "$OUT/bench_k$K.jsonl" 2> "$OUT/bench_k$K.err" || exit $?
done
echo done
