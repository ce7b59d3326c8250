# GPU session 14 (round 4): the 16-bit burst kernel with groups of 4 clients under 32 clients (6 from there on):
# 16-bit parity, then bf16 / fp16 lines across client counts.
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04_s14
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_dtypes.py > "$OUT/pytest_dtypes.log" 2>&1 || exit $?
for fmt in bfloat16 float16; do
  for K in 8 16 24 31 32 48 64; do
    P=5e8; [ $K -ge 32 ] && P=1e9
    timeout -k 10 180 python -u tools/bench_narrow.py --fmt $fmt --clients $K --params $P --steps 10 > "$OUT/${fmt}_k$K.jsonl" 2> "$OUT/${fmt}_k$K.err" || exit $?
  done
done
echo done
