# GPU box script (round 3, session 8): the fused kernel with 9 LDS-held tiles at one block per CU -- full GPU
# test suite, then config 5 A/B against the 4-LDS-tile form (variant bit 6), both sqrt modes, interleaved.
set -e
OUT=$GRAFT_REPO_ROOT/${1:-gpurun_out/r03_s8}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
for i in 1 2; do
  for v in 0 64; do
    timeout -k 10 300 python bench.py --config 5 --sqrt ieee --variant $v --no-cpu-baseline > "$OUT/c5_ieee_v${v}_$i.jsonl" 2> "$OUT/c5_ieee_v${v}_$i.err"
    timeout -k 10 300 python bench.py --config 5 --sqrt torch_cpu --variant $v --no-cpu-baseline > "$OUT/c5_tsq_v${v}_$i.jsonl" 2> "$OUT/c5_tsq_v${v}_$i.err"
  done
done
