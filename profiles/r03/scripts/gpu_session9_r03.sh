# GPU box script (round 3, session 9): launch-overlap A/B for the fused and plain burst kernels -- default vs
# any-order launches (variant bit 4) vs two blocks per CU, interleaved.
set -e
OUT=$GRAFT_REPO_ROOT/${1:-gpurun_out/r03_s9}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
for i in 1 2; do
  timeout -k 10 300 python bench.py --config 5 --no-cpu-baseline > "$OUT/c5_default_$i.jsonl" 2> "$OUT/c5_default_$i.err"
  timeout -k 10 300 python bench.py --config 5 --variant 16 --no-cpu-baseline > "$OUT/c5_anyorder_$i.jsonl" 2> "$OUT/c5_anyorder_$i.err"
  timeout -k 10 300 python bench.py --config 5 --blocks-per-cu 2 --no-cpu-baseline > "$OUT/c5_bpc2_$i.jsonl" 2> "$OUT/c5_bpc2_$i.err"
  timeout -k 10 300 python bench.py --also none --no-cpu-baseline > "$OUT/c3_default_$i.jsonl" 2> "$OUT/c3_default_$i.err"
  timeout -k 10 300 python bench.py --also none --variant 16 --no-cpu-baseline > "$OUT/c3_anyorder_$i.jsonl" 2> "$OUT/c3_anyorder_$i.err"
done
