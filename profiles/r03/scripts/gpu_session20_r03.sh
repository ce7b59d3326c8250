# GPU box script (round 3, session 20): the default bench line on the final tree (config 3; also configs 5, 4, 2h,
# 2s, 4x -- 4, 2s and 4x skip at N = 1) and smoke().
set -e
OUT=$GRAFT_REPO_ROOT/${1:-gpurun_out/r03_s20}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
timeout -k 10 400 python bench.py > "$OUT/bench.jsonl" 2> "$OUT/bench.err"
echo "bench seconds: $SECONDS" > "$OUT/bench_seconds.txt"
