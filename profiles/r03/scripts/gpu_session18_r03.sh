# GPU box script (round 3, session 18): the host-resident config-2 round in its steady state (three untimed rounds)
# through bench's 2h entry, and per-round accept / get_result times from tools/e2e_bench.py (1 key and 437 keys).
set -e
OUT=$GRAFT_REPO_ROOT/${1:-gpurun_out/r03_s18}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python bench.py --clients 8 --params 1.25e8 --also 2h --no-cpu-baseline > "$OUT/bench_2h.jsonl" 2> "$OUT/bench_2h.err"
timeout -k 10 300 python tools/e2e_bench.py --clients 8 --params 125e6 --rounds 6 > "$OUT/e2e_numpy_1key.jsonl" 2> "$OUT/e2e_numpy_1key.err"
timeout -k 10 300 python tools/e2e_bench.py --clients 8 --params 125e6 --rounds 6 --keys 437 > "$OUT/e2e_numpy_437keys.jsonl" 2> "$OUT/e2e_numpy_437keys.err"
