# GPU box script: the round-end tiers on the current tree -- full `pytest -m gpu`, smoke(), the default bench
# line and a rocprofv3 kernel-trace of the same bench command.  Every GPU step has its own time limit and
# `set -e` ends the script at the first failure.
set -e
OUT=${1:-gpurun_out/full_check}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
timeout -k 10 300 python bench.py > "$OUT/bench.jsonl" 2> "$OUT/bench.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rocprof_bench" -o bench -- python bench.py > "$OUT/bench_prof.jsonl" 2> "$OUT/bench_prof.err"
