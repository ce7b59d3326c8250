# GPU box script (round 2): full `pytest -m gpu`, smoke(), the default bench line (config 3), config 5 (Adam),
# config 2, a rocprofv3 kernel trace of the config-3 and config-5 commands, and the PMC traffic passes of both.
# Every GPU step has its own time limit; `set -e` ends the script at the first failure.
set -e
OUT=${1:-gpurun_out/r02_round}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
timeout -k 10 300 python bench.py > "$OUT/bench.jsonl" 2> "$OUT/bench.err"
timeout -k 10 300 python bench.py --epilogue adam > "$OUT/bench_config5_adam.jsonl" 2> "$OUT/bench_config5_adam.err"
timeout -k 10 300 python bench.py --clients 8 --params 1.25e8 --steps 50 > "$OUT/bench_config2.jsonl" 2> "$OUT/bench_config2.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rocprof_bench" -o bench -- python bench.py > "$OUT/bench_prof.jsonl" 2> "$OUT/bench_prof.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rocprof_adam" -o adam -- python bench.py --epilogue adam > "$OUT/bench_adam_prof.jsonl" 2> "$OUT/bench_adam_prof.err"
bash tools/gpu_pmc_bench.sh "$OUT/pmc" none adam
