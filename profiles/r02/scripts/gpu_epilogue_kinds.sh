# GPU box script: config-5 bench line (64 clients x 1e9 fp32 params, aggregation + fused server optimizer) for
# each Adam-family epilogue, then a rocprofv3 kernel-trace of the NAdam run.  Every GPU step has its own limit.
set -e
OUT=gpurun_out/epi_kinds
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for e in adam adamax nadam radam sgd; do
  timeout -k 10 240 python bench.py --epilogue $e --steps 10 --warmup 2 --no-cpu-baseline >> "$OUT/bench_epilogues.jsonl" 2>> "$OUT/bench.err"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rocprof_nadam" -o nadam -- python bench.py --epilogue nadam --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/bench_nadam_prof.jsonl" 2> "$OUT/bench_nadam_prof.err"
