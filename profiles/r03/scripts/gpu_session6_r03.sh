# GPU box script (round 3, session 6): raw torch CPU sqrt of the box host for offline analysis (CPU only), the
# torch-sqrt epilogues with the LDS-staged segment table (GPU tests + fused Adam bench, restated vs correctly
# rounded sqrt, interleaved).
set -e
OUT=$GRAFT_REPO_ROOT/${1:-gpurun_out/r03_s6}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 python tools/sqrt_dump.py "$OUT/sqrt_dump" > "$OUT/sqrt_dump.log" 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_torch_sqrt.py tests/test_gpu_fuzz_fedopt.py tests/test_gpu_fedopt_generator.py tests/test_gpu_fedopt.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_sqrt.log" 2>&1
for i in 1 2; do
  timeout -k 10 300 python bench.py --config 5 --sqrt ieee --no-cpu-baseline > "$OUT/bench_config5_ieee_$i.jsonl" 2> "$OUT/bench_config5_ieee_$i.err"
  timeout -k 10 300 python bench.py --config 5 --sqrt torch_cpu --no-cpu-baseline > "$OUT/bench_config5_torchsqrt_$i.jsonl" 2> "$OUT/bench_config5_torchsqrt_$i.err"
done
