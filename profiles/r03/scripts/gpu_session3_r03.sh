# GPU box script (round 3, session 3): torch-CPU sqrt on the device (GPU tests), the box host's own torch sqrt
# (tools/sqrt_probe.py, CPU only), fused Adam bench with the restated sqrt vs the correctly rounded one, then
# the full `pytest -m gpu`.
set -e
OUT=$GRAFT_REPO_ROOT/${1:-gpurun_out/r03_s3}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/sqrt_probe.py --save-table "$OUT/rsqrt14_box.bin" > "$OUT/sqrt_probe_box.jsonl" 2> "$OUT/sqrt_probe_box.err"
timeout -k 10 600 python -u -m pytest tests/test_gpu_torch_sqrt.py tests/test_gpu_fedopt_generator.py tests/test_gpu_fedopt_ctl.py tests/test_gpu_fedopt.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_sqrt.log" 2>&1
timeout -k 10 300 python bench.py --config 5 --sqrt torch_cpu > "$OUT/bench_config5_torchsqrt.jsonl" 2> "$OUT/bench_config5_torchsqrt.err"
timeout -k 10 300 python bench.py --config 5 --sqrt ieee > "$OUT/bench_config5_ieee.jsonl" 2> "$OUT/bench_config5_ieee.err"
timeout -k 10 300 python bench.py --config 5 --sqrt torch_cpu > "$OUT/bench_config5_torchsqrt_2.jsonl" 2> "$OUT/bench_config5_torchsqrt_2.err"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
