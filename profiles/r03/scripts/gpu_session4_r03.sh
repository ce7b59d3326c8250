# GPU box script (round 3, session 4): the box host's torch sqrt against candidate sequences (CPU only), the
# torch-sqrt epilogues without scratch (GPU tests + fused Adam bench, restated vs correctly rounded sqrt,
# interleaved), the write cache-policy probe, and the default bench line.
set -e
OUT=$GRAFT_REPO_ROOT/${1:-gpurun_out/r03_s4}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/sqrt_probe.py > "$OUT/sqrt_probe_box.jsonl" 2> "$OUT/sqrt_probe_box.err"
timeout -k 10 600 python -u -m pytest tests/test_gpu_torch_sqrt.py tests/test_gpu_fuzz_fedopt.py tests/test_gpu_fedopt_generator.py tests/test_gpu_fedopt.py tests/test_gpu_sharded_fedopt.py tests/test_gpu_deferred.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_sqrt.log" 2>&1
for i in 1 2; do
  timeout -k 10 300 python bench.py --config 5 --sqrt ieee --no-cpu-baseline > "$OUT/bench_config5_ieee_$i.jsonl" 2> "$OUT/bench_config5_ieee_$i.err"
  timeout -k 10 300 python bench.py --config 5 --sqrt torch_cpu --no-cpu-baseline > "$OUT/bench_config5_torchsqrt_$i.jsonl" 2> "$OUT/bench_config5_torchsqrt_$i.err"
done
MIX_CASES=read,write,write_aux0,write_aux2,write_aux16,write_aux17,burst_r8_l4,kernel timeout -k 10 240 python tools/hbm_mix_probe.py --ratio 8 --params 1.25e8 --rounds 5 > "$OUT/mix_probe_writes.jsonl" 2> "$OUT/mix_probe_writes.err"
timeout -k 10 400 python bench.py > "$OUT/bench.jsonl" 2> "$OUT/bench.err"
