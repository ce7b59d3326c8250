# GPU box script (round 3): full `pytest -m gpu`, smoke(), the default bench line (config 3 + configs 5 / 4 in
# `also`), config 2, the 8:1 mix probe with write-only streams, the 8-bucket result latency (direct egress vs
# concatenation) and a two-rank strong-scaling rehearsal of bench.py on the one GPU (gloo, never a measurement).
# Every GPU step has its own time limit; `set -e` ends the script at the first failure.
set -e
OUT=$GRAFT_REPO_ROOT/${1:-gpurun_out/r03_session}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
timeout -k 10 400 python bench.py > "$OUT/bench.jsonl" 2> "$OUT/bench.err"
timeout -k 10 240 python bench.py --config 2 --steps 50 > "$OUT/bench_config2.jsonl" 2> "$OUT/bench_config2.err"
timeout -k 10 240 python tools/hbm_mix_probe.py --ratio 8 --params 1.25e8 --rounds 5 > "$OUT/mix_probe_r8.jsonl" 2> "$OUT/mix_probe_r8.err"
timeout -k 10 300 python tools/result_latency.py --devices 8 --clients 8 --params 1e9 --rounds 3 > "$OUT/result_latency_8buckets.jsonl" 2> "$OUT/result_latency_8buckets.err"
NVFLARE_AMD_BENCH_SHARED_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --config 5 --global-params 2e8 --steps 5 --warmup 1 > "$OUT/rehearse_n2_strong_adam.jsonl" 2> "$OUT/rehearse_n2_strong_adam.err"
NVFLARE_AMD_BENCH_SHARED_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --clients 256 --global-params 3.5e7 --steps 5 --warmup 1 > "$OUT/rehearse_n2_strong_k256.jsonl" 2> "$OUT/rehearse_n2_strong_k256.err"
