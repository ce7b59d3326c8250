# GPU box script (round 3, session 7): the client-sharded config-4 entry of bench.py rehearsed on one GPU (two
# ranks sharing cuda:0 over gloo: the flow, the bits and the watchdog -- times mean nothing), then the default
# one-GPU bench line (the 4x entry must report "skipped" at N = 1).
set -e
OUT=$GRAFT_REPO_ROOT/${1:-gpurun_out/r03_s7}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
export NVFLARE_AMD_BENCH_SHARED_DEVICE=1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 --params 5e7 --also 4x --client-sharded-params 3e7 --no-cpu-baseline > "$OUT/rehearse_4x.jsonl" 2> "$OUT/rehearse_4x.err"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --steps 2 --warmup 1 --params 5e7 --also 4x --client-sharded-params 3e7 --watchdog-s 0.5 --no-cpu-baseline > "$OUT/rehearse_4x_watchdog.jsonl" 2> "$OUT/rehearse_4x_watchdog.err"
unset NVFLARE_AMD_BENCH_SHARED_DEVICE
timeout -k 10 400 python bench.py > "$OUT/bench.jsonl" 2> "$OUT/bench.err"
