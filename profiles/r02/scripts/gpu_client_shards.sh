# GPU box script: client-sharded ingest -- parity tests (ranks sharing cuda:0 over gloo), the bench at N=1
# (config 4's per-GPU share) and a two-rank shared-device rehearsal of its multi-rank flow.
set -e
OUT=${1:-gpurun_out/client_shards}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python tools/debug_client_shards_nccl.py nccl 16e6 > "$OUT/debug_nccl_16M.log" 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_client_shards.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
timeout -k 10 240 python tools/bench_client_shards.py --clients 64 --params-per-gpu 16e6 --steps 3 > "$OUT/bench_small.jsonl" 2> "$OUT/bench_small.err"
timeout -k 10 300 python tools/bench_client_shards.py > "$OUT/bench_n1.jsonl" 2> "$OUT/bench_n1.err"
NVFLARE_AMD_BENCH_SHARED_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 tools/bench_client_shards.py --clients 16 --params-per-gpu 4e6 --steps 2 > "$OUT/rehearse_n2.jsonl" 2> "$OUT/rehearse_n2.err"
