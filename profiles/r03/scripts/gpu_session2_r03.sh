# GPU box script (round 3, session 2): client-sharded exchange overlapped with the kernels and the sharded FedOpt
# rebind (GPU tests), the dynamic-burst mix probe at config 2's shape, the client-sharded bench at G = 1 (config 4's
# per-GPU share) and a two-rank gloo rehearsal on the one GPU (host-copied collectives: the overlap, not the rate).
set -e
OUT=$GRAFT_REPO_ROOT/${1:-gpurun_out/r03_s2}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_client_shards.py tests/test_gpu_sharded_fedopt.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_shards.log" 2>&1
MIX_CASES=read,write,burst_r8_l4,burst_r8_l10,dyn_r8_l9_avg12,dyn_r8_l9_avg15,dyn_r8_l4_avg11,dyn_r8_l4_avg12,kernel timeout -k 10 240 python tools/hbm_mix_probe.py --ratio 8 --params 1.25e8 --rounds 5 > "$OUT/mix_probe_dyn.jsonl" 2> "$OUT/mix_probe_dyn.err"
timeout -k 10 300 python tools/bench_client_shards.py > "$OUT/client_shards_g1.jsonl" 2> "$OUT/client_shards_g1.err"
NVFLARE_AMD_BENCH_SHARED_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29535 tools/bench_client_shards.py --clients 64 --params-per-gpu 8e6 --max-peer-mib 16 --steps 3 > "$OUT/client_shards_rehearse_n2.jsonl" 2> "$OUT/client_shards_rehearse_n2.err"
