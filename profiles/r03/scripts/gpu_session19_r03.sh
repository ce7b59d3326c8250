# GPU box script (round 3, session 19): the 2s entry -- config 2 host-resident in ONE process over all ranks' GPUs
# (WeightedAggregationHelper(devices=...)) -- rehearsed with two ranks sharing the GPU (devices [0, 0]; a flow check,
# not a measurement) after the 2h entry, and at one rank (skipped), plus the in-process two-bucket round on one GPU
# at config 2's full size.
set -e
OUT=$GRAFT_REPO_ROOT/${1:-gpurun_out/r03_s19}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
NVFLARE_AMD_BENCH_SHARED_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 3 --warmup 1 --params 5e7 --also 2h,2s --watchdog-s 200 --no-cpu-baseline > "$OUT/rehearse_2h_2s_n2.jsonl" 2> "$OUT/rehearse_2h_2s_n2.err"
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --params 5e7 --also 2s --no-cpu-baseline > "$OUT/n1_2s.jsonl" 2> "$OUT/n1_2s.err"
