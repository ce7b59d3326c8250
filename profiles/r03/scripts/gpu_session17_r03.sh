# GPU box script (round 3, session 17): the guarded `also` entries in sequence after the watchdog refactor -- two ranks
# sharing the GPU (gloo barriers and gloo exchange; a flow check, not a measurement) run the host-resident config-2
# entry and then the client-sharded config-4 entry, each under its own watchdog; then a one-rank run of the same pair
# (4x skips at N = 1).
set -e
OUT=$GRAFT_REPO_ROOT/${1:-gpurun_out/r03_s17}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
NVFLARE_AMD_BENCH_SHARED_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29551 bench.py --gpus 2 --steps 2 --warmup 1 --params 5e7 --also 2h,4x --host-resident-params 3e7 --client-sharded-params 3e7 --watchdog-s 120 --no-cpu-baseline > "$OUT/rehearse_2h_4x_n2.jsonl" 2> "$OUT/rehearse_2h_4x_n2.err"
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --params 5e7 --also 2h,4x --host-resident-params 3e7 --no-cpu-baseline > "$OUT/n1_2h_4x.jsonl" 2> "$OUT/n1_2h_4x.err"
