# GPU box script (round 3, session 23): four ranks sharing the GPU (gloo barriers and gloo exchange; a flow check of
# the N = 4 bench, not a measurement) with every default `also` entry (5, 4, 2h, 2s, 4x) at reduced sizes -- the
# earlier rehearsals ran two ranks.
set -e
OUT=$GRAFT_REPO_ROOT/${1:-gpurun_out/r03_s23}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
NVFLARE_AMD_BENCH_SHARED_DEVICE=1 timeout -k 10 480 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29553 bench.py --gpus 4 --steps 2 --warmup 1 --params 5e7 --also 5,4,2h,2s,4x --host-resident-params 2e7 --client-sharded-params 2e7 --watchdog-s 200 --no-cpu-baseline > "$OUT/rehearse_all_n4.jsonl" 2> "$OUT/rehearse_all_n4.err"
