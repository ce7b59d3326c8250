# GPU box script (round 3, session 14): the AMD-host sqrt with its callout as a branch (the correctly rounded sqrt
# off the hot path) -- full `pytest -m gpu`, config 5 with the AMD-host and the correctly rounded sqrt interleaved
# (the gap between them is what the branch should shrink; session 13 measured 1.45 points), and the host-resident
# "2h" entry rehearsed at two ranks sharing the GPU (gloo barriers; a flow check, not a measurement).
set -e
OUT=$GRAFT_REPO_ROOT/${1:-gpurun_out/r03_s14}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
for i in 1 2 3; do
  for S in ieee torch_cpu_amd; do
    timeout -k 10 300 python bench.py --config 5 --sqrt $S --no-cpu-baseline > "$OUT/c5_${S}_$i.jsonl" 2> "$OUT/c5_${S}_$i.err"
  done
done
NVFLARE_AMD_BENCH_SHARED_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 2 --warmup 1 --params 5e7 --also 2h --host-resident-params 3e7 --no-cpu-baseline > "$OUT/rehearse_2h_n2.jsonl" 2> "$OUT/rehearse_2h_n2.err"
# config 4's per-GPU shares (256 clients) against single-pass client counts of the same bytes: where does K = 256
# (two chained 128-client passes) lose?
for KP in "256 4.375e7" "128 8.75e7" "64 1.75e8" "256 8.75e7" "128 1.75e8"; do
  set -- $KP
  timeout -k 10 300 python bench.py --clients $1 --params $2 --also none --no-cpu-baseline --steps 20 > "$OUT/k$1_p$2.jsonl" 2> "$OUT/k$1_p$2.err"
done
