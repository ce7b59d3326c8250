# GPU session 8 (round 5): (1) the self-launched multi-rank bench on the box -- `python bench.py --gpus 2` with no
# WORLD_SIZE, both ranks on cuda:0 (NVFLARE_AMD_BENCH_SHARED_DEVICE=1: gloo barriers; RCCL refuses two ranks on one
# device), a small config-3 workload plus the 2h / 2s entries: the launcher path the driver's 8-GPU run takes;
# (2) the 16-bit and fp64 kernels at 1 / 2 / 8 clients (tiled slabs), for the few-client picture of the other dtypes.
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05_s8
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
NVFLARE_AMD_BENCH_SHARED_DEVICE=1 timeout -k 10 600 python -u bench.py --gpus 2 --clients 64 --params 1e8 --steps 5 --warmup 2 --also 2h,2s --host-resident-params 2e7 --no-cpu-baseline > "$OUT/spawn2.jsonl" 2> "$OUT/spawn2.err" || exit $?
echo "spawn done"
for K in 1 2 8; do
  timeout -k 10 300 python -u tools/bench_narrow.py --clients $K --params 1e9 --fmt bfloat16 --steps 10 >> "$OUT/bf16.jsonl" 2>> "$OUT/err.log" || exit $?
  timeout -k 10 300 python -u tools/bench_generic.py --clients $K --params 5e8 --dtype float64 --layout tiled --steps 10 >> "$OUT/f64.jsonl" 2>> "$OUT/err.log" || exit $?
done
echo done
