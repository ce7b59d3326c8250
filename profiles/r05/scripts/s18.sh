# GPU session 18 (round 5): (1) the fused kernels split over two units per (mode, finalisation) pair (product
# library): the fused GPU tests; (2) the 16-bit few-client kernel on tile PAIRS (A/B forms 1-2: K x 16 KiB contiguous
# per unit, the fp32 forms' geometry in bytes) against single tiles -- the few-client tests on the A/B library, then
# bf16 x 1e9 at 1 / 2 / 3 clients in torch and copy modes, outputs checked bit-equal.
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05_s18
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/nvflare_amd/lib
T="python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $T tests/test_gpu_fedopt.py tests/test_gpu_fused_wide.py tests/test_gpu_sharded_fedopt.py > "$OUT/pytest_fused.log" 2>&1 || exit $?
NVFLARE_AMD_FEDAVG_LIB=$L/ab/few.so timeout -k 10 900 $T tests/test_gpu_dtypes.py -k "tiled16_few" > "$OUT/pytest_few_ab.log" 2>&1 || exit $?
echo "tests done"
N="python -u tools/bench_narrow.py --params 1e9 --steps 10 --fmt bfloat16 --check --variants 0,512,1024,1536,2048"
for K in 1 2 3; do
  for M in torch copy; do
    NVFLARE_AMD_FEDAVG_LIB=$L/ab/few.so timeout -k 10 300 $N --clients $K --mode $M >> "$OUT/sweep.jsonl" 2>> "$OUT/err.log" || exit $?
  done
done
echo done
