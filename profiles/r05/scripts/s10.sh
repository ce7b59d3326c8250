# GPU session 10 (round 5): the 16-bit few-client burst kernel with packed arithmetic (pack2 / step2: v_pk_* and
# v_cvt_pk_*), after session 9's per-element form (bf16 1 / 2 / 3 clients 62.6 / 68.2 / 73.2 % at the best forms).
# (0) tools/cvt_pk_probe: the packed conversions against the per-element ones, all 2^32 inputs.  (1) the 16-bit GPU
# tests on the product library and the few-client forms' tests on the -DFEDAVG_AB_FEW library
# (nvflare_amd/lib/ab/few.so); (2) bf16 at 1 / 2 / 3 clients x 1e9: the default form against the burst form
# (variant 256) and the A/B geometries (variant bits 9-11 = 1-4), interleaved in one process, outputs checked
# bit-equal; fp16 at 1 / 2 clients, torch and numpy modes, default against burst.
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05_s10
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 120 ./tools/cvt_pk_probe > "$OUT/cvt_pk_probe.json" 2>&1 || exit $?
T="python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_gpu_dtypes.py > "$OUT/pytest_dtypes.log" 2>&1 || exit $?
NVFLARE_AMD_FEDAVG_LIB=$GRAFT_REPO_ROOT/nvflare_amd/lib/ab/few.so timeout -k 10 600 $T tests/test_gpu_dtypes.py -k few_client > "$OUT/pytest_few_ab.log" 2>&1 || exit $?
echo "tests done"
for K in 1 2 3; do
  NVFLARE_AMD_FEDAVG_LIB=$GRAFT_REPO_ROOT/nvflare_amd/lib/ab/few.so timeout -k 10 300 python -u tools/bench_narrow.py --clients $K --params 1e9 --fmt bfloat16 --steps 10 --variants 0,256,512,1024,1536,2048 --check >> "$OUT/bf16_sweep.jsonl" 2>> "$OUT/err.log" || exit $?
done
for K in 1 2; do
  for M in torch numpy; do
    NVFLARE_AMD_FEDAVG_LIB=$GRAFT_REPO_ROOT/nvflare_amd/lib/ab/few.so timeout -k 10 300 python -u tools/bench_narrow.py --clients $K --params 1e9 --fmt float16 --steps 10 --variants 0,256 --check --mode $M >> "$OUT/f16.jsonl" 2>> "$OUT/err.log" || exit $?
  done
done
echo done
