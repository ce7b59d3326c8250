# GPU session 11 (round 5).
#   1. the 16-bit GPU tests on the product library (few-client defaults from session 10; the packed arithmetic now in
#      every 16-bit tile kernel) and the few-client forms' tests on the -DFEDAVG_AB_FEW library;
#   2. the 16-bit burst kernel at 4-64 clients, packed (product) against per-element (HEAD's library, ab/head.so),
#      alternating processes, 2 rounds;
#   3. bf16 1-3 clients: the new defaults and A/B geometries (few.so), outputs checked bit-equal;
#   4. fp32 few-client kernel: FIN_DIV's range check on the tile's max / min |a| (ab/minmax.so, -DFEDAVG_FIN_MINMAX)
#      against the product's per-element check, 1-3 clients x 1e9, 2 rounds; numpy mode (no division) at 1 client;
#      config 3 on both.
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05_s11
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/nvflare_amd/lib
T="python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_gpu_dtypes.py > "$OUT/pytest_dtypes.log" 2>&1 || exit $?
NVFLARE_AMD_FEDAVG_LIB=$L/ab/few.so timeout -k 10 600 $T tests/test_gpu_dtypes.py -k few_client > "$OUT/pytest_few_ab.log" 2>&1 || exit $?
echo "tests done"
for R in 1 2; do
  for K in 4 8 16; do
    timeout -k 10 300 python -u tools/bench_narrow.py --clients $K --params 1e9 --fmt bfloat16 --steps 10 >> "$OUT/narrow_prod.jsonl" 2>> "$OUT/err.log" || exit $?
    NVFLARE_AMD_FEDAVG_LIB=$L/ab/head.so timeout -k 10 300 python -u tools/bench_narrow.py --clients $K --params 1e9 --fmt bfloat16 --steps 10 >> "$OUT/narrow_head.jsonl" 2>> "$OUT/err.log" || exit $?
  done
  timeout -k 10 300 python -u tools/bench_narrow.py --clients 64 --params 2.5e8 --fmt bfloat16 --steps 10 >> "$OUT/narrow_prod.jsonl" 2>> "$OUT/err.log" || exit $?
  NVFLARE_AMD_FEDAVG_LIB=$L/ab/head.so timeout -k 10 300 python -u tools/bench_narrow.py --clients 64 --params 2.5e8 --fmt bfloat16 --steps 10 >> "$OUT/narrow_head.jsonl" 2>> "$OUT/err.log" || exit $?
  timeout -k 10 300 python -u tools/bench_narrow.py --clients 8 --params 1e9 --fmt float16 --mode numpy --steps 10 >> "$OUT/narrow_prod.jsonl" 2>> "$OUT/err.log" || exit $?
  NVFLARE_AMD_FEDAVG_LIB=$L/ab/head.so timeout -k 10 300 python -u tools/bench_narrow.py --clients 8 --params 1e9 --fmt float16 --mode numpy --steps 10 >> "$OUT/narrow_head.jsonl" 2>> "$OUT/err.log" || exit $?
done
echo "narrow done"
for K in 1 2 3; do
  NVFLARE_AMD_FEDAVG_LIB=$L/ab/few.so timeout -k 10 300 python -u tools/bench_narrow.py --clients $K --params 1e9 --fmt bfloat16 --steps 10 --variants 0,512,1024,1536,2048 --check >> "$OUT/bf16_sweep.jsonl" 2>> "$OUT/err.log" || exit $?
done
echo "sweep done"
B="python -u bench.py --also none --no-cpu-baseline --params 1e9"
for R in 1 2; do
  for K in 1 2 3; do
    timeout -k 10 300 $B --clients $K >> "$OUT/f32_prod.jsonl" 2>> "$OUT/err.log" || exit $?
    NVFLARE_AMD_FEDAVG_LIB=$L/ab/minmax.so timeout -k 10 300 $B --clients $K >> "$OUT/f32_minmax.jsonl" 2>> "$OUT/err.log" || exit $?
  done
  timeout -k 10 300 $B --clients 1 --mode numpy >> "$OUT/f32_numpy.jsonl" 2>> "$OUT/err.log" || exit $?
done
timeout -k 10 300 python -u bench.py --also none --no-cpu-baseline >> "$OUT/c3_prod.jsonl" 2>> "$OUT/err.log" || exit $?
NVFLARE_AMD_FEDAVG_LIB=$L/ab/minmax.so timeout -k 10 300 python -u bench.py --also none --no-cpu-baseline >> "$OUT/c3_minmax.jsonl" 2>> "$OUT/err.log" || exit $?
echo done
