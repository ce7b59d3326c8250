# GPU session 13 (round 5): the fused per-tile form (2-3 client reads, fused Adam) on half tiles -- 2048-column units,
# 128 VGPRs, so four waves per SIMD fit (ab/half.so: -DFEDAVG_EPI_TILE_CPL=2 -DFEDAVG_EPI_TILE_WAVES=4) -- against the
# product (full tiles, 236 VGPRs, two waves per SIMD).  (1) the fused GPU tests on half.so; (2) Adam at 2 / 3 clients x
# 1e9, AMD-host sqrt, alternating processes, 2 rounds: product default, half.so at 2 / 3 / 4 blocks per CU.
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05_s13
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/nvflare_amd/lib
NVFLARE_AMD_FEDAVG_LIB=$L/ab/half.so timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_fedopt.py tests/test_gpu_fused_wide.py > "$OUT/pytest_half.log" 2>&1 || exit $?
echo "tests done"
A="python -u bench.py --also none --no-cpu-baseline --steps 10 --warmup 3 --params 1e9 --epilogue adam --sqrt torch_cpu_amd"
for R in 1 2; do
  for K in 2 3; do
    timeout -k 10 300 $A --clients $K >> "$OUT/adam_k${K}_prod.jsonl" 2>> "$OUT/err.log" || exit $?
    for B in 2 3 4; do
      NVFLARE_AMD_FEDAVG_LIB=$L/ab/half.so timeout -k 10 300 $A --clients $K --blocks-per-cu $B >> "$OUT/adam_k${K}_half_b$B.jsonl" 2>> "$OUT/err.log" || exit $?
    done
  done
  echo "round $R done"
done
echo done
