# GPU session 5 (round 5).
#   1. the fused per-tile form at 2 / 3 clients x 5e8 (Adam, AMD-host sqrt), alternating processes, 3 rounds: prod
#      (epilogue arithmetic kEmFast, operands loaded after the clients), tilee (kEmElem), pipe2 (the next tile's
#      operands prefetched with its clients), pipe2e (both);
#   2. config 5 (64 x 1e9, fused Adam) prod vs pf2 (the burst epilogue phase's operands two tiles ahead), 3 rounds;
#   3. the every-kind 2-3-client fused tests on the product library;
#   4. the register-held few-client fused form (A/B only, nvflare_amd/lib/ab/epifew.so) at TWO blocks per CU (2 / 3 / 4
#      register-held tiles) against the per-tile form, interleaved in one process, outputs checked bit-equal.
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05_s5
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fedopt.py -m gpu -q -k "few_client or variants_multi" --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_fedopt.log" 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
A="--also none --no-cpu-baseline --steps 20 --warmup 3 --epilogue adam --sqrt torch_cpu_amd"
for R in 1 2 3; do
  for L in prod tilee pipe2 pipe2e; do
    if [ $L = prod ]; then unset NVFLARE_AMD_FEDAVG_LIB; else export NVFLARE_AMD_FEDAVG_LIB=$GRAFT_REPO_ROOT/nvflare_amd/lib/ab/$L.so; fi
    for K in 2 3; do
      timeout -k 10 200 python -u bench.py $A --params 5e8 --clients $K >> "$OUT/adam_k${K}_$L.jsonl" 2>> "$OUT/err.log" || exit $?
    done
  done
  for L in prod pf2; do
    if [ $L = prod ]; then unset NVFLARE_AMD_FEDAVG_LIB; else export NVFLARE_AMD_FEDAVG_LIB=$GRAFT_REPO_ROOT/nvflare_amd/lib/ab/$L.so; fi
    timeout -k 10 300 python -u bench.py --config 5 --also none --no-cpu-baseline --sqrt torch_cpu_amd >> "$OUT/c5_$L.jsonl" 2>> "$OUT/err.log" || exit $?
  done
  echo "round $R done"
done
for K in 2 3; do
  NVFLARE_AMD_FEDAVG_LIB=$GRAFT_REPO_ROOT/nvflare_amd/lib/ab/epifew.so timeout -k 10 300 python -u tools/ab_variants.py --clients $K --params 5e8 --variants 0:0:0,512:0:2,1024:0:2,1536:0:2,1024:0:1 --epilogues adam --sqrt torch_cpu_amd --rounds 3 --check > "$OUT/epifew_k$K.jsonl" 2>> "$OUT/err.log" || exit $?
done
echo done
