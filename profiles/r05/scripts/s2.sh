# GPU session 2 (round 5).
#   1. pytest -m gpu on the product library (session 1 stopped at its first failure: a tile-width A/B case);
#   2. few-client kernel geometry sweep (nvflare_amd/lib/ab/few.so: product + -DFEDAVG_AB_FEW), 1 and 2 clients x 1e9,
#      forms 0-6 interleaved in one process, outputs checked bit-equal (tools/ab_variants.py --check);
#   3. the read/write mix ceilings of 1 and 2 reads per write on this box (tools/hbm_mix_probe.py --preset few);
#   4. fused Adam epilogue A/B, alternating processes, 3 rounds, 2 / 3 clients x 5e8 (per-tile form) and 64 x 2.5e8
#      (burst form): head (round 4 final), prod (one branch per column group), epiexact (round 4's per-element
#      branches on the round-5 tree), epiieee (per-element epilogue, IEEE divisions: round 3's arithmetic).
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05_s2
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for K in 1 2; do
  NVFLARE_AMD_FEDAVG_LIB=$GRAFT_REPO_ROOT/nvflare_amd/lib/ab/few.so timeout -k 10 300 python -u tools/ab_variants.py --clients $K --params 1e9 --variants 0,512,1024,1536,2048,2560,3072 --epilogues none --rounds 3 --check > "$OUT/few_k$K.jsonl" 2>> "$OUT/err.log" || exit $?
done
echo "few sweep done"
timeout -k 10 300 python -u tools/hbm_mix_probe.py --preset few --params 5e8 --rounds 3 > "$OUT/mix_few.jsonl" 2>> "$OUT/err.log" || exit $?
echo "probe done"
B="python -u $GRAFT_REPO_ROOT/bench.py --also none --no-cpu-baseline --steps 20 --warmup 3 --epilogue adam --sqrt torch_cpu_amd"
for R in 1 2 3; do
  for L in head prod epiexact epiieee; do
    if [ $L = prod ]; then unset NVFLARE_AMD_FEDAVG_LIB; else export NVFLARE_AMD_FEDAVG_LIB=$GRAFT_REPO_ROOT/nvflare_amd/lib/ab/$L.so; fi
    for K in 2 3; do
      timeout -k 10 200 $B --params 5e8 --clients $K >> "$OUT/adam_k${K}_$L.jsonl" 2>> "$OUT/err.log" || exit $?
    done
    timeout -k 10 200 $B --params 2.5e8 --clients 64 >> "$OUT/adam_k64_$L.jsonl" 2>> "$OUT/err.log" || exit $?
    echo "round $R $L done"
  done
done
echo done
