# GPU session 4 (round 5).
#   1. pytest -m gpu on the product library (new: the few-client fused form for 2-3 reads, 2-read plain default G = 1);
#   2. the fused Adam 2-3-client bisect on ONE box, alternating processes, 3 rounds, 5e8 params, --steps 10 (round 3's
#      command): round 3's tree (229fc6e, its own bench.py and library, abtree/r3) with its per-tile form (--variant 8)
#      and its pipelined per-tile form (--variant 4); round 4's final library (head.so) with --variant 8 and its default
#      (pipelined per-tile); the product library (the few-client fused form);
#   3. the few-client fused form's register-tile sweep (2 / 3 / 4 / 5 / 6 / 8 tiles) and the plain few-client sweep 3
#      (nvflare_amd/lib/ab/few.so), interleaved in one process, outputs checked bit-equal.
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05_s4
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
A="--also none --no-cpu-baseline --steps 10 --warmup 3 --params 5e8 --epilogue adam --sqrt torch_cpu_amd"
for R in 1 2 3; do
  for K in 2 3; do
    for V in 8 4; do
      timeout -k 10 200 python -u abtree/r3/bench.py $A --clients $K --variant $V >> "$OUT/adam_k${K}_r3_v$V.jsonl" 2>> "$OUT/err.log" || exit $?
      NVFLARE_AMD_FEDAVG_LIB=$GRAFT_REPO_ROOT/nvflare_amd/lib/ab/head.so timeout -k 10 200 python -u bench.py $A --clients $K --variant $((V == 4 ? 0 : 8)) >> "$OUT/adam_k${K}_head_v$V.jsonl" 2>> "$OUT/err.log" || exit $?
    done
    timeout -k 10 200 python -u bench.py $A --clients $K >> "$OUT/adam_k${K}_prod.jsonl" 2>> "$OUT/err.log" || exit $?
  done
  echo "round $R done"
done
for K in 2 3; do
  NVFLARE_AMD_FEDAVG_LIB=$GRAFT_REPO_ROOT/nvflare_amd/lib/ab/few.so timeout -k 10 300 python -u tools/ab_variants.py --clients $K --params 5e8 --variants 0,512,1024,1536,2048,2560 --epilogues adam --sqrt torch_cpu_amd --rounds 3 --check > "$OUT/epifew_k$K.jsonl" 2>> "$OUT/err.log" || exit $?
done
for K in 1 2; do
  NVFLARE_AMD_FEDAVG_LIB=$GRAFT_REPO_ROOT/nvflare_amd/lib/ab/few.so timeout -k 10 300 python -u tools/ab_variants.py --clients $K --params 1e9 --variants 0,512,1024,1536,2048,2560,3072 --epilogues none --rounds 3 --check > "$OUT/few_k$K.jsonl" 2>> "$OUT/err.log" || exit $?
done
echo done
