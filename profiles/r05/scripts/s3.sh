# GPU session 3 (round 5).
#   1. the 1 : 1 and 2 : 1 read/write mix ceilings on this box next to the library kernel (tools/hbm_mix_probe.py);
#   2. few-client geometry sweep 2 around session 2's best forms (nvflare_amd/lib/ab/few.so), 1e9 params;
#   3. fused Adam epilogue A/B (session 2 stopped before it): head / prod / epiexact / epiieee, alternating processes;
#   4. bench lines of the product library at 1 / 2 / 3 clients x 1e9, rocprofv3 kernel stats of the 1- and 2-client
#      lines, PMC FETCH_SIZE / WRITE_SIZE passes of both (VERDICT r04 item 3's evidence).
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05_s3
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for R in 1 2; do
  MIX_CASES=read,write,burst_r8_l4,burst_r8_l10,kernel timeout -k 10 300 python -u tools/hbm_mix_probe.py --preset few --ratio $R --params 5e8 --rounds 3 > "$OUT/mix_r$R.jsonl" 2>> "$OUT/err.log" || exit $?
done
echo "probe done"
for K in 1 2; do
  NVFLARE_AMD_FEDAVG_LIB=$GRAFT_REPO_ROOT/nvflare_amd/lib/ab/few.so timeout -k 10 300 python -u tools/ab_variants.py --clients $K --params 1e9 --variants 0,512,1024,1536,2048,2560,3072 --epilogues none --rounds 3 --check > "$OUT/few_k$K.jsonl" 2>> "$OUT/err.log" || exit $?
done
echo "few sweep done"
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
unset NVFLARE_AMD_FEDAVG_LIB
P="python -u $GRAFT_REPO_ROOT/bench.py --also none --no-cpu-baseline --params 1e9"
for K in 1 2 3; do
  timeout -k 10 200 $P --clients $K > "$OUT/bench_k$K.jsonl" 2>> "$OUT/err.log" || exit $?
done
cd /tmp
for K in 1 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rocprof_k$K" -o k$K -- $P --clients $K > "$OUT/bench_k${K}_prof.jsonl" 2>> "$OUT/err.log" || exit $?
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc/k${K}_$C" -o pmc -- $P --clients $K --steps 2 --warmup 1 --spot-check 0 > "$OUT/pmc_k${K}_$C.log" 2>&1 || exit $?
  done
done
echo done
