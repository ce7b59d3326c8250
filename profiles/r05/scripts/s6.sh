# GPU session 6 (round 5): 3-6 clients x 1e9 (nvflare_amd/lib/ab/few3.so: product + -DFEDAVG_AB_FEW), interleaved in
# one process, outputs checked bit-equal: the default burst form (client count built in) against the few-client kernel
# at 3-4 reads (forms 1-6, fedavg_internal.h kFewAB34: variant bits 9-11 = 1-6) and against the remainder forms
# (bits 9-11 = 7).
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05_s6
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
export NVFLARE_AMD_FEDAVG_LIB=$GRAFT_REPO_ROOT/nvflare_amd/lib/ab/few3.so
for K in 3 4; do
  timeout -k 10 400 python -u tools/ab_variants.py --clients $K --params 1e9 --variants 0,512,1024,1536,2048,2560,3072,3584 --epilogues none --rounds 3 --check > "$OUT/few34_k$K.jsonl" 2>> "$OUT/err.log" || exit $?
done
for K in 5 6; do
  timeout -k 10 300 python -u tools/ab_variants.py --clients $K --params 1e9 --variants 0,3584 --epilogues none --rounds 3 --check > "$OUT/rem_k$K.jsonl" 2>> "$OUT/err.log" || exit $?
done
echo done
