# GPU session 13 (round 4): the 16-bit burst kernel's client group at 4 (no repeated loads at 8, 12, 16 or 64 clients;
# nvflare_amd/lib/ab/libnvflare_amd_fedavg_nu4.so built with --only fedavg_narrow.hip -D FEDAVG_NARROW_UNROLL=4) against
# the product's 6, interleaved, bf16 / fp16.
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04_s13
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for i in 1 2 3; do
  for u in 6 4; do
    lib=nvflare_amd/lib/libnvflare_amd_fedavg.so
    [ "$u" != 6 ] && lib=nvflare_amd/lib/ab/libnvflare_amd_fedavg_nu$u.so
    for fmt in bfloat16 float16; do
      NVFLARE_AMD_FEDAVG_LIB=$lib timeout -k 10 180 python -u tools/bench_narrow.py --fmt $fmt --steps 10 > "$OUT/nu${u}_${fmt}_k64_$i.jsonl" 2> "$OUT/nu${u}_${fmt}_k64_$i.err" || exit $?
    done
    for K in 8 12 16; do
      NVFLARE_AMD_FEDAVG_LIB=$lib timeout -k 10 180 python -u tools/bench_narrow.py --fmt bfloat16 --clients $K --params 5e8 --steps 10 > "$OUT/nu${u}_bfloat16_k${K}_$i.jsonl" 2> "$OUT/nu${u}_bfloat16_k${K}_$i.err" || exit $?
    done
  done
done
echo done
