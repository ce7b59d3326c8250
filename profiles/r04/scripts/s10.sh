# GPU session 10 (round 4): the 16-bit burst kernel's client group (loads in flight per lane = unroll x 2) at 3 and 4
# against the product's 6 (libraries built with tools/build_rev_lib.py --only fedavg_narrow.hip -D
# FEDAVG_NARROW_UNROLL=u), bf16 / fp16 at 64 x 1e9 and 8 x 5e8, interleaved; the few-client fused forms' per-tile
# kernel with and without the cross-tile pipeline (variant 8 / 4), five rounds.
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04_s10
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for i in 1 2; do
  for u in 6 3; do
    lib=nvflare_amd/lib/libnvflare_amd_fedavg.so
    [ "$u" != 6 ] && lib=nvflare_amd/lib/ab/libnvflare_amd_fedavg_nu$u.so
    for fmt in bfloat16 float16; do
      NVFLARE_AMD_FEDAVG_LIB=$lib timeout -k 10 180 python -u tools/bench_narrow.py --fmt $fmt --steps 10 > "$OUT/nu${u}_${fmt}_k64_$i.jsonl" 2> "$OUT/nu${u}_${fmt}_k64_$i.err" || exit $?
    done
    NVFLARE_AMD_FEDAVG_LIB=$lib timeout -k 10 180 python -u tools/bench_narrow.py --fmt bfloat16 --clients 8 --params 5e8 --steps 10 > "$OUT/nu${u}_bfloat16_k8_$i.jsonl" 2> "$OUT/nu${u}_bfloat16_k8_$i.err" || exit $?
  done
done
for K in 1 2 3; do
  timeout -k 10 300 python -u tools/ab_variants.py --clients $K --params 5e8 --variants 8,4 --epilogues adam --sqrt torch_cpu_amd --check --rounds 5 > "$OUT/epi_pipe_k$K.jsonl" 2> "$OUT/epi_pipe_k$K.err" || exit $?
done
echo done
