# GPU box script: interleaved same-box A/B of the 16-bit tiled kernel's client unroll (loads in flight per
# lane = unroll x 2 groups).  Variant libraries are built in tools/_ab with -DFEDAVG_NARROW_UNROLL=<u>;
# the product library (unroll 4) is the control.
set -e
OUT=gpurun_out/narrow_unroll
mkdir -p "$OUT"
for i in 1 2; do
  for v in 4 6 8; do
    lib=nvflare_amd/lib/libnvflare_amd_fedavg.so
    [ "$v" != 4 ] && lib=tools/_ab/libfedavg_u$v.so
    for fmt in bfloat16 float16; do
      NVFLARE_AMD_FEDAVG_LIB=$lib timeout -k 10 180 python tools/bench_narrow.py --fmt $fmt --steps 10 \
        | sed "s/^{/{\"unroll\": $v, /" >> "$OUT/ab.jsonl"
    done
  done
done
