#!/bin/bash
# round 6, GPU session 10: (a) config 4's one-GPU share (256 clients x 43.75 M: two chained 128-client launches) against
# 128 clients x 87.5 M (one pass, the same bytes) and the launch forms (64: 4 LDS tiles; 16: no barrier bit);
# (b) temporal epilogue stores (A/B library -DFEDAVG_EPI_TEMPORAL) for config 5 and the 2-client fused form, processes
# alternating with the product library
set -u
O=gpurun_out/r06_s10
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/ab_variants.py --clients 256 --params 43753472 --variants 0,64 --epilogues none --rounds 3 --prewarm-s 2 > $O/ab_c4share.jsonl 2> $O/ab_c4share.err &&
timeout -k 10 500 python -u tools/ab_variants.py --clients 128 --params 87500000 --variants 0,64 --epilogues none --rounds 3 --prewarm-s 2 > $O/ab_k128.jsonl 2> $O/ab_k128.err &&
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --config 5 --no-cpu-baseline --steps 10 --warmup 3 > $O/c5_prod_$r.jsonl 2> $O/c5_prod_$r.err || exit $?
  NVFLARE_AMD_FEDAVG_LIB=nvflare_amd/lib/ab/epi_temporal.so timeout -k 10 300 python -u bench.py --config 5 --no-cpu-baseline --steps 10 --warmup 3 > $O/c5_temp_$r.jsonl 2> $O/c5_temp_$r.err || exit $?
  timeout -k 10 300 python -u bench.py --clients 2 --params 1e9 --epilogue adam --no-cpu-baseline --steps 20 --warmup 10 > $O/k2_prod_$r.jsonl 2> $O/k2_prod_$r.err || exit $?
  NVFLARE_AMD_FEDAVG_LIB=nvflare_amd/lib/ab/epi_temporal.so timeout -k 10 300 python -u bench.py --clients 2 --params 1e9 --epilogue adam --no-cpu-baseline --steps 20 --warmup 10 > $O/k2_temp_$r.jsonl 2> $O/k2_temp_$r.err || exit $?
done
echo "rc=$?"
