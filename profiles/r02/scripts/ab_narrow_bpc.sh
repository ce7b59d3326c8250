#!/bin/bash
# 16-bit burst kernel: blocks per CU 1 vs 2 over client counts (bf16 / fp16 torch mode, fp16 numpy mode),
# interleaved in one process per case (tools/bench_narrow.py: medians of 3 rounds).
set -o pipefail
mkdir -p gpurun_out/abnb
for kp in 8:250000000 8:4000000000 16:2000000000 21:1500000000 32:2000000000 64:1000000000 128:500000000; do
  K=${kp%%:*}; P=${kp##*:}
  for fm in bfloat16:torch float16:torch float16:numpy; do
    fmt=${fm%%:*}; mode=${fm##*:}
    [ $mode = numpy ] && [ $K != 64 ] && [ $K != 8 ] && continue
    f=gpurun_out/abnb/k${K}_p${P}_${fmt}_${mode}.jsonl
    timeout -k 10 150 python -u tools/bench_narrow.py --fmt $fmt --mode $mode --clients $K --params $P --steps 10 --blocks-per-cu 1,2 > $f 2>&1 || { tail -5 $f; exit 1; }
    echo "K=$K P=$P $fmt $mode: $(grep -o '"blocks_per_cu": [0-9]*\|"frac_of_8TBs": [0-9.]*' $f | tr '\n' ' ')"
  done
done
