#!/bin/bash
# Blocks per CU of the plain and fused-epilogue (Adam, SGD) burst kernels over client counts: 0 = library
# default, 1, 2 -- interleaved in one process per client count (tools/ab_variants.py).
set -o pipefail
mkdir -p gpurun_out/abe
for kp in 8:1000000000 16:1000000000 32:1000000000 64:1000000000; do
  K=${kp%%:*}; P=${kp##*:}
  f=gpurun_out/abe/k${K}.jsonl
  timeout -k 10 240 python -u tools/ab_variants.py --clients $K --params $P --variants 0:0:0,0:0:1,0:0:2 --epilogues none,adam,sgd --rounds 3 --reps 5 > $f 2>&1 || { tail -5 $f; exit 1; }
  echo "K=$K"; grep summary $f || grep median $f | head
done
