#!/bin/bash
# round 6, GPU session 23: the LDS-DMA form's geometry per sqrt kind (NAdam, RAdam, Adagrad, RMSprop with momentum, AMD-host
# sqrt) -- A/B variant bits 9-11 = 1-7 (W4N16, W4N32T, W8N12T, W8N16T, W8N16, W4N24T, W4N40T) against the product
# geometry (0) and the per-tile form (4), 1-3 clients x 1e9, three interleaved rounds, outputs bit-equal
set -u
O=gpurun_out/r06_s23
mkdir -p $O
export TMPDIR=/tmp
V=0,4,512,1024,1536,2048,2560,3072,3584
for K in 2 1 3; do
  NVFLARE_AMD_FEDAVG_LIB=nvflare_amd/lib/ab/few_ab.so timeout -k 10 500 python -u tools/ab_variants.py --clients $K \
      --params 1e9 --variants $V --epilogues nadam,radam,adagrad,rmsprop --rounds 3 --reps 10 --check --prewarm-s 3 \
      --sqrt torch_cpu_amd > $O/ab_k$K.jsonl 2> $O/ab_k$K.err || { echo "ab K=$K rc=$?"; tail -20 $O/ab_k$K.err; exit 1; }
  grep summary $O/ab_k$K.jsonl | python -c "import sys,json; [print(d['clients'], d['epilogue'], d['variant'], d['frac_8TBps']) for d in map(json.loads, sys.stdin)]"
done
