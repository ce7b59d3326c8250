#!/bin/bash
# round 6, GPU session 19: s18's A/B again with every epilogue starting from zeroed states (s18 ran Adam on RMSprop's
# states: a negative exp_avg_sq sends every unit down the sqrt's rare path) -- RMSprop (momentum 0.9, not centered)
# and Adam, LDS-DMA form (variant 0) against the per-tile form (4), 1-3 clients x 1e9
set -u
O=gpurun_out/r06_s19
mkdir -p $O
export TMPDIR=/tmp
for K in 1 2 3; do
  timeout -k 10 300 python -u tools/ab_variants.py --clients $K --params 1e9 --variants 0,4 \
      --epilogues rmsprop,adam --rounds 3 --reps 10 --check --prewarm-s 5 \
      --sqrt torch_cpu_amd > $O/ab_k$K.jsonl 2>&1 || { echo "ab K=$K rc=$?"; tail -20 $O/ab_k$K.jsonl; exit 1; }
  grep summary $O/ab_k$K.jsonl | python -c "import sys,json; [print(d['clients'], d['epilogue'], d['variant'], d['frac_8TBps']) for d in map(json.loads, sys.stdin)]"
done
