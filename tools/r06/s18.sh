#!/bin/bash
# round 6, GPU session 18: RMSprop (not centered) on the LDS-DMA few-client form -- parity, then same-process A/B
# against the per-tile form (variant 4) at 1-3 clients x 1e9, momentum 0.9 (three operand streams)
set -u
O=gpurun_out/r06_s18
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_epi_dma.py tests/test_gpu_fedopt.py tests/test_gpu_fedopt_generator.py \
    tests/test_gpu_fuzz_fedopt.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for K in 1 2 3; do
  timeout -k 10 300 python -u tools/ab_variants.py --clients $K --params 1e9 --variants 0,4 \
      --epilogues rmsprop,adam --rounds 3 --reps 10 --check --prewarm-s 5 \
      --sqrt torch_cpu_amd > $O/ab_k$K.jsonl 2>&1 || { echo "ab K=$K rc=$?"; tail -20 $O/ab_k$K.jsonl; exit 1; }
  grep summary $O/ab_k$K.jsonl | python -c "import sys,json; [print(d['clients'], d['epilogue'], d['variant'], d['frac_8TBps']) for d in map(json.loads, sys.stdin)]"
done
