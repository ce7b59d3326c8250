#!/bin/bash
# round 6, GPU session 26: four operand streams on the LDS-DMA form (Adam with amsgrad, centered RMSprop with momentum;
# 4 waves x 24 units) -- parity, then against the per-tile form (variant 4) at 1-3 clients x 1e9
set -u
O=gpurun_out/r06_s26
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests/test_gpu_epi_dma.py tests/test_gpu_fedopt.py tests/test_gpu_torch_sqrt.py \
    tests/test_gpu_fedopt_generator.py tests/test_gpu_fuzz_fedopt.py tests/test_gpu_fedopt_ctl.py -x -q --timeout 300 \
    --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for K in 1 2 3; do
  timeout -k 10 300 python -u tools/ab_variants.py --clients $K --params 1e9 --variants 0,4 \
      --epilogues adam_ams,rmsprop_c,adam --rounds 3 --reps 10 --check --prewarm-s 3 \
      --sqrt torch_cpu_amd > $O/ab_k$K.jsonl 2>&1 || { echo "ab K=$K rc=$?"; tail -20 $O/ab_k$K.jsonl; exit 1; }
  grep summary $O/ab_k$K.jsonl | python -c "import sys,json; [print(d['clients'], d['epilogue'], d['variant'], d['frac_8TBps']) for d in map(json.loads, sys.stdin)]"
done
