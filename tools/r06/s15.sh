#!/bin/bash
# round 6, GPU session 15: the LDS-DMA few-client form for every optimizer kind but RMSprop -- parity (DMA against the
# oracle and the per-tile form), then a same-process A/B per kind at 1-3 clients x 1e9 (variant 0 = DMA, 4 = per-tile)
set -u
O=gpurun_out/r06_s15
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_epi_dma.py tests/test_gpu_fedopt.py tests/test_gpu_fedopt_generator.py \
    tests/test_gpu_fuzz_fedopt.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for K in 1 2 3; do
  timeout -k 10 400 python -u tools/ab_variants.py --clients $K --params 1e9 --variants 0,4 \
      --epilogues adagrad,adamax,nadam,radam,rprop,asgd --rounds 3 --reps 10 --check --prewarm-s 5 \
      --sqrt torch_cpu_amd > $O/ab_k$K.jsonl 2>&1 || { echo "ab K=$K rc=$?"; tail -20 $O/ab_k$K.jsonl; exit 1; }
  grep summary $O/ab_k$K.jsonl
done
