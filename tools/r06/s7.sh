#!/bin/bash
# round 6, GPU session 7: the product geometry of the LDS-DMA form (8 waves per block at 1-2 client reads, 4 at 3):
# parity suites, then the same-process A/B against the round-5 per-tile form (variant 4) and bench lines
set -u
O=gpurun_out/r06_s7
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_epi_dma.py tests/test_gpu_pair_begin.py tests/test_gpu_fedopt.py tests/test_gpu_fedopt_generator.py tests/test_gpu_fused_wide.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 &&
for k in 2 3 1; do
  timeout -k 10 400 python -u tools/ab_variants.py --clients $k --params 1e9 --variants 0,4 --epilogues adam,sgd,add_base --rounds 3 --prewarm-s 3 --check --sqrt torch_cpu_amd > $O/ab_k$k.jsonl 2> $O/ab_k$k.err || exit $?
done &&
timeout -k 10 200 python -u bench.py --clients 2 --params 1e9 --epilogue adam --no-cpu-baseline --steps 20 --warmup 10 > $O/bench_adam_k2.jsonl 2> $O/bench_adam_k2.err &&
timeout -k 10 200 python -u bench.py --clients 3 --params 1e9 --epilogue adam --no-cpu-baseline --steps 20 --warmup 10 > $O/bench_adam_k3.jsonl 2> $O/bench_adam_k3.err
echo "rc=$?"
