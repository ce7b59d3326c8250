#!/bin/bash
# round 6, GPU session 2: the LDS-DMA few-client fused form -- parity, then same-process A/Bs against the per-tile form
set -u
O=gpurun_out/r06_s2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 240 python -u tools/r06/debug_dma.py > $O/debug_dma.txt 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_epi_dma.py -x -q --timeout 120 --timeout-method thread > $O/pytest_dma.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_fedopt.py -x -q --timeout 120 --timeout-method thread > $O/pytest_fedopt.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_variants.py --clients 2 --params 1e9 --variants 0,4 --epilogues adam --rounds 3 --check --sqrt torch_cpu_amd > $O/ab_adam_k2.jsonl 2> $O/ab_adam_k2.err &&
timeout -k 10 300 python -u tools/ab_variants.py --clients 3 --params 1e9 --variants 0,4 --epilogues adam --rounds 3 --check --sqrt torch_cpu_amd > $O/ab_adam_k3.jsonl 2> $O/ab_adam_k3.err &&
timeout -k 10 300 python -u tools/ab_variants.py --clients 2 --params 1e9 --variants 0,4 --epilogues sgd,add_base --rounds 3 --check > $O/ab_sgd_k2.jsonl 2> $O/ab_sgd_k2.err &&
timeout -k 10 300 python -u tools/ab_variants.py --clients 1 --params 1e9 --variants 0,4 --epilogues adam --rounds 3 --check --sqrt torch_cpu_amd > $O/ab_adam_k1.jsonl 2> $O/ab_adam_k1.err &&
timeout -k 10 200 python -u bench.py --clients 2 --params 1e9 --epilogue adam --no-cpu-baseline --steps 10 > $O/bench_adam_k2.jsonl 2> $O/bench_adam_k2.err &&
timeout -k 10 200 python -u bench.py --clients 3 --params 1e9 --epilogue adam --no-cpu-baseline --steps 10 > $O/bench_adam_k3.jsonl 2> $O/bench_adam_k3.err
rc=$?
echo "rc=$rc"
exit $rc
