#!/bin/bash
# round 6, GPU session 9: SGD / ADD_BASE on 4 waves x 40 units -- parity; then where the operand buffers sit relative to
# the client slab (byte shifts 0 .. 2 MiB + 4 KiB of p / m / v) for the per-tile (4) and LDS-DMA (0) forms, 2 clients
set -u
O=gpurun_out/r06_s9
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_epi_dma.py tests/test_gpu_fedopt.py tests/test_gpu_fedopt_generator.py tests/test_gpu_deferred.py tests/test_gpu_sharded_fedopt.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 500 python -u tools/ab_variants.py --clients 2 --params 1e9 --variants 0,4 --epilogues adam --rounds 3 --prewarm-s 2 --op-shifts 0,256,4096,65536,1048576,2101248 --sqrt torch_cpu_amd > $O/shift_adam_k2.jsonl 2> $O/shift_adam_k2.err &&
timeout -k 10 500 python -u tools/ab_variants.py --clients 2 --params 1e9 --variants 0,4 --epilogues sgd,add_base --rounds 3 --prewarm-s 2 --check > $O/ab_sgd_k2.jsonl 2> $O/ab_sgd_k2.err &&
timeout -k 10 500 python -u tools/ab_variants.py --clients 1 --params 1e9 --variants 0,4 --epilogues sgd,add_base --rounds 3 --check > $O/ab_sgd_k1.jsonl 2> $O/ab_sgd_k1.err &&
timeout -k 10 500 python -u tools/ab_variants.py --clients 3 --params 1e9 --variants 0,4 --epilogues sgd,add_base --rounds 3 --check > $O/ab_sgd_k3.jsonl 2> $O/ab_sgd_k3.err
echo "rc=$?"
