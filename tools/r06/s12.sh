#!/bin/bash
# round 6, GPU session 12: the split-epilogue form for fused Adam at 64+ clients (config 5) -- parity, the same-process
# A/B against round 5's burst form (product library, variant 1 << 15), the geometry sweep (A/B library, variant bits 9-11
# = 1-5: (4, 9, 4), (4, 9, 5), (3, 9, 4), (4, 9, 3), (5, 9, 3)), then rocprofv3 kernel stats and PMC of config 5
set -u
O=gpurun_out/r06_s12
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests/test_gpu_fused_wide.py tests/test_gpu_fullsize.py tests/test_gpu_epi_dma.py tests/test_gpu_fedopt.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 600 python -u tools/ab_variants.py --clients 64 --params 1e9 --variants 0,32768 --epilogues adam,none --rounds 3 --prewarm-s 3 --check --sqrt torch_cpu_amd > $O/ab_c5_prod.jsonl 2> $O/ab_c5_prod.err &&
NVFLARE_AMD_FEDAVG_LIB=nvflare_amd/lib/ab/dma_ab.so timeout -k 10 600 python -u tools/ab_variants.py --clients 64 --params 1e9 --variants 0,1024,1536,2048,2560 --epilogues adam --rounds 3 --prewarm-s 3 --check --sqrt torch_cpu_amd > $O/ab_c5_split.jsonl 2> $O/ab_c5_split.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rp_c5 -o c5 -- python3 bench.py --config 5 --no-cpu-baseline --steps 10 --spot-check 0 > $O/rp_c5.jsonl 2> $O/rp_c5.err &&
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_c5_fetch -o f -- python3 bench.py --config 5 --no-cpu-baseline --steps 2 --warmup 1 --spot-check 0 > /dev/null 2> $O/pmc_c5_fetch.err &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_c5_write -o w -- python3 bench.py --config 5 --no-cpu-baseline --steps 2 --warmup 1 --spot-check 0 > /dev/null 2> $O/pmc_c5_write.err
echo "rc=$?"
