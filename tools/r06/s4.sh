#!/bin/bash
# round 6, GPU session 4: LDS-DMA form, units per wave per launch N = 16 / 24 / 32 / 36 / 40 / 44 (RSQRTPS table by
# LDS-DMA; 3584 = N 32 with the table staged by loads), launches without the barrier bit (|16), against the round-5
# per-tile form (4); fused Adam with the AMD-host sqrt, 1e9 params, three interleaved rounds, outputs bit-equal
set -u
O=gpurun_out/r06_s4
mkdir -p $O
export TMPDIR=/tmp
V=0,4,512,1024,1536,2048,2560,3072,3584,1552,2576
for k in 2 3 1; do
  NVFLARE_AMD_FEDAVG_LIB=nvflare_amd/lib/ab/dma_ab.so timeout -k 10 500 python -u tools/ab_variants.py --clients $k --params 1e9 --variants $V --epilogues adam --rounds 3 --check --sqrt torch_cpu_amd > $O/ab_k$k.jsonl 2> $O/ab_k$k.err || exit $?
done
echo "rc=0"
