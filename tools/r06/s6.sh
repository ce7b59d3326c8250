#!/bin/bash
# round 6, GPU session 6: the LDS-DMA form at 8 waves per block (two per SIMD: A/B variant bits 9-11 = 2-6) against
# 4 waves at N = 32 / 28 (1, 7) and the round-5 per-tile form (4); fused Adam, AMD-host sqrt, 1e9 params, 3 s pre-warm,
# three interleaved rounds, outputs bit-equal
set -u
O=gpurun_out/r06_s6
mkdir -p $O
export TMPDIR=/tmp
V=4,512,1024,1536,2048,2560,3072,3584
for k in 2 3 1; do
  NVFLARE_AMD_FEDAVG_LIB=nvflare_amd/lib/ab/dma_ab.so timeout -k 10 500 python -u tools/ab_variants.py --clients $k --params 1e9 --variants $V --epilogues adam --rounds 3 --prewarm-s 3 --check --sqrt torch_cpu_amd > $O/ab_k$k.jsonl 2> $O/ab_k$k.err || exit $?
done
echo "rc=0"
