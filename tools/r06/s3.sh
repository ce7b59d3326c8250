#!/bin/bash
# round 6, GPU session 3: LDS-DMA form geometry A/B (A/B library -DFEDAVG_AB_FEW: variant bits 9-11 = 1-7 ->
# units per wave per launch 16 / 24 / 32 / 8, the RSQRTPS table by LDS-DMA, the epilogue arithmetic's form; 4 = the
# round-5 per-tile form), fused Adam with the AMD-host sqrt, 1e9 params, three interleaved rounds, outputs bit-equal
set -u
O=gpurun_out/r06_s3
mkdir -p $O
export TMPDIR=/tmp
V=0,4,512,1024,1536,2048,2560,3072,3584
for k in 2 3 1; do
  NVFLARE_AMD_FEDAVG_LIB=nvflare_amd/lib/ab/dma_ab.so timeout -k 10 400 python -u tools/ab_variants.py --clients $k --params 1e9 --variants $V --epilogues adam --rounds 3 --check --sqrt torch_cpu_amd > $O/ab_k$k.jsonl 2> $O/ab_k$k.err || exit $?
done
NVFLARE_AMD_FEDAVG_LIB=nvflare_amd/lib/ab/dma_ab.so timeout -k 10 400 python -u tools/ab_variants.py --clients 2 --params 1e9 --variants 0,4,512 --epilogues adam --rounds 3 --check --sqrt ieee > $O/ab_k2_ieee.jsonl 2> $O/ab_k2_ieee.err
echo "rc=$?"
