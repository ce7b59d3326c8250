#!/bin/bash
# round 6, GPU session 11: config 5 (64 clients x 1e9, fused Adam, AMD-host sqrt) on the split-epilogue form (A/B library
# -DFEDAVG_AB_FEW, variant bits 9-11 = 1-4: 8 waves per block, waves 4-7 joining the epilogue phase) against the
# product's burst form (0), three interleaved rounds after a 3 s pre-warm, outputs bit-equal; config 3 beside it
set -u
O=gpurun_out/r06_s11
mkdir -p $O
export TMPDIR=/tmp
NVFLARE_AMD_FEDAVG_LIB=nvflare_amd/lib/ab/dma_ab.so timeout -k 10 600 python -u tools/ab_variants.py --clients 64 --params 1e9 --variants 0,512,1024,1536,2048 --epilogues adam,none --rounds 3 --prewarm-s 3 --check --sqrt torch_cpu_amd > $O/ab_c5.jsonl 2> $O/ab_c5.err
echo "rc=$?"
