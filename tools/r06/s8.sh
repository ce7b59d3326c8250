#!/bin/bash
# round 6, GPU session 8: (a) LDS-DMA geometry for SGD and ADD_BASE at 1-3 client reads (A/B library, variant bits 9-11:
# 1 W4 N16, 2 W4 N32 +table DMA, 3 W8 N12, 4 W8 N16, 5 W8 N16 (table by loads), 6 W4 N24, 7 W4 N40; 0 = product);
# (b) rocprofv3 kernel stats and PMC FETCH_SIZE / WRITE_SIZE of the product's fused Adam at 2 and 3 clients
set -u
O=gpurun_out/r06_s8
mkdir -p $O
export TMPDIR=/tmp
V=0,512,1024,1536,2048,2560,3072,3584
for k in 2 3 1; do
  NVFLARE_AMD_FEDAVG_LIB=nvflare_amd/lib/ab/dma_ab.so timeout -k 10 500 python -u tools/ab_variants.py --clients $k --params 1e9 --variants $V --epilogues sgd,add_base --rounds 3 --prewarm-s 2 --check > $O/ab_k$k.jsonl 2> $O/ab_k$k.err || exit $?
done
for k in 2 3; do
  A="--clients $k --params 1e9 --epilogue adam --no-cpu-baseline"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rp_k$k -o k$k -- python3 bench.py $A --steps 10 --spot-check 0 > $O/rp_k$k.jsonl 2> $O/rp_k$k.err || exit $?
  timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_k${k}_fetch -o f -- python3 bench.py $A --steps 3 --warmup 1 --spot-check 0 > /dev/null 2> $O/pmc_k${k}_fetch.err || exit $?
  timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_k${k}_write -o w -- python3 bench.py $A --steps 3 --warmup 1 --spot-check 0 > /dev/null 2> $O/pmc_k${k}_write.err || exit $?
done
echo "rc=0"
