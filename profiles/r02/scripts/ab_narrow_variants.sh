#!/bin/bash
# Same-box A/B of 16-bit burst kernel builds (tools/build_rev_lib.py -D ...) at one block per CU: in-tree
# library vs side libraries under nvflare_amd/lib/ab/, alternating rounds.
set -o pipefail
mkdir -p gpurun_out/abv
for r in 0 1; do
  for lib in base $(cd nvflare_amd/lib/ab && ls *.so | sed 's/\.so$//'); do
    if [ $lib = base ]; then unset NVFLARE_AMD_FEDAVG_LIB; else export NVFLARE_AMD_FEDAVG_LIB=$PWD/nvflare_amd/lib/ab/$lib.so; fi
    for cfg in bfloat16:64:1000000000 float16:64:1000000000 bfloat16:128:500000000; do
      IFS=: read fmt K P <<< "$cfg"
      f=gpurun_out/abv/${lib}_${fmt}_k${K}_r$r.jsonl
      timeout -k 10 150 python -u tools/bench_narrow.py --fmt $fmt --clients $K --params $P --steps 10 --blocks-per-cu 1 > $f 2>&1 || { tail -5 $f; exit 1; }
      echo "$lib $fmt K=$K r$r: $(grep -o '"frac_of_8TBs": [0-9.]*' $f | tr '\n' ' ')"
    done
  done
done
