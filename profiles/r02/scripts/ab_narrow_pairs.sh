#!/bin/bash
# Same-box A/B of the 16-bit tile kernel: in-tree library vs the HEAD build (tools/build_rev_lib.py), three
# alternating rounds, bf16 and fp16, 64 x 1e9, default and 1 block per CU; dtype parity suite first.
set -o pipefail
mkdir -p gpurun_out/abn
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dtypes.py > gpurun_out/abn/pytest_dtypes.log 2>&1 || { tail -30 gpurun_out/abn/pytest_dtypes.log; exit 1; }
tail -2 gpurun_out/abn/pytest_dtypes.log
for r in 0 1 2; do
  for lib in new head; do
    if [ $lib = head ]; then export NVFLARE_AMD_FEDAVG_LIB=$PWD/nvflare_amd/lib/ab/libnvflare_amd_fedavg_head.so; else unset NVFLARE_AMD_FEDAVG_LIB; fi
    for fmt in bfloat16 float16; do
      timeout -k 10 120 python -u tools/bench_narrow.py --fmt $fmt --clients 64 --params 1e9 --steps 10 --blocks-per-cu 0,1 > gpurun_out/abn/${lib}_${fmt}_r$r.jsonl 2>&1 || { tail -5 gpurun_out/abn/${lib}_${fmt}_r$r.jsonl; exit 1; }
      echo "$lib $fmt r$r: $(grep -o '"frac_of_8TBs": [0-9.]*\|"blocks_per_cu": [0-9]*' gpurun_out/abn/${lib}_${fmt}_r$r.jsonl | tr '\n' ' ')"
    done
  done
done
