#!/bin/bash
# After the 16-bit default change: dtype parity, the 16-bit default (0) against explicit 1 / 2 blocks per CU at
# 48 / 64 / 128 clients, and the fp64 arena burst kernel's blocks per CU over client counts.
set -o pipefail
mkdir -p gpurun_out/bpc
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dtypes.py > gpurun_out/bpc/pytest_dtypes.log 2>&1 || { tail -30 gpurun_out/bpc/pytest_dtypes.log; exit 1; }
tail -1 gpurun_out/bpc/pytest_dtypes.log
for kp in 48:1300000000 64:1000000000 128:500000000; do
  K=${kp%%:*}; P=${kp##*:}
  f=gpurun_out/bpc/narrow_k${K}.jsonl
  timeout -k 10 150 python -u tools/bench_narrow.py --fmt bfloat16 --clients $K --params $P --steps 10 --blocks-per-cu 0,1,2 > $f 2>&1 || { tail -5 $f; exit 1; }
  echo "bf16 K=$K: $(grep -o '"blocks_per_cu": [0-9]*\|"frac_of_8TBs": [0-9.]*' $f | tr '\n' ' ')"
done
for kp in 8:2000000000 16:1000000000 32:800000000 64:400000000; do
  K=${kp%%:*}; P=${kp##*:}
  f=gpurun_out/bpc/f64_k${K}.jsonl
  timeout -k 10 150 python -u tools/bench_generic.py --dtype float64 --layout tiled --clients $K --params $P --steps 10 --blocks-per-cu 1,2 > $f 2>&1 || { tail -5 $f; exit 1; }
  echo "f64 K=$K: $(grep -o '"blocks_per_cu": [0-9]*\|"frac_of_8TBs": [0-9.]*' $f | tr '\n' ' ')"
done
