#!/bin/bash
# round 6, GPU session 21: s20's failing case (test_dma_adam_matches_oracle_and_per_tile[ieee-4-3]) on the new and the
# previous library, mismatches listed
set -u
O=gpurun_out/r06_s21
mkdir -p $O
export TMPDIR=/tmp
T="tests/test_gpu_epi_dma.py::test_dma_adam_matches_oracle_and_per_tile"
timeout -k 10 300 python -u -m pytest "$T" -q --timeout 200 --timeout-method thread -k "ieee" > $O/new.log 2>&1
echo "new rc=$?"
NVFLARE_AMD_FEDAVG_LIB=nvflare_amd/lib/ab/pre_zero.so timeout -k 10 300 python -u -m pytest "$T" -q --timeout 200 \
    --timeout-method thread -k "ieee" > $O/old.log 2>&1
echo "old rc=$?"
grep -E "^E .*\(|passed|failed" $O/new.log | head -20
grep -E "^E .*\(|passed|failed" $O/old.log | head -20
