#!/bin/bash
# round 6, GPU session 14: the whole GPU suite on an A/B library built from this tree
# (tools/build_rev_lib.py --rev WORKTREE: every kernel form, -DFEDAVG_AB), so the A/B-only cases a product library skips run
set -u
O=gpurun_out/r06_s14
mkdir -p $O
export TMPDIR=/tmp
NVFLARE_AMD_FEDAVG_LIB=nvflare_amd/lib/ab/full_ab.so timeout -k 10 2000 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread > $O/pytest_gpu_ab.log 2>&1
echo "rc=$?"
