#!/bin/bash
# round 6, GPU session 22: what the LDS-DMA Adam form wrote into the elements it got wrong (tools/r06/diag_u14.py)
set -u
O=gpurun_out/r06_s22
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/r06/diag_u14.py 3 > $O/diag_k3.txt 2>&1; echo "rc=$?"
cat $O/diag_k3.txt | tail -30
