#!/bin/bash
# round 6, GPU session 1: the new default bench line, fused Adam at 2 / 3 clients (bench, rocprofv3 kernel stats,
# PMC FETCH_SIZE / WRITE_SIZE), the full GPU suite on the product library
set -u
O=gpurun_out/r06_s1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
A2="--clients 2 --params 1e9 --epilogue adam --no-cpu-baseline"
A3="--clients 3 --params 1e9 --epilogue adam --no-cpu-baseline"
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.jsonl 2> $O/bench.err &&
timeout -k 10 200 python -u bench.py $A2 --steps 10 > $O/adam_k2.jsonl 2> $O/adam_k2.err &&
timeout -k 10 200 python -u bench.py $A3 --steps 10 > $O/adam_k3.jsonl 2> $O/adam_k3.err &&
timeout -k 10 200 python -u bench.py $A2 --steps 10 > $O/adam_k2b.jsonl 2> $O/adam_k2b.err &&
timeout -k 10 200 python -u bench.py $A3 --steps 10 > $O/adam_k3b.jsonl 2> $O/adam_k3b.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rp_k2 -o k2 -- python3 bench.py $A2 --steps 10 --spot-check 0 > $O/rp_k2.jsonl 2> $O/rp_k2.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rp_k3 -o k3 -- python3 bench.py $A3 --steps 10 --spot-check 0 > $O/rp_k3.jsonl 2> $O/rp_k3.err &&
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_k2_fetch -o f -- python3 bench.py $A2 --steps 3 --warmup 1 --spot-check 0 > /dev/null 2> $O/pmc_k2_fetch.err &&
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_k2_write -o w -- python3 bench.py $A2 --steps 3 --warmup 1 --spot-check 0 > /dev/null 2> $O/pmc_k2_write.err &&
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_k3_fetch -o f -- python3 bench.py $A3 --steps 3 --warmup 1 --spot-check 0 > /dev/null 2> $O/pmc_k3_fetch.err &&
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_k3_write -o w -- python3 bench.py $A3 --steps 3 --warmup 1 --spot-check 0 > /dev/null 2> $O/pmc_k3_write.err &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
