#!/bin/bash
# round 6, GPU session 27: the tree's product library end to end -- smoke, the whole GPU suite, the default bench line,
# and config 3 under rocprofv3 (kernel stats)
set -u
O=gpurun_out/r06_s27
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.jsonl 2> $O/bench.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rp_bench -o bench -- python3 bench.py --also none --no-cpu-baseline --steps 20 --warmup 5 > $O/bench_prof.jsonl 2> $O/bench_prof.err
echo "rc=$?"
