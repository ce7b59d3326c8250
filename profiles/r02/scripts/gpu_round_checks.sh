set -e
mkdir -p gpurun_out/r01b
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r01b/rocprof_narrow -o narrow -- python tools/bench_narrow.py --blocks-per-cu 2 --steps 5 > gpurun_out/r01b/narrow_prof.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r01b/rocprof_sag_defer -o sag -- python tools/sag_fedopt_bench.py --defer --rounds 4 > gpurun_out/r01b/sag_prof.log 2>&1
