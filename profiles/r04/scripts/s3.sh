# GPU session 3 (round 4): the round's new GPU tests that session 2 did not reach, config 5 at full size in every sqrt,
# a memory-copy trace of the host-resident config-2 round, then few-client A/Bs: tile-stride pads
# (DRAM channel mapping of the power-of-two slab strides at 2 and 4 clients), numpy mode (no division), plain + Adam.
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04_s3
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_sharded_fedopt.py tests/test_gpu_fedopt_ctl.py > "$OUT/pytest_new.log" 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 500 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_fullsize.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$OUT/trace2h" -o trace -- python -u bench.py --config 2 --also 2h --no-cpu-baseline --steps 5 > "$OUT/bench_2h_trace.jsonl" 2> "$OUT/bench_2h_trace.err" || exit $?
ab() { local name=$1; shift; timeout -k 10 300 python -u tools/ab_variants.py "$@" --rounds 3 > "$OUT/$name.jsonl" 2> "$OUT/$name.err"; }
ab pad_k2 --clients 2 --params 5e8 --variants 0,256 --epilogues none,adam --pads 0,64,2048 || exit $?
ab pad_k4 --clients 4 --params 5e8 --variants 0,8 --epilogues none,adam --pads 0,64 || exit $?
ab rem_k --clients 10 --params 5e8 --variants 0,128 --epilogues none || exit $?
ab rem_k7 --clients 7 --params 5e8 --variants 0,128 --epilogues none || exit $?
ab pad_k1 --clients 1 --params 5e8 --variants 0 --epilogues adam --pads 0,64 || exit $?
ab pad_k3 --clients 3 --params 5e8 --variants 0 --epilogues adam --pads 0,64 || exit $?
ab np_k2 --clients 2 --params 5e8 --variants 8,256 --epilogues none --mode numpy || exit $?
ab np_k4 --clients 4 --params 5e8 --variants 0,8 --epilogues none --mode numpy || exit $?
