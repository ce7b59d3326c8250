# GPU session 2 (round 4): the burst kernel with the client count built in (tile_sum_kc) against the per-tile-store
# form and the runtime-K burst form, 1-8 clients, interleaved in one process (tools/ab_variants.py --check: every
# variant's output bit-equal to the first's); the parity tests of the launch forms; the round's new GPU tests; config 5
# at full size in every sqrt; a memory-copy trace of the host-resident config-2 round.
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04_s2
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
ab() { local name=$1; shift; timeout -k 10 300 python -u tools/ab_variants.py "$@" --epilogues none --rounds 3 --check > "$OUT/$name.jsonl" 2> "$OUT/$name.err"; }
for K in 2 1 3; do ab ab_k$K --clients $K --params 1e9 --variants 8,256,384 || exit $?; done
for K in 4 5 6 8; do ab ab_k$K --clients $K --params 5e8 --variants 0,128,8 || exit $?; done
ab ab_k8_c2 --clients 8 --params 1.25e8 --variants 0,128 || exit $?
for R in 2 1 3; do
  timeout -k 10 300 python -u tools/hbm_mix_probe.py --ratio $R --params 2.5e8 --preset epi --rounds 3 > "$OUT/epi_r$R.jsonl" 2> "$OUT/epi_r$R.err" || exit $?
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py tests/test_gpu_torch_sqrt.py tests/test_gpu_sharded_fedopt.py tests/test_gpu_fedopt_ctl.py > "$OUT/pytest_new.log" 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 500 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_fullsize.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$OUT/trace2h" -o trace -- python -u bench.py --config 2 --also 2h --no-cpu-baseline --steps 5 > "$OUT/bench_2h_trace.jsonl" 2> "$OUT/bench_2h_trace.err"
