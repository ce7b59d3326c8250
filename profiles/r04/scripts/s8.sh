# GPU session 8 (round 4): the tree with pairs as the default client-group shape from 8 clients on (plain and fused
# burst kernels): the whole GPU suite and smoke; the default bench line; interleaved against session 6's "pre" library
# (four loads together): configs 3 / 5 / 2, plain at 7 / 10 / 12 clients, fused Adam at 5-8 clients; rocprofv3 kernel
# stats of configs 3 and 5, PMC FETCH / WRITE of config 3.
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04_s8
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
PRE=nvflare_amd/lib/ab/libnvflare_amd_fedavg_pre.so
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests \
  > "$OUT/pytest_gpu.log" 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > "$OUT/bench.jsonl" 2> "$OUT/bench.err" || exit $?
B="python -u bench.py --also none --no-cpu-baseline"
for i in 1 2; do
  for C in 3 5 2; do
    timeout -k 10 300 $B --config $C > "$OUT/c${C}_new_$i.jsonl" 2> "$OUT/c${C}_new_$i.err" || exit $?
    NVFLARE_AMD_FEDAVG_LIB=$PRE timeout -k 10 300 $B --config $C > "$OUT/c${C}_pre_$i.jsonl" 2> "$OUT/c${C}_pre_$i.err" || exit $?
  done
  for K in 7 10 12; do
    timeout -k 10 300 $B --clients $K --params 5e8 --steps 10 > "$OUT/plain_k${K}_new_$i.jsonl" 2> "$OUT/plain_k${K}_new_$i.err" || exit $?
    NVFLARE_AMD_FEDAVG_LIB=$PRE timeout -k 10 300 $B --clients $K --params 5e8 --steps 10 > "$OUT/plain_k${K}_pre_$i.jsonl" 2> "$OUT/plain_k${K}_pre_$i.err" || exit $?
  done
  for K in 5 6 7 8; do
    timeout -k 10 300 $B --clients $K --params 5e8 --epilogue adam --steps 10 > "$OUT/adam_k${K}_new_$i.jsonl" 2> "$OUT/adam_k${K}_new_$i.err" || exit $?
    NVFLARE_AMD_FEDAVG_LIB=$PRE timeout -k 10 300 $B --clients $K --params 5e8 --epilogue adam --steps 10 > "$OUT/adam_k${K}_pre_$i.jsonl" 2> "$OUT/adam_k${K}_pre_$i.err" || exit $?
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rocprof_bench" -o bench -- python -u bench.py --also none --no-cpu-baseline > "$OUT/bench_prof.jsonl" 2> "$OUT/bench_prof.err" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rocprof_adam" -o adam -- python -u bench.py --config 5 --also none --no-cpu-baseline > "$OUT/bench_adam_prof.jsonl" 2> "$OUT/bench_adam_prof.err" || exit $?
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc/none_$C" -o pmc -- python -u bench.py --also none --steps 2 --warmup 1 --no-cpu-baseline --spot-check 0 > "$OUT/pmc_none_$C.log" 2>&1 || exit $?
done
echo done
