# GPU session 11 (round 4): fused few-client launches routed to the pipelined per-tile form from 2 reads (bench lines at
# 1-3 clients, Adam), the fused burst kernel's epilogue phase with its operand loads after the stores (variant 6 <<
# 9) against the default prefetch, Adam with the AMD-host sqrt at 8 / 16 / 64 clients; parity of the fused kernels.
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04_s11
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_fedopt.py tests/test_gpu_fedopt_generator.py tests/test_gpu_fused_wide.py > "$OUT/pytest.log" 2>&1 || exit $?
ab() { local name=$1; shift; timeout -k 10 300 python -u tools/ab_variants.py "$@" > "$OUT/$name.jsonl" 2> "$OUT/$name.err"; }
ab epre_k64 --clients 64 --params 1e9 --variants 0,3072 --epilogues adam --sqrt torch_cpu_amd --check --rounds 4 --reps 3 || exit $?
ab epre_k16 --clients 16 --params 5e8 --variants 0,3072 --epilogues adam --sqrt torch_cpu_amd --check --rounds 4 --reps 5 || exit $?
ab epre_k8 --clients 8 --params 5e8 --variants 0,3072 --epilogues adam --sqrt torch_cpu_amd --check --rounds 4 --reps 5 || exit $?
B="python -u bench.py --also none --no-cpu-baseline"
for K in 1 2 3; do
  timeout -k 10 300 $B --clients $K --params 1e9 --epilogue adam --steps 10 > "$OUT/adam_k$K.jsonl" 2> "$OUT/adam_k$K.err" || exit $?
done
timeout -k 10 300 $B --config 5 > "$OUT/c5.jsonl" 2> "$OUT/c5.err" || exit $?
echo done
