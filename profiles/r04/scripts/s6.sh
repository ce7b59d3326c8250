# GPU session 6 (round 4): burst kernels whose register-held tiles carry no control flow and are finalised in the store
# / epilogue phase (the library of this tree, "new") against the same tree before that change ("pre",
# nvflare_amd/lib/ab/libnvflare_amd_fedavg_pre.so): parity first; the 1-4-client forms per library in one process
# each (per-tile vs burst, outputs checked bit-equal); configs 3 / 2 / 5 interleaved; then the fused burst kernel's
# client-loop shapes (launch variant bits 9-11: 0 = run-time remainder form, 1 = round 3's GROUPED loop with repeats,
# 2 = two pairs, 3 = clients 0, 2, 3 then 1, 4 = one client at a time), Adam with the AMD-host sqrt, checked bit-equal.
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04_s6
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
PRE=nvflare_amd/lib/ab/libnvflare_amd_fedavg_pre.so
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_fedopt.py tests/test_gpu_parity.py > "$OUT/pytest.log" 2>&1 || exit $?
ab() { local name=$1; shift; timeout -k 10 300 python -u tools/ab_variants.py "$@" > "$OUT/$name.jsonl" 2> "$OUT/$name.err"; }
abp() { local name=$1; shift; NVFLARE_AMD_FEDAVG_LIB=$PRE timeout -k 10 300 python -u tools/ab_variants.py "$@" > "$OUT/$name.jsonl" 2> "$OUT/$name.err"; }
for K in 1 2; do
  ab few_new_k$K --clients $K --params 1e9 --variants 8,256 --epilogues none --check --rounds 3 || exit $?
  abp few_pre_k$K --clients $K --params 1e9 --variants 8,256 --epilogues none --check --rounds 3 || exit $?
done
for K in 3 4; do
  ab few_new_k$K --clients $K --params 1e9 --variants 0,8 --epilogues none --check --rounds 3 || exit $?
  abp few_pre_k$K --clients $K --params 1e9 --variants 0,8 --epilogues none --check --rounds 3 || exit $?
done
B="python -u bench.py --also none --no-cpu-baseline"
for i in 1 2; do
  for C in 3 2 5; do
    timeout -k 10 300 $B --config $C > "$OUT/c${C}_new_$i.jsonl" 2> "$OUT/c${C}_new_$i.err" || exit $?
    NVFLARE_AMD_FEDAVG_LIB=$PRE timeout -k 10 300 $B --config $C > "$OUT/c${C}_pre_$i.jsonl" 2> "$OUT/c${C}_pre_$i.err" || exit $?
  done
  for K in 5 8; do
    timeout -k 10 300 $B --clients $K --params 5e8 --epilogue adam --steps 10 > "$OUT/adam_k${K}_new_$i.jsonl" 2> "$OUT/adam_k${K}_new_$i.err" || exit $?
    NVFLARE_AMD_FEDAVG_LIB=$PRE timeout -k 10 300 $B --clients $K --params 5e8 --epilogue adam --steps 10 > "$OUT/adam_k${K}_pre_$i.jsonl" 2> "$OUT/adam_k${K}_pre_$i.err" || exit $?
  done
done
V=0,512,1024,1536,2048
ab loop_k64 --clients 64 --params 1e9 --variants $V --epilogues adam --sqrt torch_cpu_amd --check --rounds 3 --reps 3 || exit $?
ab loop_k8 --clients 8 --params 5e8 --variants $V --epilogues adam --sqrt torch_cpu_amd --check --rounds 3 --reps 5 || exit $?
ab loop_k32 --clients 32 --params 5e8 --variants $V --epilogues adam --sqrt torch_cpu_amd --check --rounds 3 --reps 5 || exit $?
ab loop_k6 --clients 6 --params 5e8 --variants $V --epilogues adam --sqrt torch_cpu_amd --check --rounds 3 --reps 5 || exit $?
ab loop_k10 --clients 10 --params 5e8 --variants $V --epilogues adam --sqrt torch_cpu_amd --check --rounds 3 --reps 5 || exit $?
echo done
