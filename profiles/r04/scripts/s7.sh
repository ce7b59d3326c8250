# GPU session 7 (round 4): the fused burst kernel's default client loop as two pairs per four-client group ("new")
# against the four-loads-together loop of session 6's "pre" library (nvflare_amd/lib/ab/libnvflare_amd_fedavg_pre.so):
# parity, then interleaved bench runs (config 5; Adam at 5, 6, 8, 10, 16 clients; config 3 and 2 as controls: the plain
# kernels are unchanged); then the same client-loop shapes on the plain burst kernel at 8-64 clients (launch variant
# bits 9-11, torch mode, K % 4 == 0: 0 = four loads together, 1 = round 3's GROUPED loop, 2 = pairs, 3 = clients
# 0, 2, 3 then 1, 4 = one at a time), outputs checked bit-equal.
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04_s7
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
PRE=nvflare_amd/lib/ab/libnvflare_amd_fedavg_pre.so
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_fedopt.py tests/test_gpu_parity.py > "$OUT/pytest.log" 2>&1 || exit $?
B="python -u bench.py --also none --no-cpu-baseline"
for i in 1 2; do
  for C in 5 3 2; do
    timeout -k 10 300 $B --config $C > "$OUT/c${C}_new_$i.jsonl" 2> "$OUT/c${C}_new_$i.err" || exit $?
    NVFLARE_AMD_FEDAVG_LIB=$PRE timeout -k 10 300 $B --config $C > "$OUT/c${C}_pre_$i.jsonl" 2> "$OUT/c${C}_pre_$i.err" || exit $?
  done
  for K in 5 6 8 10 16; do
    timeout -k 10 300 $B --clients $K --params 5e8 --epilogue adam --steps 10 > "$OUT/adam_k${K}_new_$i.jsonl" 2> "$OUT/adam_k${K}_new_$i.err" || exit $?
    NVFLARE_AMD_FEDAVG_LIB=$PRE timeout -k 10 300 $B --clients $K --params 5e8 --epilogue adam --steps 10 > "$OUT/adam_k${K}_pre_$i.jsonl" 2> "$OUT/adam_k${K}_pre_$i.err" || exit $?
  done
done
ab() { local name=$1; shift; timeout -k 10 300 python -u tools/ab_variants.py "$@" > "$OUT/$name.jsonl" 2> "$OUT/$name.err"; }
V=0,512,1024,1536,2048
ab plain_k64 --clients 64 --params 1e9 --variants $V --epilogues none --check --rounds 3 --reps 3 || exit $?
ab plain_k32 --clients 32 --params 1e9 --variants $V --epilogues none --check --rounds 3 --reps 3 || exit $?
ab plain_k16 --clients 16 --params 5e8 --variants $V --epilogues none --check --rounds 3 --reps 5 || exit $?
ab plain_k8 --clients 8 --params 5e8 --variants $V --epilogues none --check --rounds 3 --reps 5 || exit $?
ab plain_k8s --clients 8 --params 1.25e8 --variants $V --epilogues none --check --rounds 3 --reps 10 || exit $?
echo done
