# GPU session 17 (round 5): where the 16-bit few-client kernel's 1-client time goes.  bf16 x 1e9 at 1 client in torch
# mode (division), numpy mode (two products) and copy mode (unweighted, no finalisation: bytes only), each on the
# default form, the burst form (256) and the A/B geometries (512-2048), outputs checked bit-equal per mode; the same
# at 2 clients in copy mode.  If copy runs no faster than torch, the arithmetic is not what holds the line under the
# fp32 kernel's.
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05_s17
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/nvflare_amd/lib
N="python -u tools/bench_narrow.py --params 1e9 --steps 10 --fmt bfloat16 --check --variants 0,256,512,1024,1536,2048"
for M in torch numpy copy; do
  NVFLARE_AMD_FEDAVG_LIB=$L/ab/few.so timeout -k 10 300 $N --clients 1 --mode $M >> "$OUT/k1.jsonl" 2>> "$OUT/err.log" || exit $?
done
NVFLARE_AMD_FEDAVG_LIB=$L/ab/few.so timeout -k 10 300 $N --clients 2 --mode copy >> "$OUT/k2.jsonl" 2>> "$OUT/err.log" || exit $?
echo done
