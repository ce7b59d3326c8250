# GPU session 14 (round 5): the fp64 few-client burst kernel (fedavg_kernels.hip fedavg_tiles_f64x2_few, 1-3 client
# reads).  (1) the dtype GPU tests on the product library and the few-client forms' tests on the -DFEDAVG_AB_FEW library
# (nvflare_amd/lib/ab/few.so); (2) fp64 at 1 / 2 / 3 clients x 5e8, numpy mode (and torch at 2): the default form
# against the burst form (variant 256) and the A/B geometries (variant bits 9-11 = 1-4), interleaved in one process,
# outputs checked bit-equal.
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05_s14
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/nvflare_amd/lib
T="python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider"
# (the tests ran in this script's first run: profiles/r05/s14/pytest_*.log; its sweep stopped on a stream race in
# the tools' output check, since fixed)
echo "tests done"
G="python -u tools/bench_generic.py --dtype float64 --layout tiled --params 5e8 --steps 10 --check --variants 0,256,512,1024,1536,2048"
for K in 1 2 3; do
  NVFLARE_AMD_FEDAVG_LIB=$L/ab/few.so timeout -k 10 300 $G --clients $K >> "$OUT/f64_sweep.jsonl" 2>> "$OUT/err.log" || exit $?
done
NVFLARE_AMD_FEDAVG_LIB=$L/ab/few.so timeout -k 10 300 $G --clients 2 --mode torch >> "$OUT/f64_sweep.jsonl" 2>> "$OUT/err.log" || exit $?
timeout -k 10 300 python -u tools/bench_generic.py --dtype float64 --layout tiled --params 5e8 --steps 10 --clients 8 >> "$OUT/f64_k8.jsonl" 2>> "$OUT/err.log" || exit $?
echo done
