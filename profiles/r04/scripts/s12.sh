# GPU session 12 (round 4): the per-tile-store kernel with the client count built in for 1-2 clients (variant 8 now
# takes it; 8 + 128 = the runtime-K per-tile loop; 256 = the burst form), blocks per CU 1-4, one process per count,
# outputs checked equal; the default bench lines at 1-2 clients; fp64 tiled with one client's loads in flight
# (FEDAVG_F64_UNROLL=1, nvflare_amd/lib/ab/libnvflare_amd_fedavg_f64u1.so) against the product's 2; parity.
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04_s12
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py > "$OUT/pytest_parity.log" 2>&1 || exit $?
ab() { local name=$1; shift; timeout -k 10 300 python -u tools/ab_variants.py "$@" > "$OUT/$name.jsonl" 2> "$OUT/$name.err"; }
for K in 2 1; do
  ab kc_k$K --clients $K --params 1e9 --variants 136,8,8:0:1,8:0:3,8:0:4,256 --epilogues none --check --rounds 4 || exit $?
done
B="python -u bench.py --also none --no-cpu-baseline"
for K in 1 2; do
  timeout -k 10 300 $B --clients $K --params 1e9 --steps 20 > "$OUT/bench_k$K.jsonl" 2> "$OUT/bench_k$K.err" || exit $?
done
for i in 1 2; do
  for L in prod f64u1; do
    lib=nvflare_amd/lib/libnvflare_amd_fedavg.so
    [ "$L" = f64u1 ] && lib=nvflare_amd/lib/ab/libnvflare_amd_fedavg_f64u1.so
    for K in 32 8; do
      NVFLARE_AMD_FEDAVG_LIB=$lib timeout -k 10 180 python -u tools/bench_generic.py --dtype float64 --layout tiled --clients $K --params 2e8 --steps 10 > "$OUT/f64_${L}_k${K}_$i.jsonl" 2> "$OUT/f64_${L}_k${K}_$i.err" || exit $?
    done
  done
done
echo done
