# GPU session 5 (round 4): the fused kernel's client loop with the K mod 4 remainder chosen per tile (tile_sum_rrem)
# against the per-slot-branch GROUPED loop of commit 42f2b5f and round 3's branch-free repeats (both with the
# constant-divisor quotient) and commit 4f8a188 (repeats, IEEE division): parity first, then interleaved bench runs at
# 5-10 clients and config 5; kernel traces of the 1-client burst kernel next to the mix probe's burst pattern (is the
# 20-point gap inside the launches or between them).
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04_s5
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
AB=nvflare_amd/lib/ab
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_fedopt.py > "$OUT/pytest_fedopt.log" 2>&1 || exit $?
B="python -u bench.py --epilogue adam --also none --no-cpu-baseline"
run() {  # name lib args...
  local name=$1 lib=$2; shift 2
  if [ "$lib" = new ]; then
    timeout -k 10 300 $B "$@" > "$OUT/$name.jsonl" 2> "$OUT/$name.err"
  else
    NVFLARE_AMD_FEDAVG_LIB=$AB/libnvflare_amd_fedavg_$lib.so timeout -k 10 300 $B "$@" > "$OUT/$name.jsonl" 2> "$OUT/$name.err"
  fi
}
for i in 1 2; do
  for K in 8 5 6 7 10; do
    for L in new grp rep; do
      run "k${K}_${L}_$i" $L --clients $K --params 5e8 --steps 10 || exit $?
    done
  done
  for L in new grp rep; do
    run "c5_${L}_$i" $L --config 5 || exit $?
  done
done
MIX_CASES=burst_r8_l4,tile timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$OUT/gap_probe" -o probe -- \
  python -u tools/hbm_mix_probe.py --ratio 1 --params 5e8 --rounds 2 --reps 5 --preset few > "$OUT/gap_probe.jsonl" 2> "$OUT/gap_probe.err" || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$OUT/gap_lib" -o lib -- \
  python -u tools/ab_variants.py --clients 1 --params 1e9 --variants 256,8,256:0:1 --epilogues none --rounds 2 --reps 5 > "$OUT/gap_lib.jsonl" 2> "$OUT/gap_lib.err" || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$OUT/gap_lib2" -o lib2 -- \
  python -u tools/ab_variants.py --clients 2 --params 1e9 --variants 256,8 --epilogues none --rounds 2 --reps 5 > "$OUT/gap_lib2.jsonl" 2> "$OUT/gap_lib2.err" || exit $?
echo done
