# GPU session 22 (round 5): the 16-bit 1-client few-client form on tile QUADS (A/B forms 3-4, p = 4: K x 32 KiB per
# unit, the fp32 pair form's bytes) against pairs (the default) -- the few-client tests on the A/B library, then bf16 /
# fp16 x 1e9 at 1 client, torch and copy modes, outputs checked bit-equal.
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05_s22
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/nvflare_amd/lib
NVFLARE_AMD_FEDAVG_LIB=$L/ab/few.so timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_dtypes.py -k tiled16_few > "$OUT/pytest_few_ab.log" 2>&1 || exit $?
echo "tests done"
N="python -u tools/bench_narrow.py --params 1e9 --steps 10 --check --variants 0,512,1024,1536,2048 --clients 1"
for F in bfloat16 float16; do
  for M in torch copy; do
    NVFLARE_AMD_FEDAVG_LIB=$L/ab/few.so timeout -k 10 300 $N --fmt $F --mode $M >> "$OUT/sweep.jsonl" 2>> "$OUT/err.log" || exit $?
  done
done
echo done
