# GPU session 20 (round 5): the fp32 few-client kernel on tile PAIRS (A/B forms, p = 2: K x 32 KiB contiguous per
# unit) against its single-tile product forms -- the few-client forms' parity tests on the -DFEDAVG_AB_FEW library,
# then 1 / 2 / 3 clients x 1e9, torch mode, interleaved in one process, outputs checked bit-equal.
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05_s20
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/nvflare_amd/lib
NVFLARE_AMD_FEDAVG_LIB=$L/ab/few.so timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py -k "few_client_burst_forms" > "$OUT/pytest_few_ab.log" 2>&1 || exit $?
echo "tests done"
A="python -u tools/ab_variants.py --params 1e9 --epilogues none --rounds 3 --check"
NVFLARE_AMD_FEDAVG_LIB=$L/ab/few.so timeout -k 10 300 $A --clients 1 --variants 0,2560,3072 >> "$OUT/f32_k1.jsonl" 2>> "$OUT/err.log" || exit $?
NVFLARE_AMD_FEDAVG_LIB=$L/ab/few.so timeout -k 10 300 $A --clients 2 --variants 0,2560,3072 >> "$OUT/f32_k2.jsonl" 2>> "$OUT/err.log" || exit $?
NVFLARE_AMD_FEDAVG_LIB=$L/ab/few.so timeout -k 10 300 $A --clients 3 --variants 0,2048,2560 >> "$OUT/f32_k3.jsonl" 2>> "$OUT/err.log" || exit $?
echo done
