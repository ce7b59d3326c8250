# GPU box script: hardware bf16 rounding in the narrow kernel.
# 1) exhaustive v_cvt_pk_bf16_f32 vs c10 recipe, 2) interleaved same-box A/B of the 16-bit tiled kernel
# (software rounding library built from the previous source vs the current library), 3) 16-bit parity tests.
set -e
OUT=gpurun_out/bf16ab
mkdir -p "$OUT"
timeout -k 10 60 ./tools/bf16_cvt_probe > "$OUT/probe.jsonl"
for i in 1 2; do
  NVFLARE_AMD_FEDAVG_LIB=tools/_ab/libfedavg_swbf16.so timeout -k 10 180 python tools/bench_narrow.py --fmt bfloat16 --steps 10 \
    | sed 's/^{/{"variant": "software_rne", /' >> "$OUT/ab.jsonl"
  timeout -k 10 180 python tools/bench_narrow.py --fmt bfloat16 --steps 10 \
    | sed 's/^{/{"variant": "v_cvt_pk_bf16_f32", /' >> "$OUT/ab.jsonl"
done
timeout -k 10 180 python tools/bench_narrow.py --fmt float16 --steps 10 | sed 's/^{/{"variant": "v_cvt_f16_f32", /' >> "$OUT/ab.jsonl"
timeout -k 10 600 python -u -m pytest tests/test_gpu_dtypes.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_dtypes.log" 2>&1
