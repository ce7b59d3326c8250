# GPU box script: amsgrad parity (kernel, generator) and an A/B of the Adam epilogue kernel against the
# library built before amsgrad (tools/_ab/libfedavg_noams.so), alternating processes.
set -e
OUT=gpurun_out/amsgrad
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_fedopt.py tests/test_gpu_fedopt_generator.py tests/test_gpu_deferred.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
for i in 1 2; do
  NVFLARE_AMD_FEDAVG_LIB=tools/_ab/libfedavg_noams.so timeout -k 10 200 python tools/ab_variants.py --variants 0 --epilogues adam,sgd --rounds 2 \
    | grep summary | sed 's/^{/{"lib": "before", /' >> "$OUT/ab.jsonl"
  timeout -k 10 200 python tools/ab_variants.py --variants 0 --epilogues adam,sgd --rounds 2 \
    | grep summary | sed 's/^{/{"lib": "amsgrad", /' >> "$OUT/ab.jsonl"
done
