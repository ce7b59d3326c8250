# e2e rates with quantized client payloads (row f4): lazy device dequantization vs eager
export TMPDIR=/tmp; mkdir -p gpurun_out
for q in float16 blockwise8 normfloat4; do
  timeout -k 10 300 python tools/e2e_bench.py --quant $q > gpurun_out/e2e_q_$q.jsonl 2>&1 || exit 1
  timeout -k 10 300 python tools/e2e_bench.py --quant $q --eager > gpurun_out/e2e_q_${q}_eager.jsonl 2>&1 || exit 1
done
