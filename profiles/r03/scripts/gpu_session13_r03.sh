# GPU box script (round 3, session 13): the AMD-host torch sqrt (FEDAVG_SQRT_TORCH_AMD, the box CPU's RSQRTPS table
# staged in LDS) -- which vsSqrt kernel the box's torch runs and whether the restatement equals it on every probe
# input and a stride-61 sample of all 2^32 (CPU only), the full `pytest -m gpu`, smoke(), then config 5 (fused Adam)
# with each sqrt, interleaved twice, and the default bench line.  Every GPU step has its own time limit; `set -e`
# ends the script at the first failure.
set -e
OUT=$GRAFT_REPO_ROOT/${1:-gpurun_out/r03_s13}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/sqrt_box_kernels.py "$OUT/sqrt" > "$OUT/sqrt_box_kernels.log" 2>&1
timeout -k 10 600 python tools/sqrt_mkl_sse_check.py torch --stride 61 --workers 12 > "$OUT/sqrt_check_torch_s61.log" 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
for i in 1 2; do
  for S in ieee torch_cpu torch_cpu_amd; do
    timeout -k 10 300 python bench.py --config 5 --sqrt $S --no-cpu-baseline > "$OUT/c5_${S}_$i.jsonl" 2> "$OUT/c5_${S}_$i.err"
  done
done
timeout -k 10 400 python bench.py > "$OUT/bench.jsonl" 2> "$OUT/bench.err"
