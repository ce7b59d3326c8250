set -o pipefail
mkdir -p gpurun_out/abe2
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fedopt.py > gpurun_out/abe2/pytest.log 2>&1 || { tail -30 gpurun_out/abe2/pytest.log; exit 1; }
tail -1 gpurun_out/abe2/pytest.log
for K in 16 24 32; do
  f=gpurun_out/abe2/k${K}.jsonl
  timeout -k 10 240 python -u tools/ab_variants.py --clients $K --params 1e9 --variants 0:0:0,0:0:1,0:0:2 --epilogues none,adam --rounds 3 --reps 5 > $f 2>&1 || { tail -5 $f; exit 1; }
  echo "K=$K"; grep summary $f | grep -o '"epilogue": "[a-z]*", "variant": "[0-9:]*"\|"frac_8TBps": [0-9.]*' | paste - - 
done
