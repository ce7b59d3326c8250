#!/bin/bash
# round 6, GPU session 20: +0 on the restated sqrt's and the constant-divisor quotient's fast forms (a frozen
# parameter's zero states and sums no longer recompute their column group per element) -- parity of the new library,
# then old (nvflare_amd/lib/ab/pre_zero.so, the previous commit's product library) against new in alternating
# processes: Adam at 1-3 clients, every parameter live and with the leading half frozen; the plain aggregation at 2
set -u
O=gpurun_out/r06_s20
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_torch_sqrt.py tests/test_gpu_epi_dma.py tests/test_gpu_fedopt.py -x -q \
    --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for lib in old new; do
    L=""; [ $lib = old ] && L=nvflare_amd/lib/ab/pre_zero.so
    for K in 1 2 3; do
      for F in 0 0.5; do
        env ${L:+NVFLARE_AMD_FEDAVG_LIB=$L} timeout -k 10 200 python -u tools/ab_variants.py --clients $K --params 1e9 --variants 0,4 \
            --epilogues adam --rounds 3 --reps 10 --prewarm-s 3 --frozen-frac $F --sqrt torch_cpu_amd \
            > $O/ab_${lib}_r${rep}_k${K}_f${F}.jsonl 2>&1 || { echo "ab rc=$?"; tail -20 $O/ab_${lib}_r${rep}_k${K}_f${F}.jsonl; exit 1; }
        grep summary $O/ab_${lib}_r${rep}_k${K}_f${F}.jsonl | python -c "import sys,json; [print('$lib', $rep, 'f=$F', d['clients'], d['epilogue'], d['variant'], d['frac_8TBps']) for d in map(json.loads, sys.stdin)]"
      done
    done
    env ${L:+NVFLARE_AMD_FEDAVG_LIB=$L} timeout -k 10 200 python -u tools/ab_variants.py --clients 2 --params 1e9 --variants 0 \
        --epilogues none --rounds 3 --reps 10 --prewarm-s 3 > $O/ab_${lib}_r${rep}_plain.jsonl 2>&1 || { echo "ab rc=$?"; exit 1; }
    grep summary $O/ab_${lib}_r${rep}_plain.jsonl | python -c "import sys,json; [print('$lib', $rep, d['clients'], d['epilogue'], d['variant'], d['frac_8TBps']) for d in map(json.loads, sys.stdin)]"
  done
done
