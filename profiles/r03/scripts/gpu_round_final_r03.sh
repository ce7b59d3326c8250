# GPU box script (round 3, final build): full `pytest -m gpu`, smoke(), the default bench line (config 3 with configs
# 5, 4, 2h and 4x in `also`; config 5 takes this host's sqrt -- the AMD form on the pool), config 5 with the correctly
# rounded sqrt, config 2, rocprofv3 kernel traces of the config-3 and config-5 commands, the PMC traffic passes of
# both, and the two exhaustive sqrt checks (the box's torch.sqrt and the device's restatements over all 2^32 inputs).
# Every GPU step has its own time limit; `set -e` ends the script at the first failure.
set -e
OUT=${1:-gpurun_out/r03_final}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
timeout -k 10 400 python bench.py > "$OUT/bench.jsonl" 2> "$OUT/bench.err"
timeout -k 10 300 python bench.py --config 5 --sqrt ieee --no-cpu-baseline > "$OUT/bench_config5_ieee.jsonl" 2> "$OUT/bench_config5_ieee.err"
timeout -k 10 300 python bench.py --config 2 --steps 50 > "$OUT/bench_config2.jsonl" 2> "$OUT/bench_config2.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rocprof_bench" -o bench -- python bench.py --also none --no-cpu-baseline > "$OUT/bench_prof.jsonl" 2> "$OUT/bench_prof.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rocprof_adam" -o adam -- python bench.py --config 5 --no-cpu-baseline > "$OUT/bench_adam_prof.jsonl" 2> "$OUT/bench_adam_prof.err"
bash tools/gpu_pmc_bench.sh "$OUT/pmc" none adam
timeout -k 10 600 python tools/sqrt_mkl_sse_check.py torch --stride 1 --workers 12 > "$OUT/sqrt_check_torch_all.log" 2>&1
timeout -k 10 600 python tools/sqrt_device_exhaustive.py --workers 12 > "$OUT/sqrt_device_exhaustive.log" 2>&1
