# GPU box script (round 3, session 16): the Intel-host sqrt's specials through the correctly rounded sqrt (negative
# subnormals gave -0, torch NaN) -- full `pytest -m gpu`, smoke(), and the device-vs-oracle sqrt over all 2^32 inputs.
set -e
OUT=$GRAFT_REPO_ROOT/${1:-gpurun_out/r03_s16}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
timeout -k 10 600 python tools/sqrt_device_exhaustive.py --workers 12 > "$OUT/sqrt_device_exhaustive.log" 2>&1
timeout -k 10 300 python bench.py --config 5 --sqrt torch_cpu --no-cpu-baseline > "$OUT/bench_config5_torch_cpu.jsonl" 2> "$OUT/bench_config5_torch_cpu.err"
