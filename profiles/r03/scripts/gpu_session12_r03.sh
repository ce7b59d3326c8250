# GPU box script (round 3, session 12): rebuilt tree check -- full `pytest -m gpu` (with the SSE2 vsSqrt epilogue
# variant), smoke(), the default bench line (now with the host-resident config-2 entry "2h"), and two CPU-only
# diagnostics of the box host's torch sqrt: which MKL vsSqrt kernel it runs (tools/sqrt_box_kernels.py) and its
# RSQRTPS / RCPPS estimates (tools/rsqrtps_dump.c).  Every GPU step has its own time limit; `set -e` ends the
# script at the first failure.
set -e
OUT=$GRAFT_REPO_ROOT/${1:-gpurun_out/r03_s12}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/sqrt_box_kernels.py "$OUT/sqrt" > "$OUT/sqrt_box_kernels.log" 2>&1
gcc -O2 -msse2 tools/rsqrtps_dump.c -o /tmp/rsqrtps_dump
/tmp/rsqrtps_dump "$OUT/sqrt/rsqrtps_amd.bin" "$OUT/sqrt/rcpps_amd.bin" > "$OUT/rsqrtps_dump.log" 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
timeout -k 10 400 python bench.py > "$OUT/bench.jsonl" 2> "$OUT/bench.err"
