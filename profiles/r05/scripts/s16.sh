# GPU session 16 (round 5): the 16-bit source compiled as two units (fedavg_narrow.hip FEDAVG_NARROW_PART 1 / 2):
# the dtype GPU tests (every 16-bit path: rows, tiles, few-client, tails, scatter) and smoke().
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05_s16
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_dtypes.py tests/test_gpu_fedopt.py > "$OUT/pytest.log" 2>&1 || exit $?
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || exit $?
echo done
