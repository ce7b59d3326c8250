# GPU session 23 (round 5): the committed final product library (rebuilt after session 21 with A/B-only changes):
# smoke(), the dtype GPU tests and the fp32 few-client parity tests.
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05_s23
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_dtypes.py tests/test_gpu_parity.py > "$OUT/pytest.log" 2>&1 || exit $?
echo done
