# GPU box script (round 3, session 22): the rebuilt tree (container re-created) -- full `pytest -m gpu`, smoke(),
# then session 21's fused-Adam blocks-per-CU sweep at few clients (tools/gpu_session21_r03.sh).
set -e
OUT=$GRAFT_REPO_ROOT/${1:-gpurun_out/r03_s22}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
bash tools/gpu_session21_r03.sh "${1:-gpurun_out/r03_s22}/bpc"
