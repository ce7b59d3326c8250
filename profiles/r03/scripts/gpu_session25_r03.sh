# GPU box script (round 3, session 25): few-client launches take the per-tile-store kernel
# (fedavg_capi.cpp kBurstMinClients) -- full `pytest -m gpu`, then plain and fused-Adam aggregation at 1-4 clients,
# the default form against the per-tile-store form (variant bit 3), interleaved twice, 1e9 params (Adam 5e8).
set -e
OUT=$GRAFT_REPO_ROOT/${1:-gpurun_out/r03_s25}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
for i in 1 2; do
  for K in 1 2 3 4; do
    for cfg in "dflt:--variant 0" "tile:--variant 8"; do
      name=${cfg%%:*}; flags=${cfg#*:}
      timeout -k 10 300 python bench.py --clients $K --params 1e9 $flags --also none --no-cpu-baseline --steps 10 > "$OUT/k${K}_${name}_$i.jsonl" 2> "$OUT/k${K}_${name}_$i.err"
      timeout -k 10 300 python bench.py --clients $K --params 5e8 --epilogue adam $flags --also none --no-cpu-baseline --steps 10 > "$OUT/adam_k${K}_${name}_$i.jsonl" 2> "$OUT/adam_k${K}_${name}_$i.err"
    done
  done
done
