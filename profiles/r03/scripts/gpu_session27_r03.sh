# GPU box script (round 3, session 27): the few-client routing as built (plain and fused launches with fewer than 4
# row reads take the per-tile-store kernels, fedavg_capi.cpp kBurstMinClients / kEpiBurstMinClients) -- full
# `pytest -m gpu`, smoke, the default bench line, then 1-4 clients default vs forced per-tile (variant bit 3) for plain, Adam and SGD.
set -e
OUT=$GRAFT_REPO_ROOT/${1:-gpurun_out/r03_s27}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
timeout -k 10 600 python bench.py > "$OUT/bench.jsonl" 2> "$OUT/bench.err"
for K in 1 2 3 4; do
  for cfg in "dflt:--variant 0" "tile:--variant 8"; do
    name=${cfg%%:*}; flags=${cfg#*:}
    timeout -k 10 300 python bench.py --clients $K --params 1e9 $flags --also none --no-cpu-baseline --steps 10 > "$OUT/k${K}_${name}.jsonl" 2> "$OUT/k${K}_${name}.err"
    for E in adam sgd; do
      timeout -k 10 300 python bench.py --clients $K --params 5e8 --epilogue $E $flags --also none --no-cpu-baseline --steps 10 > "$OUT/${E}_k${K}_${name}.jsonl" 2> "$OUT/${E}_k${K}_${name}.err"
    done
  done
done
