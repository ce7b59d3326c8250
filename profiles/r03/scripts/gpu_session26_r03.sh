# GPU box script (round 3, session 26): fused Adam at 5-16 clients, the burst form (default) against the per-tile
# epilogue form (variant bit 3), interleaved twice, 5e8 params -- where the burst form starts to pay (at 1-4 clients
# the per-tile form won by 4-14 points, profiles/r03/s25/).
set -e
OUT=$GRAFT_REPO_ROOT/${1:-gpurun_out/r03_s26}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
for i in 1 2; do
  for K in 5 6 8 12 16; do
    for cfg in "dflt:--variant 0" "tile:--variant 8"; do
      name=${cfg%%:*}; flags=${cfg#*:}
      timeout -k 10 300 python bench.py --clients $K --params 5e8 --epilogue adam $flags --also none --no-cpu-baseline --steps 10 > "$OUT/adam_k${K}_${name}_$i.jsonl" 2> "$OUT/adam_k${K}_${name}_$i.err"
      timeout -k 10 300 python bench.py --clients $K --params 5e8 --epilogue sgd $flags --also none --no-cpu-baseline --steps 10 > "$OUT/sgd_k${K}_${name}_$i.jsonl" 2> "$OUT/sgd_k${K}_${name}_$i.err"
    done
  done
done
