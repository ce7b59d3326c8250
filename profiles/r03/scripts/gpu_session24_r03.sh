# GPU box script (round 3, session 24): the plain kernel at 2 / 4 clients (NVFlare's examples mostly run 2) --
# burst form at one and two blocks per CU, the register-only burst form (variant bit 5) and the per-tile-store form
# (variant bit 3), interleaved twice, 1e9 params; plus the 8:1 ... 2:1 mix probe for the ceiling of those shapes.
set -e
OUT=$GRAFT_REPO_ROOT/${1:-gpurun_out/r03_s24}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
for i in 1 2; do
  for K in 2 4; do
    for cfg in "b1:--blocks-per-cu 1" "b2:--blocks-per-cu 2" "reg:--variant 32" "tile:--variant 8"; do
      name=${cfg%%:*}; flags=${cfg#*:}
      timeout -k 10 300 python bench.py --clients $K --params 1e9 $flags --also none --no-cpu-baseline --steps 10 > "$OUT/k${K}_${name}_$i.jsonl" 2> "$OUT/k${K}_${name}_$i.err"
    done
  done
done
for R in 2 4; do
  timeout -k 10 300 python tools/hbm_mix_probe.py --ratio $R --params 1e9 --rounds 3 --reps 5 > "$OUT/mix_r$R.jsonl" 2> "$OUT/mix_r$R.err"
done
