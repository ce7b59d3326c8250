# GPU session 15 (round 4): the plain burst kernel at 5-7 clients (one full group plus a remainder) with the group's
# loads as two pairs (variant 1024) against four together (0), one process per count, outputs checked equal.
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04_s15
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for K in 5 6 7; do
  timeout -k 10 300 python -u tools/ab_variants.py --clients $K --params 1e9 --variants 0,1024 --epilogues none --check --rounds 4 > "$OUT/pairs_k$K.jsonl" 2> "$OUT/pairs_k$K.err" || exit $?
done
echo done
