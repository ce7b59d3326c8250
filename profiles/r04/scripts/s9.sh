# GPU session 9 (round 4): occupancy of the per-tile-store forms that 1-2 plain and 1-3 fused clients take (blocks per
# CU 1-8, variant 8 = per-tile stores), against the burst forms, one process per client count, outputs checked equal.
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04_s9
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
ab() { local name=$1; shift; timeout -k 10 300 python -u tools/ab_variants.py "$@" > "$OUT/$name.jsonl" 2> "$OUT/$name.err"; }
ab bpc_k1 --clients 1 --params 1e9 --variants 8:0:1,8:0:2,8:0:3,8:0:4,8:0:6,8:0:8,256 --epilogues none --check --rounds 3 || exit $?
ab bpc_k2 --clients 2 --params 1e9 --variants 8:0:1,8:0:2,8:0:3,8:0:4,8:0:6,8:0:8,256 --epilogues none --check --rounds 3 || exit $?
ab bpc_k3 --clients 3 --params 1e9 --variants 8:0:1,8:0:2,8:0:3,8:0:4,8:0:6,8:0:8,0 --epilogues none --check --rounds 3 || exit $?
for K in 1 2 3; do
  ab epi_bpc_k$K --clients $K --params 5e8 --variants 8:0:1,8:0:2,8:0:3,8:0:4,8:0:6,8:0:8,4:0:2,4:0:4 --epilogues adam --sqrt torch_cpu_amd --check --rounds 3 || exit $?
done
echo done
