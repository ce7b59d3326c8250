# GPU box script (round 3, session 21): fused Adam at few clients (FedOpt's usual case) -- one block per CU (the
# 9-LDS-tile form) against two (the 4-LDS-tile form the library picks below 64 clients), now that the Adam epilogue
# holds more than 256 VGPRs and two blocks no longer share a CU; both sqrts, interleaved twice.
set -e
OUT=$GRAFT_REPO_ROOT/${1:-gpurun_out/r03_s21}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
for i in 1 2; do
  for K in 8 16 32 48; do
    for B in 1 2; do
      for S in ieee torch_cpu_amd; do
        timeout -k 10 300 python bench.py --clients $K --params 2.5e8 --epilogue adam --sqrt $S --blocks-per-cu $B --also none --no-cpu-baseline --steps 10 > "$OUT/k${K}_b${B}_${S}_$i.jsonl" 2> "$OUT/k${K}_b${B}_${S}_$i.err"
      done
    done
  done
done
