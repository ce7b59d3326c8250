# GPU box script: PMC HBM traffic of the bench kernels on the current build, FETCH_SIZE and WRITE_SIZE in
# separate rocprofv3 passes (the program itself directly after --), each under its own hard time limit.
# Usage: bash tools/gpu_pmc_bench.sh OUT_DIR [EPILOGUE ...]   (EPILOGUE: none | adam | sgd | ...; default none)
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/${1:-gpurun_out/pmc_bench}
shift || true
EPIS=${@:-none}
mkdir -p "$OUT"
cd /tmp
for E in $EPIS; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d "$OUT/${E}_$C" -o pmc -- python $R/bench.py --epilogue $E --steps 2 --warmup 1 --no-cpu-baseline --spot-check 0 > "$OUT/${E}_$C.log" 2>&1
  done
done
