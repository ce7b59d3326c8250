# GPU box script (round 3, session 15): the fused kernel's epilogue phase with two tiles of operand loads in flight
# (one-block-per-CU form) -- full `pytest -m gpu` on the new build, then config 5 (fused Adam, both sqrts) on the new
# library and on HEAD's (nvflare_amd/lib/ab/libnvflare_amd_fedavg_head.so, tools/build_rev_lib.py), interleaved three
# times on the same box.
set -e
OUT=$GRAFT_REPO_ROOT/${1:-gpurun_out/r03_s15}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
HEADLIB=$GRAFT_REPO_ROOT/nvflare_amd/lib/ab/libnvflare_amd_fedavg_head.so
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
for i in 1 2 3; do
  for S in ieee torch_cpu_amd; do
    timeout -k 10 300 python bench.py --config 5 --sqrt $S --no-cpu-baseline > "$OUT/c5_${S}_new_$i.jsonl" 2> "$OUT/c5_${S}_new_$i.err"
    NVFLARE_AMD_FEDAVG_LIB=$HEADLIB timeout -k 10 300 python bench.py --config 5 --sqrt $S --no-cpu-baseline > "$OUT/c5_${S}_head_$i.jsonl" 2> "$OUT/c5_${S}_head_$i.err"
  done
done
