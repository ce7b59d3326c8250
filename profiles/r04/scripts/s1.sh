# GPU session 1 (round 4): the few-client read/write mix ceilings (R = 1..4 reads per result write; VERDICT r03
# item 2) with the multi forms (G chunks' loads in flight per lane, stores immediate / deferred) next to the
# library's kernel on the same box; the few-client bench baselines; the round's new GPU tests (run-time RSQRTPS
# table, short sqrt calls, independent sharded FedOpt weights, live sqrt guard); config 5 at full size in every
# sqrt (item 1).
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04_s1
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 300 "$@" > "$OUT/$name.jsonl" 2> "$OUT/$name.err"; }
for R in 2 1 3 4; do
  run mix_r$R python -u tools/hbm_mix_probe.py --ratio $R --params 5e8 --preset few --rounds 3 || exit $?
done
for K in 1 2 3; do
  run k${K}_plain python -u bench.py --clients $K --params 1e9 --also none --no-cpu-baseline --steps 10 || exit $?
  run k${K}_adam python -u bench.py --clients $K --params 5e8 --epilogue adam --also none --no-cpu-baseline --steps 10 || exit $?
done
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_torch_sqrt.py tests/test_gpu_sharded_fedopt.py tests/test_gpu_fedopt_ctl.py > "$OUT/pytest_new.log" 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 500 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_fullsize.log" 2>&1
