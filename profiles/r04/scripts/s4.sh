# GPU session 4 (round 4): is the constant-divisor quotient (Markstein's correction from RN(1/b)) the IEEE quotient for
# every dividend significand, for integer / fractional / random / all divisor significands; the launch-form parity
# tests on the remainder-form build; the host-resident config-2 round with the staging drain attributed and the
# cyclic collector frozen.
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04_s4
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/div_const_probe.py > "$OUT/div_probe.jsonl" 2> "$OUT/div_probe.err" || exit $?
timeout -k 10 300 python -u tools/div_const_probe.py --all > "$OUT/div_probe_all.jsonl" 2> "$OUT/div_probe_all.err" || exit $?
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py > "$OUT/pytest_parity.log" 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --config 2 --also 2h --no-cpu-baseline --steps 10 > "$OUT/bench_2h.jsonl" 2> "$OUT/bench_2h.err" || exit $?
ab() { local name=$1; shift; timeout -k 10 300 python -u tools/ab_variants.py "$@" --rounds 3 > "$OUT/$name.jsonl" 2> "$OUT/$name.err"; }
ab divc_k2 --clients 2 --params 1e9 --variants 8,256 --epilogues none --check || exit $?
ab divc_k3 --clients 3 --params 1e9 --variants 8,256 --epilogues none --check || exit $?
ab divc_k4 --clients 4 --params 5e8 --variants 0,8 --epilogues none --check || exit $?
ab divc_k1 --clients 1 --params 1e9 --variants 8,256 --epilogues none --check || exit $?
