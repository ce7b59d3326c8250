# GPU box script: the system-level measurements of DESIGN.md sections 4, 8 and 10 re-taken on the burst
# kernels -- host-array e2e (PCIe-inclusive), round-end get_result latency, SAG FedOpt round end eager vs
# deferred, FedOpt controller round end.  Each step under its own time limit; `set -e` stops at a failure.
set -e
OUT=${1:-gpurun_out/r02_system}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/e2e_bench.py --clients 8 --params 1.25e8 > "$OUT/e2e_numpy_1key.jsonl" 2> "$OUT/e2e_1.err"
timeout -k 10 300 python tools/e2e_bench.py --clients 8 --params 1.25e8 --keys 437 > "$OUT/e2e_numpy_437keys.jsonl" 2> "$OUT/e2e_437.err"
timeout -k 10 300 python tools/result_latency.py --clients 8 --params 1e9 > "$OUT/result_latency_8x1e9.jsonl" 2> "$OUT/rl.err"
timeout -k 10 300 python tools/sag_fedopt_bench.py --rounds 6 > "$OUT/sag_eager_1key.jsonl" 2> "$OUT/sag_e.err"
timeout -k 10 300 python tools/sag_fedopt_bench.py --rounds 6 --defer > "$OUT/sag_defer_1key.jsonl" 2> "$OUT/sag_d.err"
timeout -k 10 300 python tools/sag_fedopt_bench.py --rounds 6 --keys 437 > "$OUT/sag_eager_437keys.jsonl" 2> "$OUT/sag_e437.err"
timeout -k 10 300 python tools/sag_fedopt_bench.py --rounds 6 --keys 437 --defer > "$OUT/sag_defer_437keys.jsonl" 2> "$OUT/sag_d437.err"
timeout -k 10 400 python tools/sag_fedopt_bench.py --rounds 4 --params 1e9 --defer > "$OUT/sag_defer_8x1e9.jsonl" 2> "$OUT/sag_d1e9.err"
timeout -k 10 300 python tools/fedopt_ctl_bench.py --rounds 4 --defer > "$OUT/fedopt_ctl_defer.jsonl" 2> "$OUT/ctl_d.err"
