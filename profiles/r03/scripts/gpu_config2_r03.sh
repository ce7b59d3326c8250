# GPU box script (round 3): config 2 (8 clients x 125 M fp32) evidence -- the 8:1 read/write mix probe next to the
# real kernel, the bench line, a rocprofv3 kernel trace of the bench command and its PMC FETCH/WRITE passes.
# Every GPU step has its own time limit; `set -e` ends the script at the first failure.
set -e
OUT=$GRAFT_REPO_ROOT/${1:-gpurun_out/r03_config2}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
B="bench.py --clients 8 --params 1.25e8"
timeout -k 10 240 python tools/hbm_mix_probe.py --ratio 8 --params 1.25e8 --rounds 5 > "$OUT/mix_probe_r8.jsonl" 2> "$OUT/mix_probe_r8.err"
timeout -k 10 240 python $B --steps 50 > "$OUT/bench_config2.jsonl" 2> "$OUT/bench_config2.err"
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rocprof_config2" -o c2 -- python $GRAFT_REPO_ROOT/$B --steps 50 --no-cpu-baseline > "$OUT/bench_config2_prof.jsonl" 2> "$OUT/bench_config2_prof.err"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_$C" -o pmc -- python $GRAFT_REPO_ROOT/$B --steps 2 --warmup 1 --no-cpu-baseline --spot-check 0 > "$OUT/pmc_$C.log" 2>&1
done
