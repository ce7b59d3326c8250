export TMPDIR=/tmp; mkdir -p gpurun_out
B="python bench.py --epilogue adam --steps 3 --warmup 1 --no-cpu-baseline --spot-check 0"
timeout -k 10 300 python -m pytest tests/test_gpu_fedopt.py -x -q > gpurun_out/pytest_fedopt.log 2>&1 &&
timeout -k 10 300 python bench.py --epilogue adam --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_adam2.jsonl 2>&1 &&
timeout -k 10 300 python bench.py --epilogue sgd --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_sgd2.jsonl 2>&1 &&
timeout -k 10 300 python bench.py --epilogue add_base --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_addbase2.jsonl 2>&1 &&
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_adam -o kt -- python $GRAFT_REPO_ROOT/bench.py --epilogue adam --steps 3 --warmup 1 --no-cpu-baseline --spot-check 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_adam.log 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $GRAFT_REPO_ROOT/gpurun_out/pmc_adam -o fetch -- python $GRAFT_REPO_ROOT/bench.py --epilogue adam --steps 2 --warmup 1 --no-cpu-baseline --spot-check 0 > $GRAFT_REPO_ROOT/gpurun_out/pmc_adam_fetch.log 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $GRAFT_REPO_ROOT/gpurun_out/pmc_adam -o write -- python $GRAFT_REPO_ROOT/bench.py --epilogue adam --steps 2 --warmup 1 --no-cpu-baseline --spot-check 0 > $GRAFT_REPO_ROOT/gpurun_out/pmc_adam_write.log 2>&1
