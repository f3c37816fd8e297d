# iteration loop on one MI355X: op parity, default bench line, kernel-trace stats (each GPU step time-limited, chained)
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_hough.py -m gpu -q -p no:cacheprovider -x --timeout 120 --timeout-method thread > gpurun_out/t_ops.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err &&
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-graph > $R/gpurun_out/prof.log 2>&1
echo "exit=$?"
