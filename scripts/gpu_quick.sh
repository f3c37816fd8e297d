# quick GPU iteration: op parity, GEMM microbench, full bench (each step time-limited, chained with &&)
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_gpu_ops.py tests/test_gpu_pth.py -m gpu -q -p no:cacheprovider -x > gpurun_out/t_ops.log 2>&1 &&
timeout -k 10 300 python scripts/gemm_bench.py > gpurun_out/gemm_bench.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
echo "exit=$?"
