# full GPU parity suite, GEMM microbench and the default bench line (each step time-limited, chained)
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/t_gpu.log 2>&1 &&
timeout -k 10 300 python scripts/gemm_bench.py > gpurun_out/gemm_bench.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
echo "exit=$?"
