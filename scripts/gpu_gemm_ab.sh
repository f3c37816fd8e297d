cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_gpu_ops.py -m gpu -q -p no:cacheprovider -x -k gemm > gpurun_out/t_gemm.log 2>&1 &&
PCNN_GEMM_X3=1 timeout -k 10 300 python -m pytest tests/test_gpu_ops.py -m gpu -q -p no:cacheprovider -x -k gemm >> gpurun_out/t_gemm.log 2>&1 &&
echo "== x4" > gpurun_out/gemm_bench.log && timeout -k 10 300 python scripts/gemm_bench.py >> gpurun_out/gemm_bench.log 2>&1 &&
echo "== x3" >> gpurun_out/gemm_bench.log && PCNN_GEMM_X3=1 timeout -k 10 300 python scripts/gemm_bench.py >> gpurun_out/gemm_bench.log 2>&1
echo "exit=$?"
