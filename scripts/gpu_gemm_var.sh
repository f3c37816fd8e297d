# GEMM parity of scratch/$1.so, then gemm_bench of the tree and of each scratch/V.so
cd $GRAFT_REPO_ROOT
POSECNN_HIP_LIB=$GRAFT_REPO_ROOT/scratch/$1.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k gemm > gpurun_out/t_gemm_var.log 2>&1 || exit 1
echo "== tree" > gpurun_out/gemm_var.log
timeout -k 10 300 python scripts/gemm_bench.py >> gpurun_out/gemm_var.log 2>&1 || exit 1
for v in "$@"; do echo "== $v" >> gpurun_out/gemm_var.log; POSECNN_HIP_LIB=$GRAFT_REPO_ROOT/scratch/$v.so timeout -k 10 300 python scripts/gemm_bench.py >> gpurun_out/gemm_var.log 2>&1 || exit 1; done
echo "exit=0"
