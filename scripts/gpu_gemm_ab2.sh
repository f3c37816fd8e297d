# GEMM parity of each scratch/V.so + GEMM microbench of the tree and each variant
cd $GRAFT_REPO_ROOT
echo "== tree" > gpurun_out/ab.log
timeout -k 10 300 python -m pytest tests/test_gpu_ops.py -m gpu -q -p no:cacheprovider -x -k gemm > gpurun_out/t_gemm.log 2>&1 &&
timeout -k 10 120 python scripts/gemm_bench.py >> gpurun_out/ab.log 2>&1 || exit 1
for v in "$@"; do
  echo "== $v" >> gpurun_out/ab.log
  POSECNN_HIP_LIB=$GRAFT_REPO_ROOT/scratch/$v.so timeout -k 10 300 python -m pytest tests/test_gpu_ops.py -m gpu -q -p no:cacheprovider -x -k gemm >> gpurun_out/t_gemm.log 2>&1 &&
  POSECNN_HIP_LIB=$GRAFT_REPO_ROOT/scratch/$v.so timeout -k 10 120 python scripts/gemm_bench.py >> gpurun_out/ab.log 2>&1 || exit 1
done
echo "exit=0"
