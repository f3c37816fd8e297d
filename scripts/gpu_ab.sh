# gpu_ab.sh V1 V2 ...: GEMM timings of the in-tree library and of each scratch/V.so
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_gpu_ops.py -m gpu -q -p no:cacheprovider -x -k gemm > gpurun_out/t_gemm.log 2>&1 &&
echo "== tree" > gpurun_out/ab.log &&
timeout -k 10 120 python scripts/gemm_bench.py >> gpurun_out/ab.log 2>&1 || exit 1
for v in "$@"; do echo "== $v" >> gpurun_out/ab.log; POSECNN_HIP_LIB=$GRAFT_REPO_ROOT/scratch/$v.so timeout -k 10 120 python scripts/gemm_bench.py >> gpurun_out/ab.log 2>&1 || exit 1; done
echo "exit=0"
