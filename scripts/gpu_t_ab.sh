# gpu_t_ab.sh V1 V2 ...: the GEMM tests against each scratch/V.so
cd $GRAFT_REPO_ROOT
for v in "$@"; do echo "== $v" >> gpurun_out/t_ab.log; POSECNN_HIP_LIB=$GRAFT_REPO_ROOT/scratch/$v.so timeout -k 10 300 python -m pytest tests/test_gpu_ops.py -m gpu -q -p no:cacheprovider -k gemm 2>&1 | tail -3 >> gpurun_out/t_ab.log; done
echo "exit=0"
