# RoI op parity + RoI microbench (+ stamps / variants from scratch/); each GPU step time-limited, chained
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -q -p no:cacheprovider -x -k roi --timeout 120 --timeout-method thread > gpurun_out/t_roi.log 2>&1 &&
timeout -k 10 120 python scripts/roi_bench.py > gpurun_out/roi_bench.log 2>&1 || exit 1
if [ -f scratch/rb_stamp.so ]; then POSECNN_HIP_LIB=$GRAFT_REPO_ROOT/scratch/rb_stamp.so timeout -k 10 120 python scripts/roi_stamp.py > gpurun_out/roi_stamp.log 2>&1 || exit 1; fi
for v in "$@"; do echo "== $v" >> gpurun_out/roi_bench.log; POSECNN_HIP_LIB=$GRAFT_REPO_ROOT/scratch/$v.so timeout -k 10 120 python scripts/roi_bench.py >> gpurun_out/roi_bench.log 2>&1 || exit 1; done
echo "exit=0"
