# RoI parity (tree) + roi_bench of the tree and of each scratch/V.so
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_golden.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "roi or golden" > gpurun_out/t_roi.log 2>&1 || exit 1
echo "== tree" > gpurun_out/roi_var.log
timeout -k 10 120 python scripts/roi_bench.py >> gpurun_out/roi_var.log 2>&1 || exit 1
for v in "$@"; do echo "== $v" >> gpurun_out/roi_var.log; POSECNN_HIP_LIB=$GRAFT_REPO_ROOT/scratch/$v.so timeout -k 10 120 python scripts/roi_bench.py >> gpurun_out/roi_var.log 2>&1 || exit 1; done
echo "exit=0"
