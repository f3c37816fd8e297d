# Hough parity (GPU) + microbench; each GPU step time-limited, chained
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_hough.py tests/test_gpu_golden.py tests/test_gpu_pth.py -m gpu -q -p no:cacheprovider -x --timeout 120 --timeout-method thread > gpurun_out/t_hough.log 2>&1 &&
timeout -k 10 120 python scripts/hough_bench.py > gpurun_out/hough_bench.log 2>&1 &&
timeout -k 10 120 python scripts/hough_bench.py --batch 1 --test >> gpurun_out/hough_bench.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/hough_kt -o run -- python3 $GRAFT_REPO_ROOT/scripts/hough_bench.py --iters 10 > $GRAFT_REPO_ROOT/gpurun_out/hough_kt.log 2>&1
echo "exit=$?"
