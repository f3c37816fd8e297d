# NMS GPU parity; time-limited
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_nms.py -m gpu -q -p no:cacheprovider -x --timeout 120 --timeout-method thread > gpurun_out/t_nms.log 2>&1
echo "exit=$?"
