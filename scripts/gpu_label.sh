# Label producer parity + microbench on one MI355X.
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_label.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_label.log 2>&1 &&
timeout -k 10 300 python scripts/label_bench.py > gpurun_out/label_bench.json 2> gpurun_out/label_bench.err
echo "exit=$?"
