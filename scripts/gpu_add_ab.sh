# ADD parity + timings of the in-tree library and each scratch/V.so
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -q -p no:cacheprovider -x -k "add or average" --timeout 120 --timeout-method thread > gpurun_out/t_add.log 2>&1 || exit 1
echo "== tree" > gpurun_out/add_ab.log
timeout -k 10 120 python scripts/add_bench.py >> gpurun_out/add_ab.log 2>&1 || exit 1
for v in "$@"; do echo "== $v" >> gpurun_out/add_ab.log; POSECNN_HIP_LIB=$GRAFT_REPO_ROOT/scratch/$v.so timeout -k 10 120 python scripts/add_bench.py >> gpurun_out/add_ab.log 2>&1 || exit 1; done
echo "exit=0"
