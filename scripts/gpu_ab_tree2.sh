# ADD/parity tests of the tree, then bench of the tree vs scratch/prev, alternating
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_golden.py tests/test_gpu_pth.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "add or golden or module" > gpurun_out/t_add.log 2>&1 || exit 1
bash scripts/gpu_ab_tree.sh
