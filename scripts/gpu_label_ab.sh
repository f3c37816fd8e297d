# label_bench.py of the in-tree library and of each scratch/V.so
cd $GRAFT_REPO_ROOT
echo "== tree" > gpurun_out/label_ab.log
timeout -k 10 120 python scripts/label_bench.py >> gpurun_out/label_ab.log 2>&1 || exit 1
for v in "$@"; do echo "== $v" >> gpurun_out/label_ab.log; POSECNN_HIP_LIB=$GRAFT_REPO_ROOT/scratch/$v.so timeout -k 10 120 python scripts/label_bench.py >> gpurun_out/label_ab.log 2>&1 || exit 1; done
echo "exit=0"
