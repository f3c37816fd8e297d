# gpu_roi_ab.sh V1 V2 ...: RoI pool timings of the in-tree library and of each scratch/V.so
cd $GRAFT_REPO_ROOT
echo "== tree" > gpurun_out/roi_ab.log &&
timeout -k 10 120 python scripts/roi_bench.py >> gpurun_out/roi_ab.log 2>&1 || exit 1
for v in "$@"; do echo "== $v" >> gpurun_out/roi_ab.log; POSECNN_HIP_LIB=$GRAFT_REPO_ROOT/scratch/$v.so timeout -k 10 120 python scripts/roi_bench.py >> gpurun_out/roi_ab.log 2>&1 || exit 1; done
echo "exit=0"
