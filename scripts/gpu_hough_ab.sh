# Hough timings (B=8 train, B=1 test) of the in-tree library and of each scratch/V.so
cd $GRAFT_REPO_ROOT
echo "== tree" > gpurun_out/hough_ab.log
timeout -k 10 120 python scripts/hough_bench.py >> gpurun_out/hough_ab.log 2>&1 &&
timeout -k 10 120 python scripts/hough_bench.py --batch 1 --test >> gpurun_out/hough_ab.log 2>&1 || exit 1
for v in "$@"; do echo "== $v" >> gpurun_out/hough_ab.log; POSECNN_HIP_LIB=$GRAFT_REPO_ROOT/scratch/$v.so timeout -k 10 120 python scripts/hough_bench.py >> gpurun_out/hough_ab.log 2>&1 && POSECNN_HIP_LIB=$GRAFT_REPO_ROOT/scratch/$v.so timeout -k 10 120 python scripts/hough_bench.py --batch 1 --test >> gpurun_out/hough_ab.log 2>&1 || exit 1; done
echo "exit=0"
