cd $GRAFT_REPO_ROOT
timeout -k 10 120 python scripts/hough_bench.py > gpurun_out/abl.log 2>&1 &&
for v in rows inner atomexact; do POSECNN_HIP_LIB=$GRAFT_REPO_ROOT/scratch/abl_$v.so timeout -k 10 120 python scripts/hough_bench.py >> gpurun_out/abl.log 2>&1 || exit 1; done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/profh -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/hough_bench.py > $GRAFT_REPO_ROOT/gpurun_out/profh.log 2>&1
echo "exit=$?"
