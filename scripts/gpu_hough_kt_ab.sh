# per-kernel Hough stats for the in-tree library and each scratch/V.so
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in tree "$@"; do
  if [ $v = tree ]; then L=$R/posecnn_amd/libposecnn_hip.so; else L=$R/scratch/$v.so; fi
  POSECNN_HIP_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/hkt_$v -o run -- python3 $R/scripts/hough_bench.py --iters 10 > $R/gpurun_out/hkt_$v.log 2>&1 || exit 1
done
echo "exit=0"
