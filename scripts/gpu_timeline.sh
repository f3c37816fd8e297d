# kernel trace of the eager and graph steps (timeline of one step: scripts/timeline.py)
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tl_eager -o run -- python3 $R/bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-graph > $R/gpurun_out/tl_eager.log 2>&1
echo "exit=$?"
