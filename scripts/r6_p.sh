#!/bin/bash
# round-6 call P: one profiled step timeline of the tree (eager)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R; export TMPDIR=/tmp
ulimit -c 0
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/prof_p -o run -- \
   python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-fp32-leg --no-graph > $O/prof_p.log 2>&1) || exit 1
python scripts/timeline.py $O/prof_p/run_kernel_trace.csv > $O/timeline_p.txt; cat $O/timeline_p.txt
