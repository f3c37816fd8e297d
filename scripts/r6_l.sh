#!/bin/bash
# round-6 call L: the "fwd" fork point (prefetch issued by the host after the fc6 forward's launch)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/t_pipe.log 2>&1 || { tail -20 $O/t_pipe.log; exit 1; }
tail -2 $O/t_pipe.log
: > $O/fork_fwd_ab.log
for i in 1 2 3; do
  for f in start fwd; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-fp32-leg --steps 40 --prefetch-at $f 2>/dev/null | \
      python -c "import json,sys; d=json.load(sys.stdin); print('$f', d['value'], d['timing_ms_per_step'])" >> $O/fork_fwd_ab.log || exit 1
  done
done
cat $O/fork_fwd_ab.log
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/prof_fwd -o run -- \
   python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-fp32-leg --no-graph --prefetch-at fwd > $O/prof_fwd.log 2>&1) || exit 1
python scripts/timeline.py $O/prof_fwd/run_kernel_trace.csv > $O/timeline_fwd.txt; cat $O/timeline_fwd.txt
