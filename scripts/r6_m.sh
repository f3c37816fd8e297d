#!/bin/bash
# round-6 call M: deferred weight-gradient join (tests + same-box A/B + one profiled step)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R; export TMPDIR=/tmp
ulimit -c 0
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/t_pipe.log 2>&1 || { tail -30 $O/t_pipe.log; exit 1; }
tail -3 $O/t_pipe.log
timeout -k 10 200 python bench.py --no-cpu-baseline --no-fp32-leg --steps 10 --defer-side-join on > $O/d2.json 2> $O/d2.err || { tail -5 $O/d2.err; exit 1; }
: > $O/defer_ab.log
for i in 1 2 3; do
  for d in off on; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-fp32-leg --steps 40 --defer-side-join $d 2>>$O/defer_ab.err | \
      python -c "import json,sys; d=json.load(sys.stdin); print('defer-$d', d['value'], d['timing_ms_per_step'])" >> $O/defer_ab.log || exit 1
  done
done
cat $O/defer_ab.log
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/prof_defer -o run -- \
   python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-fp32-leg --no-graph --defer-side-join on > $O/prof_defer.log 2>&1) || exit 1
python scripts/timeline.py $O/prof_defer/run_kernel_trace.csv > $O/timeline_defer.txt; cat $O/timeline_defer.txt
