#!/bin/bash
# round-6 call S: the step stream at high priority with the final schedule
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R; export TMPDIR=/tmp
ulimit -c 0
: > $O/prio_ab.log
for i in 1 2 3; do
  for v in normal high; do
    X=""; [ $v = high ] && X="--step-priority high"
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-fp32-leg --no-graph --steps 40 $X 2>>$O/prio_ab.err | \
      python -c "import json,sys; d=json.load(sys.stdin); print('$v', d['value'], d['timing_ms_per_step'])" >> $O/prio_ab.log || exit 1
  done
done
cat $O/prio_ab.log
