#!/bin/bash
# round-6 call Q: fork points again under the deferred join + signalled forks
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R; export TMPDIR=/tmp
ulimit -c 0
: > $O/fork_q.log
for i in 1 2 3; do
  for f in start loss bwd tail; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-fp32-leg --no-graph --steps 40 --prefetch-at $f 2>>$O/fork_q.err | \
      python -c "import json,sys; d=json.load(sys.stdin); print('$f', d['value'], d['timing_ms_per_step'])" >> $O/fork_q.log || exit 1
  done
done
cat $O/fork_q.log
