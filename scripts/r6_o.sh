#!/bin/bash
# round-6 call O: HIP-graph replay with 2 / 4 / 8 pipelined steps per replay
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R; export TMPDIR=/tmp
ulimit -c 0
: > $O/graph_rep.log
for i in 1 2; do
  for g in 1 2 4; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-fp32-leg --steps 40 --graph-repeat $g 2>>$O/graph_rep.err | \
      python -c "import json,sys; d=json.load(sys.stdin); print('rep$g', d['value'], d['timing_ms_per_step'])" >> $O/graph_rep.log || exit 1
  done
done
cat $O/graph_rep.log
