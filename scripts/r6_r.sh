#!/bin/bash
# round-6 call R: the prefetched RoI-pool forward issued at the tail (pool_at_tail), A/B against the loss fork
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R; export TMPDIR=/tmp
ulimit -c 0
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/t_pipe.log 2>&1 || { tail -30 $O/t_pipe.log; exit 1; }
tail -2 $O/t_pipe.log
: > $O/pool_tail_ab.log
for i in 1 2 3; do
  for v in base tail; do
    X=""; [ $v = tail ] && X="--pool-at-tail"
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-fp32-leg --no-graph --steps 40 $X 2>>$O/pool_tail_ab.err | \
      python -c "import json,sys; d=json.load(sys.stdin); print('$v', d['value'], d['timing_ms_per_step'])" >> $O/pool_tail_ab.log || exit 1
  done
done
cat $O/pool_tail_ab.log
