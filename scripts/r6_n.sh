#!/bin/bash
# round-6 call N: host-side A/B of the tree against scratch/prev (the previous commit's posecnn_amd + bench.py)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R; export TMPDIR=/tmp
ulimit -c 0
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_step_full.py tests/test_gpu_ops.py tests/test_gpu_gemm_fc6.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > $O/t_n.log 2>&1 || { tail -30 $O/t_n.log; exit 1; }
tail -2 $O/t_n.log
: > $O/host_ab.log
for i in 1 2 3; do
  for v in prev tree; do
    B=bench.py; [ $v = prev ] && B=scratch/prev/bench.py
    timeout -k 10 300 python $B --no-cpu-baseline --no-fp32-leg --steps 40 2>>$O/host_ab.err | \
      python -c "import json,sys; d=json.load(sys.stdin); print('$v', d['value'], d['timing_ms_per_step'])" >> $O/host_ab.log || exit 1
  done
done
cat $O/host_ab.log
