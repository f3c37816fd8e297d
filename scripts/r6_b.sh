#!/bin/bash
# round-6 call B: pipeline / fused-loss-tail parity, A/B of the fused tail, kernel trace + SQ of the pipelined step
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_step.py tests/test_gpu_step_full.py \
  tests/test_gpu_head.py tests/test_gpu_dist.py tests/test_gpu_ops.py -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > $O/b_tests.log 2>&1 || { echo tests failed; exit 1; }
: > $O/b_ab.log
for i in 1 2; do
  for m in fused unfused; do
    a=""; [ $m = unfused ] && a="--no-fuse-loss-tail"
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-fp32-leg --steps 30 $a > $O/b_b_${m}_$i.json 2> $O/b_b_${m}_$i.err || { echo bench $m failed; exit 1; }
    python -c "import json,sys; d=json.load(open('$O/b_b_${m}_$i.json')); print('$m', d['value'], d['timing_ms_per_step'], d['ops_ms_per_step'].get('head_add_loss_fwd'))" >> $O/b_ab.log
  done
done
cat $O/b_ab.log
bash scripts/gpu.sh prof sq || exit 1
echo done
