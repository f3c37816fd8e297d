#!/bin/bash
# round-6 call C: pruned ADD-S search parity + A/B (pruned vs full scan; pipeline fork points), timeline
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 700 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_pipeline.py tests/test_gpu_step.py \
  tests/test_gpu_step_full.py tests/test_gpu_golden.py -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > $O/c_tests.log 2>&1 || { echo tests failed; tail -30 $O/c_tests.log; exit 1; }
: > $O/c_ab.log
for i in 1 2; do
  for m in pruned full off loss; do
    a=""; e=""
    [ $m = full ] && e="PCNN_ADD_SEARCH=full"
    [ $m = off ] && a="--pipeline off"
    [ $m = loss ] && a="--prefetch-at loss"
    env $e timeout -k 10 300 python bench.py --no-cpu-baseline --no-fp32-leg --steps 30 $a > $O/c_b_${m}_$i.json 2> $O/c_b_${m}_$i.err || { echo bench $m failed; exit 1; }
    python -c "import json,sys; d=json.load(open('$O/c_b_${m}_$i.json')); print('$m', d['value'], d['timing_ms_per_step'], d['ops_ms_per_step'].get('head_add_loss_fwd'))" >> $O/c_ab.log
  done
done
cat $O/c_ab.log
bash scripts/gpu.sh prof || exit 1
python scripts/timeline.py $O/prof/run_kernel_trace.csv 3 > $O/c_timeline.txt
echo done
