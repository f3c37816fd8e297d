#!/bin/bash
# Round-4 GPU batch p: the scalar ADD loss folded on the side stream
# (pcnn_add_loss_fwd_rows + pcnn_add_loss_total): parity, then step A/B
# against --loss-on-main in the same tree.
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_step_full.py tests/test_gpu_ops.py \
  tests/test_gpu_dist.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $O/t_p.log 2>&1 || { echo "tests failed"; exit 1; }
: > $O/loss_side_ab.log
for i in 1 2 3; do
  for v in side main; do
    F=""; [ $v = main ] && F=--loss-on-main
    echo "== $v" >> $O/loss_side_ab.log
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-fp32-leg --steps 30 $F 2>/dev/null | \
      python -c "import json,sys; d=json.load(sys.stdin); print('step', d['value'], d['timing_ms_per_step'])" \
      >> $O/loss_side_ab.log || exit 1
  done
done
echo "exit=0"
