#!/bin/bash
# Round-4 GPU batch q: the pruned ADD-S nearest-point search (Morton-ordered
# candidates with bounding boxes): ADD parity, step parity, ADD op timing and
# the whole step against the previous tree (scratch/prev_tree, built from HEAD).
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
O=$PWD/gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_golden.py -m gpu -x -v --timeout 120 \
  --timeout-method thread -p no:cacheprovider -k "add" > $O/t_q1.log 2>&1 || { echo "add tests failed"; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $O/t_q2.log 2>&1 || { echo "suite failed"; exit 1; }
: > $O/add_prune_ab.log
for i in 1 2 3; do
  for v in tree prev; do
    D=$PWD; [ $v = prev ] && D=$PWD/scratch/prev_tree
    echo "== $v" >> $O/add_prune_ab.log
    (cd $D && timeout -k 10 300 python bench.py --no-cpu-baseline --no-fp32-leg --steps 30 2>/dev/null) | \
      python -c "import json,sys; d=json.load(sys.stdin); print('step', d['value'], d['timing_ms_per_step'], 'head_add_loss_fwd', d['ops_ms_per_step']['head_add_loss_fwd'])" \
      >> $O/add_prune_ab.log || exit 1
  done
done
echo "exit=0"
