#!/bin/bash
# Round-4 GPU batch s: the fc7 weight-gradient fork merged into fc6's
# (PoseStep.merge_w7_fork, bench --merge-w7) against the default, same tree.
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
O=gpurun_out; mkdir -p $O
: > $O/merge_w7_ab.log
for i in 1 2 3; do
  for v in default merge; do
    F=""; [ $v = merge ] && F=--merge-w7
    echo "== $v" >> $O/merge_w7_ab.log
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-fp32-leg --steps 30 $F 2>/dev/null | \
      python -c "import json,sys; d=json.load(sys.stdin); print('step', d['value'], d['timing_ms_per_step'], d['step_ms_distribution']['median'])" \
      >> $O/merge_w7_ab.log || exit 1
  done
done
echo "exit=0"
