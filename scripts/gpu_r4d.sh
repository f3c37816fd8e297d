#!/bin/bash
# Round-4 GPU batch d: the ICP / step parity tests touched by the grid score
# search and the side_prep option, then a same-box A/B of the step with the
# post-vote work on the side stream (default) vs on the step's stream, and the
# refinement timings.  Stops at the first failure.
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_icp.py tests/test_gpu_step.py tests/test_gpu_dropout.py tests/test_gpu_step_full.py -m gpu -x -v --timeout 300 \
  --timeout-method thread -p no:cacheprovider > $O/t_d.log 2>&1 || { echo "tests failed"; exit 1; }
: > $O/prep_ab.log
for i in 1 2 3; do
  for v in side main; do
    a=""; [ $v = main ] && a="--prep-on-main"
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-fp32-leg --steps 30 $a 2>/dev/null | \
      python -c "import json,sys; d=json.load(sys.stdin); print('$v', d['value'], d['timing_ms_per_step'])" \
      >> $O/prep_ab.log || exit 1
  done
done
timeout -k 10 300 python scripts/icp_bench.py > $O/icp_bench.json 2> $O/icp_bench.err || exit 1
echo "exit=0"
