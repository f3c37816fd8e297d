#!/bin/bash
# Round-4 GPU batch f: estimatePose2D after the threaded host subsets (parity,
# timing, kernel trace), then the in-reduce dropout bits vs the mask kernel
# on the whole step (same-box A/B).
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_pose2d.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $O/t_f.log 2>&1 || { echo "tests failed"; exit 1; }
timeout -k 10 300 python scripts/pose2d_bench.py > $O/pose2d_bench.json 2> $O/pose2d_bench.err || exit 1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_p2d -o run -- \
   python3 $GRAFT_REPO_ROOT/scripts/pose2d_bench.py --no-cpu --iters 5 > $GRAFT_REPO_ROOT/$O/prof_p2d.log 2>&1) || exit 1
: > $O/maskk_ab.log
for i in 1 2 3; do
  for v in reduce kernel; do
    a=""; [ $v = kernel ] && a="--mask-kernel"
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-fp32-leg --steps 30 $a 2>/dev/null | \
      python -c "import json,sys; d=json.load(sys.stdin); print('$v', d['value'], d['timing_ms_per_step'])" \
      >> $O/maskk_ab.log || exit 1
  done
done
echo "exit=0"
