#!/bin/bash
# Round-4 GPU batch k: estimatePose2D after the wave-per-column list building:
# parity, timing and kernel trace.
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_pose2d.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $O/t_k.log 2>&1 || { echo "tests failed"; exit 1; }
timeout -k 10 300 python scripts/pose2d_bench.py > $O/pose2d_bench.json 2> $O/pose2d_bench.err || exit 1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_p2d -o run -- \
   python3 $GRAFT_REPO_ROOT/scripts/pose2d_bench.py --no-cpu --iters 5 > $GRAFT_REPO_ROOT/$O/prof_p2d.log 2>&1) || exit 1
echo "exit=0"
