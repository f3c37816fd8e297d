#!/bin/bash
# round-6 call K: RoI-pool backward (pixel-argmax form) alone: timing + SQ counters
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R; export TMPDIR=/tmp
timeout -k 10 200 python scripts/roi_bench.py --px --iters 50 > $O/roi_px.log 2>&1 || exit 1
cat $O/roi_px.log
bash scripts/gpu.sh sqmicro roi_bench "--px --iters 5" "" || exit 1
python3 scripts/sq_summary.py $O/sq_tree_1 $O/sq_tree_2 --grep=k_roi > $O/roi_sq.txt; cat $O/roi_sq.txt
