#!/bin/bash
# round-6 call D: ADD microbench (pruned vs full), kernel stats, parity
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R; export TMPDIR=/tmp
timeout -k 10 300 python scripts/add_bench.py > $O/d_add.log 2>&1 || { cat $O/d_add.log; exit 1; }
timeout -k 10 300 python scripts/add_bench.py --near >> $O/d_add.log 2>&1 || { cat $O/d_add.log; exit 1; }
cat $O/d_add.log
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/d_prof -o run -- python3 $R/scripts/add_bench.py --iters 10 > $O/d_prof.log 2>&1) || exit 1
python scripts/kstats.py $O/d_prof/run_kernel_stats.csv 2>/dev/null | head -20 || head -20 $O/d_prof/run_kernel_stats.csv
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -x -q -k "add" --timeout 180 --timeout-method thread -p no:cacheprovider > $O/d_tests.log 2>&1 || { tail -30 $O/d_tests.log; exit 1; }
tail -2 $O/d_tests.log
