#!/bin/bash
# round-6 call T: the default bench line five times on one box (run-to-run spread)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R; export TMPDIR=/tmp
ulimit -c 0
: > $O/bench_repeat.log
for i in 1 2 3 4 5; do
  timeout -k 10 300 python bench.py --no-cpu-baseline 2>>$O/bench_repeat.err | \
    python -c "import json,sys; d=json.load(sys.stdin); print('run$i', d['value'], d['timing_ms_per_step'], d['step_ms_distribution']['median'], d['roofline']['frac'])" >> $O/bench_repeat.log || exit 1
done
cat $O/bench_repeat.log
