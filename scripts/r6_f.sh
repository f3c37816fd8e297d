#!/bin/bash
# round-6 call F: same-box A/B of the pipelined step's fork point and the step stream's priority
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
: > $O/f_ab.log
for i in 1 2; do
  for m in off start starthi losshi offhi bwdhi; do
    case $m in
      off) a="--pipeline off";; start) a="--prefetch-at start";; starthi) a="--prefetch-at start --step-priority high";;
      losshi) a="--prefetch-at loss --step-priority high";; offhi) a="--pipeline off --step-priority high";;
      bwdhi) a="--prefetch-at bwd --step-priority high";;
    esac
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-fp32-leg --steps 40 $a > $O/f_b_${m}_$i.json 2> $O/f_b_${m}_$i.err || { echo bench $m failed; tail -5 $O/f_b_${m}_$i.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$O/f_b_${m}_$i.json')); print('$m', d['value'], d['timing_ms_per_step'], d['step_ms_distribution']['median'])" >> $O/f_ab.log
  done
done
cat $O/f_ab.log
