#!/bin/bash
# round-6 call G: validation (GPU suite, smoke, both bench lines, rocprofv3 + PMC) + the tail fork A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
: > $O/g_ab.log
for i in 1 2; do
  for m in start tail; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-fp32-leg --steps 40 --prefetch-at $m > $O/g_b_${m}_$i.json 2> $O/g_b_${m}_$i.err || { echo bench $m failed; tail -5 $O/g_b_${m}_$i.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$O/g_b_${m}_$i.json')); print('$m', d['value'], d['timing_ms_per_step'], d['step_ms_distribution']['median'])" >> $O/g_ab.log
  done
done
cat $O/g_ab.log
bash scripts/gpu.sh test smoke bench prof pmc || exit 1
tail -3 $O/t_gpu.log; cat $O/smoke.log | tail -2
python -c "import json; d=json.load(open('$O/bench_full.json')); print(d['value'], d['ms_per_step'], d['vs_baseline'], d['roofline']['frac'], d['cpu_baseline']['value'])"
echo done
