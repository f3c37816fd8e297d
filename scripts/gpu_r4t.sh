#!/bin/bash
# Round-4 GPU batch t: the fc6 weight gradient on a stream of its own
# (PoseStep.w6_own_stream, bench --w6-stream) against the default, same tree.
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
O=gpurun_out; mkdir -p $O
: > $O/w6_stream_ab.log
for i in 1 2 3; do
  for v in default w6s; do
    F=""; [ $v = w6s ] && F=--w6-stream
    echo "== $v" >> $O/w6_stream_ab.log
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-fp32-leg --steps 30 $F 2>/dev/null | \
      python -c "import json,sys; d=json.load(sys.stdin); print('step', d['value'], d['timing_ms_per_step'], d['step_ms_distribution']['median'])" \
      >> $O/w6_stream_ab.log || exit 1
  done
done
echo "exit=0"
