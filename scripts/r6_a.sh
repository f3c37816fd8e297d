#!/bin/bash
# round-6 call A: pipelined-step parity, then pipeline A/B of the bench, then an RCCL transport probe
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 700 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_step.py tests/test_gpu_step_full.py tests/test_gpu_icp.py tests/test_gpu_pose3d.py tests/test_gpu_hough.py \
  tests/test_gpu_dist.py -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > $O/a_tests.log 2>&1 || { echo tests failed; exit 1; }
for i in 1 2; do
  for m in off loss bwd start; do
    if [ $m = off ]; then a="--pipeline off"; else a="--pipeline on --prefetch-at $m"; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-fp32-leg --steps 30 $a > $O/a_b_${m}_$i.json 2> $O/a_b_${m}_$i.err || { echo bench $m failed; exit 1; }
    python -c "import json,sys; d=json.load(open('$O/a_b_${m}_$i.json')); print('$m', d['value'], d['timing_ms_per_step'], d['config']['roi_rows_rank0'], d['config'].get('roi_rows_minibatches_rank0'))" >> $O/a_ab.log
  done
done
cat $O/a_ab.log
timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 scripts/rccl_smoke.py > $O/a_rccl.log 2>&1; echo "rccl rc=$?" >> $O/a_rccl.log
tail -5 $O/a_rccl.log
echo done
