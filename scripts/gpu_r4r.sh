#!/bin/bash
# Round-4 GPU batch r: split-K reduce with eight slab loads in flight and a
# grid of one float4 per thread: GEMM / dropout / step parity, then the step
# and the nine-GEMM microbench against HEAD (scratch/redprev.so).
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_dropout.py tests/test_gpu_step.py tests/test_gpu_step_full.py \
  tests/test_gpu_gemm_fc6.py tests/test_gpu_ops.py tests/test_gpu_dist.py -m gpu -x -v --timeout 300 \
  --timeout-method thread -p no:cacheprovider > $O/t_r.log 2>&1 || { echo "tests failed"; exit 1; }
: > $O/reduce_ab.log
for i in 1 2; do
  for v in tree redprev; do
    L=$PWD/posecnn_amd/libposecnn_hip.so; [ $v = tree ] || L=$PWD/scratch/$v.so
    echo "== $v" >> $O/reduce_ab.log
    POSECNN_HIP_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-fp32-leg --steps 30 2>/dev/null | \
      python -c "import json,sys; d=json.load(sys.stdin); print('step', d['value'], d['timing_ms_per_step'])" \
      >> $O/reduce_ab.log || exit 1
  done
done
echo "exit=0"
