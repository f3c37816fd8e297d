#!/bin/bash
# Round-4 GPU batch o: parity of the fc8 changes (1/keep in the 128-tile
# epilogue, split-K cap 32), then gemm microbench and whole-step A/B against
# the previous tree (scratch/prev.so).
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_dropout.py tests/test_gpu_step.py tests/test_gpu_step_full.py \
  tests/test_gpu_gemm_fc6.py tests/test_gpu_ops.py tests/test_gpu_dist.py -m gpu -x -v --timeout 300 \
  --timeout-method thread -p no:cacheprovider > $O/t_o.log 2>&1 || { echo "tests failed"; exit 1; }
: > $O/fc8_ab.log
for i in 1 2 3; do
  for v in tree prev; do
    L=$PWD/posecnn_amd/libposecnn_hip.so; [ $v = tree ] || L=$PWD/scratch/$v.so
    echo "== $v" >> $O/fc8_ab.log
    POSECNN_HIP_LIB=$L timeout -k 10 120 python scripts/gemm_bench.py --only fc8_fwd,fc8_dx,fc8_dw >> $O/fc8_ab.log 2>&1 || exit 1
    POSECNN_HIP_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-fp32-leg --steps 30 2>/dev/null | \
      python -c "import json,sys; d=json.load(sys.stdin); print('step', d['value'], d['timing_ms_per_step'])" \
      >> $O/fc8_ab.log || exit 1
  done
done
echo "exit=0"
