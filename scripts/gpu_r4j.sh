#!/bin/bash
# Round-4 GPU batch j: the x6 GEMM on v_mfma_f32_16x16x32_bf16 with plane
# pairs concatenated along K (scratch/x6m16.so): its fp64 parity on the fc6 /
# fc7 shapes first, then GEMM microbench and whole-step A/B against the tree.
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
O=gpurun_out; mkdir -p $O
POSECNN_HIP_LIB=$PWD/scratch/x6m16.so timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm_fc6.py -m gpu -x -v \
  --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t_j.log 2>&1 || { echo "tests failed"; exit 1; }
: > $O/x6m16_ab.log
for i in 1 2 3; do
  for v in tree x6m16; do
    L=$PWD/posecnn_amd/libposecnn_hip.so; [ $v = tree ] || L=$PWD/scratch/$v.so
    echo "== $v" >> $O/x6m16_ab.log
    POSECNN_HIP_LIB=$L timeout -k 10 120 python scripts/gemm_bench.py >> $O/x6m16_ab.log 2>&1 || exit 1
    POSECNN_HIP_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-fp32-leg --steps 30 2>/dev/null | \
      python -c "import json,sys; d=json.load(sys.stdin); print('step', d['value'], d['timing_ms_per_step'])" \
      >> $O/x6m16_ab.log || exit 1
  done
done
echo "exit=0"
