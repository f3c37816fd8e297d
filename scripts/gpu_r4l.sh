#!/bin/bash
# Round-4 GPU batch i: the x6 A0-early read (scratch/x6a0.so) against
# the tree on the GEMM microbench and the whole step, alternating, same box.
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
O=gpurun_out; mkdir -p $O
: > $O/x6a0_ab.log
for i in 1 2 3; do
  for v in tree x6a0; do
    L=$PWD/posecnn_amd/libposecnn_hip.so; [ $v = tree ] || L=$PWD/scratch/$v.so
    echo "== $v" >> $O/x6a0_ab.log
    POSECNN_HIP_LIB=$L timeout -k 10 120 python scripts/gemm_bench.py >> $O/x6a0_ab.log 2>&1 || exit 1
    POSECNN_HIP_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-fp32-leg --steps 30 2>/dev/null | \
      python -c "import json,sys; d=json.load(sys.stdin); print('step', d['value'], d['timing_ms_per_step'])" \
      >> $O/x6a0_ab.log || exit 1
  done
done
echo "exit=0"
