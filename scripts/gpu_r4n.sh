#!/bin/bash
# Round-4 GPU batch n: every FC GEMM on 128-row tiles (scratch/t128.so, two
# workgroups per CU, less split-K) against the tree's 256 / 128 choice.
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
O=gpurun_out; mkdir -p $O
: > $O/t128_ab.log
for i in 1 2; do
  for v in tree t128; do
    L=$PWD/posecnn_amd/libposecnn_hip.so; [ $v = tree ] || L=$PWD/scratch/$v.so
    echo "== $v" >> $O/t128_ab.log
    POSECNN_HIP_LIB=$L timeout -k 10 120 python scripts/gemm_bench.py >> $O/t128_ab.log 2>&1 || exit 1
  done
done
echo "exit=0"
