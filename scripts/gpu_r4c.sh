#!/bin/bash
# Round-4 GPU batch c: the 2-D blocked dW tile order (scratch/dwblk.so) A/B on
# the fc6 / fc7 weight gradients and the whole step, the estimatePose2D timing,
# and the bench line with its no-dropout leg.  Stops at the first failure.
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
O=gpurun_out; mkdir -p $O
: > $O/dwblk_ab.log
for i in 1 2; do
  for v in tree dwblk; do
    L=$PWD/posecnn_amd/libposecnn_hip.so; [ $v = tree ] || L=$PWD/scratch/$v.so
    echo "== $v" >> $O/dwblk_ab.log
    POSECNN_HIP_LIB=$L timeout -k 10 120 python scripts/gemm_bench.py --only fc6_dw,fc7_dw >> $O/dwblk_ab.log 2>&1 || exit 1
    POSECNN_HIP_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-fp32-leg --steps 30 2>/dev/null | \
      python -c "import json,sys; d=json.load(sys.stdin); print('step', d['value'], d['timing_ms_per_step'], d['gemm_us_in_step'].get('fc6_dw'))" \
      >> $O/dwblk_ab.log || exit 1
  done
done
: > $O/x6noread_ab.log
for i in 1 2; do
  for v in tree x6noread; do
    L=$PWD/posecnn_amd/libposecnn_hip.so; [ $v = tree ] || L=$PWD/scratch/$v.so
    echo "== $v" >> $O/x6noread_ab.log
    POSECNN_HIP_LIB=$L timeout -k 10 120 python scripts/gemm_bench.py --only fc6_fwd,fc6_dx,fc6_dw,fc7_fwd,fc7_dx >> $O/x6noread_ab.log 2>&1 || exit 1
  done
done
timeout -k 10 300 python scripts/pose2d_bench.py > $O/pose2d_bench.json 2> $O/pose2d_bench.err || exit 1
timeout -k 10 600 python bench.py > $O/bench_full2.json 2> $O/bench_full2.err || exit 1
echo "exit=0"
