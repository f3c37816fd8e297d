#!/bin/bash
# Round-4 GPU batch c: parity tests of this round's step changes (drop bits in
# the reduce, side_prep, the grid SegICP score), then the A/Bs -- the 2-D
# blocked dW tile order (scratch/dwblk.so), the x6 fragment-read ablation
# (scratch/x6noread.so), post-vote work on the side stream vs the step's
# stream -- and the timings (estimatePose2D, ICP / score, the bench line with
# its no-dropout leg).  Stops at the first failure.
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_dropout.py tests/test_gpu_step.py tests/test_gpu_icp.py \
  tests/test_gpu_step_full.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $O/t_c.log 2>&1 || { echo "tests failed"; exit 1; }
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
: > $O/prep_ab.log
for i in 1 2 3; do
  for v in side main; do
    a=""; [ $v = main ] && a="--prep-on-main"
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-fp32-leg --steps 30 $a 2>/dev/null | \
      python -c "import json,sys; d=json.load(sys.stdin); print('$v', d['value'], d['timing_ms_per_step'])" \
      >> $O/prep_ab.log || exit 1
  done
done
timeout -k 10 300 python scripts/icp_bench.py > $O/icp_bench.json 2> $O/icp_bench.err || exit 1
timeout -k 10 300 python scripts/pose2d_bench.py > $O/pose2d_bench.json 2> $O/pose2d_bench.err || exit 1
timeout -k 10 600 python bench.py > $O/bench_full2.json 2> $O/bench_full2.err || exit 1
echo "exit=0"
