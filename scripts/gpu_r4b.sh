#!/bin/bash
# Round-4 GPU batch b: the tiled-plane GEMM's parity tests, then its timing
# beside the staged x6 GEMMs (only if pytest ended without a crash / timeout).
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm_tp.py tests/test_gpu_pose2d.py tests/test_gpu_dist_configs3.py \
  -m gpu -v --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/t2.log 2>&1
rc=$?
echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python scripts/gemm_bench.py --precision 2,-1 > gpurun_out/gemm_tp_bench.log 2>&1
