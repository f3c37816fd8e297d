#!/bin/bash
# Round-4 GPU batch: new parity tests, then (only if pytest ended normally,
# i.e. passed or failed without a crash / timeout) the bench line, the
# backprojection bench and the XCD-remap A/B.
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/test_gpu_dropout.py tests/test_gpu_pose2d.py tests/test_gpu_icp.py tests/test_gpu_step.py \
  tests/test_gpu_step_full.py tests/test_gpu_dist.py tests/test_gpu_dist_configs3.py \
  "tests/test_gpu_ops.py::test_backproject_linemod_config" tests/test_gpu_gemm_fc6.py -m gpu -v --timeout 600 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/t1.log 2>&1
rc=$?
echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench1.json 2> gpurun_out/bench1.err || exit 1
timeout -k 10 300 python scripts/bp_bench.py > gpurun_out/bp_bench.json 2>&1 || exit 1
timeout -k 10 300 python scripts/icp_bench.py > gpurun_out/icp_bench.json 2> gpurun_out/icp_bench.err || exit 1
bash scripts/gpu.sh microab gemm_bench oldxcd
