cd $GRAFT_REPO_ROOT
timeout -k 10 120 python scripts/gemm_bench.py --only fc6_fwd,fc6_dw,fc6_dx > gpurun_out/abl.log 2>&1 &&
for v in gload store gs; do echo "== $v" >> gpurun_out/abl.log; POSECNN_HIP_LIB=$GRAFT_REPO_ROOT/scratch/abl_$v.so timeout -k 10 120 python scripts/gemm_bench.py --only fc6_fwd,fc6_dw,fc6_dx >> gpurun_out/abl.log 2>&1 || exit 1; done
echo "exit=$?"
