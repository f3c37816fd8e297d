# gemm_bench of each scratch/V.so (timing ablations: no parity)
cd $GRAFT_REPO_ROOT
: > gpurun_out/gemm_abl.log
for v in "$@"; do echo "== $v" >> gpurun_out/gemm_abl.log; POSECNN_HIP_LIB=$GRAFT_REPO_ROOT/scratch/$v.so timeout -k 10 300 python scripts/gemm_bench.py --only fc6_fwd,fc6_dw,fc6_dx,fc7_dw >> gpurun_out/gemm_abl.log 2>&1 || exit 1; done
echo "exit=0"
