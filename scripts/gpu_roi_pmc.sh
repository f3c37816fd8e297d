# SQ counters for the RoI kernels (roi_bench.py), separate passes
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM --kernel-trace --output-format csv -d $R/gpurun_out/roi_sq1 -o run -- python3 $R/scripts/roi_bench.py --iters 3 > $R/gpurun_out/roi_sq1.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_IFETCH SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAVES --kernel-trace --output-format csv -d $R/gpurun_out/roi_sq2 -o run -- python3 $R/scripts/roi_bench.py --iters 3 > $R/gpurun_out/roi_sq2.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_BRANCH SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/roi_sq3 -o run -- python3 $R/scripts/roi_bench.py --iters 3 > $R/gpurun_out/roi_sq3.log 2>&1
echo "exit=$?"
