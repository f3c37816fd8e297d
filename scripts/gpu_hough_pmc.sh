# Hough microbench + kernel trace + SQ counters (separate passes), each GPU step time-limited
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
timeout -k 10 120 python scripts/hough_bench.py > gpurun_out/hough_bench.log 2>&1 &&
timeout -k 10 120 python scripts/hough_bench.py --batch 1 --test >> gpurun_out/hough_bench.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/hough_kt -o run -- python3 $R/scripts/hough_bench.py --iters 10 > $R/gpurun_out/hough_kt.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --kernel-trace --output-format csv -d $R/gpurun_out/hough_sq1 -o run -- python3 $R/scripts/hough_bench.py --iters 3 > $R/gpurun_out/hough_sq1.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/hough_sq2 -o run -- python3 $R/scripts/hough_bench.py --iters 3 > $R/gpurun_out/hough_sq2.log 2>&1
echo "exit=$?"
