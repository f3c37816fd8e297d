# HBM traffic counters for the roofline `traffic` field: FETCH_SIZE and
# WRITE_SIZE in separate rocprofv3 passes (they do not fit one TCC pass),
# kernel-trace only beside them; eager launches so each kernel is a dispatch.
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_fetch -o run -- python3 $R/bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-graph > $R/gpurun_out/pmc_fetch.log 2>&1 &&
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_write -o run -- python3 $R/bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-graph > $R/gpurun_out/pmc_write.log 2>&1 &&
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_fetch_vr -o run -- python3 $R/bench.py --workload vote_roi --steps 20 --warmup 2 --no-cpu-baseline --no-graph > $R/gpurun_out/pmc_fetch_vr.log 2>&1 &&
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_write_vr -o run -- python3 $R/bench.py --workload vote_roi --steps 20 --warmup 2 --no-cpu-baseline --no-graph > $R/gpurun_out/pmc_write_vr.log 2>&1
echo "exit=$?"
