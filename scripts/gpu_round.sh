# Round artifacts on one MI355X: parity suite, smoke, PMC traffic passes ->
# profiles/pmc_traffic.json, bench (full + vote_roi) reading it, kernel-trace
# profile.  Every GPU step has its own time limit; steps are chained with &&.
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_fetch -o run -- python3 $R/bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-graph > $R/gpurun_out/pmc_fetch.log 2>&1 &&
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_write -o run -- python3 $R/bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-graph > $R/gpurun_out/pmc_write.log 2>&1 &&
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_fetch_vr -o run -- python3 $R/bench.py --workload vote_roi --steps 20 --warmup 2 --no-cpu-baseline --no-graph > $R/gpurun_out/pmc_fetch_vr.log 2>&1 &&
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_write_vr -o run -- python3 $R/bench.py --workload vote_roi --steps 20 --warmup 2 --no-cpu-baseline --no-graph > $R/gpurun_out/pmc_write_vr.log 2>&1 &&
cd $R && python scripts/pmc_traffic.py gpurun_out > gpurun_out/pmc_traffic.txt && cp profiles/pmc_traffic.json gpurun_out/pmc_traffic.json &&
timeout -k 10 600 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err &&
timeout -k 10 300 python bench.py --workload vote_roi --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/bench_vr.json 2> gpurun_out/bench_vr.err &&
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-graph > $R/gpurun_out/prof.log 2>&1 &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_graph -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/gpurun_out/prof_graph.log 2>&1
echo "exit=$?"
