# GPU round: parity tests, smoke, benches, kernel-trace profile (each step time-limited, chained with &&)
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/t_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err &&
timeout -k 10 300 python bench.py --workload vote_roi --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/bench_vr.json 2> gpurun_out/bench_vr.err &&
cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-graph > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1
echo "exit=$?"
