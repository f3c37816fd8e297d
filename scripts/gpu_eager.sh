cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --no-graph --no-cpu-baseline > gpurun_out/bench_eager.json 2> gpurun_out/bench_eager.err
echo "exit=$?"
