# GPU parity suite + smoke + one bench line
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
echo "exit=$?"
