# bench (full + vote_roi) twice each on one MI355X
cd $GRAFT_REPO_ROOT
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_full_$i.json 2> gpurun_out/bench_full_$i.err || exit 1
done
timeout -k 10 300 python bench.py --workload vote_roi --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/bench_vr.json 2> gpurun_out/bench_vr.err
echo "exit=$?"
