# bench (full) three times on one MI355X: run-to-run spread
cd $GRAFT_REPO_ROOT
for i in 1 2 3; do
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_full_$i.json 2> gpurun_out/bench_full_$i.err || exit 1
done
echo "exit=0"
