# bench of the tree vs scratch/prev (an older tree), alternating, same box
cd $GRAFT_REPO_ROOT
: > gpurun_out/ab_tree.log
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print('tree', d['value'], d['timing_ms_per_step'])" >> gpurun_out/ab_tree.log || exit 1
(cd scratch/prev && timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 2>/dev/null) | python -c "import json,sys; d=json.load(sys.stdin); print('prev', d['value'], d['timing_ms_per_step'])" >> gpurun_out/ab_tree.log || exit 1
done
echo "exit=0"
