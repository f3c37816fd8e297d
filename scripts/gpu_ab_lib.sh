# bench (full) of the in-tree library vs each scratch/V.so, alternating, same box
cd $GRAFT_REPO_ROOT
: > gpurun_out/ab_lib.log
for i in 1 2; do
  for v in tree "$@"; do
    if [ $v = tree ]; then L=$GRAFT_REPO_ROOT/posecnn_amd/libposecnn_hip.so; else L=$GRAFT_REPO_ROOT/scratch/$v.so; fi
    POSECNN_HIP_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print('$v', d['value'], d['timing_ms_per_step'])" >> gpurun_out/ab_lib.log || exit 1
  done
done
echo "exit=0"
