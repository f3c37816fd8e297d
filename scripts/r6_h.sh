#!/bin/bash
# round-6 call H: ADD kernel geometry sweep (full scan) + the counter list (DRAM vs MALL traffic counters)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R; export TMPDIR=/tmp
: > $O/h_add.log
for v in tree ppl8 ppl2 grp4 grp16 blk16 grid1024 grid512 tree; do
  L=$R/posecnn_amd/libposecnn_hip.so; [ $v = tree ] || L=$R/scratch/$v.so
  echo "== $v" >> $O/h_add.log
  POSECNN_HIP_LIB=$L timeout -k 10 200 python scripts/add_bench.py --no-check --modes full,full --iters 30 2>&1 | grep -v amdgpu.ids >> $O/h_add.log || exit 1
done
cat $O/h_add.log
(cd /tmp && timeout -k 10 120 rocprofv3 -L > $O/h_counters.txt 2>&1) || echo "counter list failed"
grep -iE "TCC_EA0_RD|TCC_EA0_WR|DRAM|MALL|TCC_BUBBLE|TCC_HIT|TCC_MISS" $O/h_counters.txt | head -40
