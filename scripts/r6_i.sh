#!/bin/bash
# round-6 call I: ADD geometry combinations + the DRAM / MALL split of the step's L2-miss reads
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R; export TMPDIR=/tmp
: > $O/i_add.log
for v in tree ppl2 grp4 p2g4 p2g4grid1024 g4grid1024 p2g2 tree; do
  L=$R/posecnn_amd/libposecnn_hip.so; [ $v = tree ] || L=$R/scratch/$v.so
  echo "== $v" >> $O/i_add.log
  POSECNN_HIP_LIB=$L timeout -k 10 200 python scripts/add_bench.py --no-check --modes full,full --iters 30 2>&1 | grep -v amdgpu.ids >> $O/i_add.log || exit 1
done
cat $O/i_add.log
bash scripts/gpu.sh dram || exit 1
cat $O/dram_split.json
