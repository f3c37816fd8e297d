#!/bin/bash
# round-6 call E: ADD search ablations + SQ counters of k_add_search
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R; export TMPDIR=/tmp
: > $O/e_add.log
for v in tree noprune stageonly; do
  L=$R/posecnn_amd/libposecnn_hip.so; [ $v = tree ] || L=$R/scratch/$v.so
  echo "== $v" >> $O/e_add.log
  POSECNN_HIP_LIB=$L timeout -k 10 200 python scripts/add_bench.py --no-check --modes pruned,full >> $O/e_add.log 2>&1 || exit 1
done
cat $O/e_add.log
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU"
C2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_SMEM SQ_INSTS_BRANCH"
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $C1 --kernel-trace --output-format csv -d $O/e_sq1 -o run -- python3 $R/scripts/add_bench.py --iters 3 --modes pruned > $O/e_sq1.log 2>&1) || exit 1
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $C2 --kernel-trace --output-format csv -d $O/e_sq2 -o run -- python3 $R/scripts/add_bench.py --iters 3 --modes pruned > $O/e_sq2.log 2>&1) || exit 1
python scripts/sq_summary.py $O/e_sq1 $O/e_sq2 --grep=k_add
