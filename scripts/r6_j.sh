#!/bin/bash
# round-6 call J: SQ counters of fc6 forward, dX and dW, each alone (scripts/gemm_bench.py --only)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R; export TMPDIR=/tmp
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM"
C2="SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE SQ_WAVES"
for s in fc6_fwd fc6_dx fc6_dw; do
  for p in 1 2; do
    C=$C1; [ $p = 2 ] && C=$C2
    (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/sqg_${s}_$p -o run -- \
       python3 $R/scripts/gemm_bench.py --only $s --iters 5 > $O/sqg_${s}_$p.log 2>&1) || exit 1
  done
done
for s in fc6_fwd fc6_dx fc6_dw; do
  echo "== $s"; python3 scripts/sq_summary.py $O/sqg_${s}_1 $O/sqg_${s}_2 --grep=k_gemm_x6
done > $O/sqg_summary.txt
cat $O/sqg_summary.txt
