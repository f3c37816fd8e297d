#!/bin/bash
# One parameterised GPU runner (run through gpurun from the repo root):
#   gpurun --timeout 1200 -- bash scripts/gpu.sh TASK [TASK ...]
# Tasks run in order, each under its own time limit, and the script stops at
# the first failure (no retries).  Outputs land under gpurun_out/.
#   test [PYTEST_ARGS]  GPU parity suite (default: all of tests/ -m gpu)
#   smoke               __graft_entry__.smoke()
#   bench               default bench line (configs[2]) + vote_roi (configs[1])
#   prof                rocprofv3 --kernel-trace --stats of the eager and graph steps
#   pmc                 FETCH_SIZE / WRITE_SIZE / VALUBusy passes -> profiles/pmc_traffic.json
#   sq                  SQ instruction / stall counters of the eager step (two passes)
#   ab V1,V2,...        alternating bench of the tree vs scratch/V.so (scripts/build_variant.sh)
#   micro NAME          scripts/NAME.py microbench (gemm_bench, roi_bench, hough_bench, label_bench, pcie_rate)
#   microab NAME V1,... alternating scripts/NAME.py $MICRO_ARGS runs of the tree vs scratch/V.so (two rounds)
#   sqmicro NAME ARGS V1,...  the two SQ counter passes over scripts/NAME.py ARGS, tree and each scratch/V.so
#   bppmc               back-projection bench + FETCH / WRITE passes -> bp_bench_pmc.json (scripts/bp_pmc.py)
#   pose                estimatePose2D / 3D and solve_icp benches (tests/perf_*.py) + rocprofv3 kernel stats
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
prof() {  # prof NAME STEPS WARMUP [bench args] (eager launches, one dispatch per kernel)
  local n=$1 s=$2 w=$3; shift 3
  (cd /tmp && timeout -k 10 600 rocprofv3 "${PMC[@]}" --kernel-trace --output-format csv -d $O/$n -o run -- \
     python3 $R/bench.py --steps $s --warmup $w --no-cpu-baseline --no-fp32-leg "$@" > $O/$n.log 2>&1)
}
while [ $# -gt 0 ]; do
  task=$1; shift
  cd $R
  case $task in
    test)
      args=(tests)
      if [ $# -gt 0 ] && [[ $1 != test && $1 != smoke && $1 != bench && $1 != prof && $1 != pmc && $1 != sq && $1 != ab && $1 != micro && $1 != microab && $1 != sqmicro && $1 != bppmc && $1 != pose && $1 != dram ]]; then
        args=($1); shift
      fi
      timeout -k 10 900 python -u -m pytest "${args[@]}" -m gpu -x -v --timeout 120 --timeout-method thread \
        -p no:cacheprovider > $O/t_gpu.log 2>&1 || { echo "test failed"; exit 1; } ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1 ;;
    bench)
      timeout -k 10 600 python bench.py > $O/bench_full.json 2> $O/bench_full.err || exit 1
      timeout -k 10 300 python bench.py --workload vote_roi --steps 200 --warmup 20 \
        > $O/bench_vr.json 2> $O/bench_vr.err || exit 1 ;;
    prof)
      PMC=(--stats)
      prof prof 10 3 --no-graph || exit 1
      prof prof_graph 20 5 || exit 1 ;;
    pmc)
      PMC=(--pmc FETCH_SIZE); prof pmc_fetch 4 2 --no-graph || exit 1
      PMC=(--pmc WRITE_SIZE); prof pmc_write 4 2 --no-graph || exit 1
      PMC=(--pmc FETCH_SIZE); prof pmc_fetch_vr 20 2 --workload vote_roi --no-graph || exit 1
      PMC=(--pmc WRITE_SIZE); prof pmc_write_vr 20 2 --workload vote_roi --no-graph || exit 1
      PMC=(--pmc VALUBusy); prof pmc_valu 4 2 --no-graph || exit 1
      PMC=(--pmc VALUBusy); prof pmc_valu_vr 20 2 --workload vote_roi --no-graph || exit 1
      python scripts/pmc_traffic.py gpurun_out > $O/pmc_traffic.txt && cp profiles/pmc_traffic.json $O/ || exit 1 ;;
    dram)  # L2-miss reads split into MALL hits and HBM reads (the fc6 dW over-fetch question)
      PMC=(--pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_DRAM_sum); prof pmc_dram 4 2 --no-graph || exit 1
      python scripts/dram_split.py $O/pmc_dram > $O/dram_split.json || exit 1 ;;
    sq)
      PMC=(--pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM)
      prof sq1 2 1 --no-graph || exit 1
      PMC=(--pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE SQ_WAVES)
      prof sq2 2 1 --no-graph || exit 1 ;;
    ab)
      IFS=, read -ra vs <<< "$1"; shift
      : > $O/ab_lib.log
      for i in 1 2; do
        for v in tree "${vs[@]}"; do
          L=$R/posecnn_amd/libposecnn_hip.so; [ $v = tree ] || L=$R/scratch/$v.so
          POSECNN_HIP_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 2>/dev/null | \
            python -c "import json,sys; d=json.load(sys.stdin); print('$v', d['value'], d['timing_ms_per_step'])" \
            >> $O/ab_lib.log || exit 1
        done
      done ;;
    microab)
      n=$1; IFS=, read -ra vs <<< "$2"; shift 2
      : > $O/${n}_ab.log
      for i in 1 2; do
        for v in tree "${vs[@]}"; do
          L=$R/posecnn_amd/libposecnn_hip.so; [ $v = tree ] || L=$R/scratch/$v.so
          echo "== $v" >> $O/${n}_ab.log
          POSECNN_HIP_LIB=$L timeout -k 10 300 python scripts/$n.py $MICRO_ARGS >> $O/${n}_ab.log 2>&1 || exit 1
        done
      done ;;
    sqmicro)
      n=$1; margs=$2; IFS=, read -ra vs <<< "$3"; shift 3
      for v in tree "${vs[@]}"; do
        L=$R/posecnn_amd/libposecnn_hip.so; [ $v = tree ] || L=$R/scratch/$v.so
        for pass in 1 2; do
          if [ $pass = 1 ]; then C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM"
          else C="SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE SQ_WAVES"; fi
          (cd /tmp && POSECNN_HIP_LIB=$L timeout -s KILL 180 rocprofv3 --pmc $C --kernel-trace --output-format csv \
             -d $O/sq_${v}_$pass -o run -- python3 $R/scripts/$n.py $margs > $O/sq_${v}_$pass.log 2>&1) || exit 1
        done
      done ;;
    bppmc)  # back-projection bench + its rocprofv3 FETCH / WRITE passes per scene -> bp_bench_pmc.json
      timeout -k 10 300 python scripts/bp_bench.py > $O/bp_bench.json 2> $O/bp_bench.err || exit 1
      for sc in scene objects; do
        for c in FETCH_SIZE WRITE_SIZE; do
          n=fetch; [ $c = WRITE_SIZE ] && n=write
          (cd /tmp && timeout -s KILL 180 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/bp_${sc}_$n \
             -o run -- python3 $R/scripts/bp_bench.py --scene $sc --iters 5 > $O/bp_${sc}_$n.log 2>&1) || exit 1
        done
      done
      python scripts/bp_pmc.py $O $O/bp_bench.json > $O/bp_bench_pmc.json || exit 1 ;;
    pose)
      timeout -k 10 300 python tests/perf_pose.py --mode 2d > $O/pose2d_bench.json 2> $O/pose2d_bench.err || exit 1
      timeout -k 10 300 python tests/perf_pose.py --mode 3d > $O/pose3d_bench.json 2> $O/pose3d_bench.err || exit 1
      timeout -k 10 500 python tests/perf_icp.py > $O/icp_bench.json 2> $O/icp_bench.err || exit 1
      for m in 2d 3d; do
        (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_p$m -o run -- \
           python3 $R/tests/perf_pose.py --mode $m --no-cpu --iters 5 > $O/prof_p$m.log 2>&1) || exit 1
      done ;;
    micro)
      n=$1; shift
      timeout -k 10 300 python scripts/$n.py > $O/$n.log 2>&1 || exit 1 ;;
    *) echo "unknown task $task"; exit 2 ;;
  esac
done
echo "exit=0"
