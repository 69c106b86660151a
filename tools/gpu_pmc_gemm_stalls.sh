#!/bin/bash
# Where the split GEMM's wave cycles go on the c5 cross forward (B = 16384, precision 6): one pass of
# 8 SQ counters (wave cycles split into active / parked on waitcnt or barrier / issue-stalled,
# instruction mixes, LDS conflicts), one pass of L2 hit / miss, one of the MFMA busy cycles + clock.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT"
P2="TCC_HIT_sum TCC_MISS_sum"
P3="SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVES"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  SHAPES="${SHAPES:-c5 cross fwd}" timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P --output-format csv \
      -d gpurun_out/pmc_st_$i -o x -- python3 tools/microbench_gemm_prec.py ${PRECS:-6} > gpurun_out/pmc_st_$i.log 2>&1 \
      || { echo "pass $i failed"; tail -5 gpurun_out/pmc_st_$i.log; exit 1; }
done
for i in 1 2 3; do
  f=$(find gpurun_out/pmc_st_$i -name '*counter_collection.csv' | head -1); echo "== pass $i"; python tools/pmc_summary.py $f ${KPAT:-gemm_x3}
done
t=$(find gpurun_out/pmc_st_3 -name '*kernel_trace.csv' | head -1); python tools/ktrace_avg.py $t ${KPAT:-gemm_x3}
