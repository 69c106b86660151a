#!/bin/bash
# Round-2 PMC passes on the two dominant kernels of the benched configs: the in-batch stored pair
# (C3, B = 65536, precision 6: inbatch_row_m16 / inbatch_col_m16) and the plane-pair GEMM (C5 shapes,
# B = 16384: xgemm_kernel). Per target three passes, each its own run: wave-cycle split +
# instruction mix + LDS conflicts; L2 hit / miss; MFMA busy + clock.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT"
P2="TCC_HIT_sum TCC_MISS_sum"
P3="SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVES"
declare -A CMD=( [ib]="tools/microbench_inbatch_prec.py 65536 6" [xg]="tools/microbench_xgemm.py 16384" )
declare -A PAT=( [ib]="inbatch_" [xg]="xgemm_kernel" )
for t in ${TARGETS:-ib xg}; do
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $P --output-format csv \
        -d gpurun_out/pmc_${t}_$i -o x -- python3 ${CMD[$t]} > gpurun_out/pmc_${t}_$i.log 2>&1 \
        || { echo "$t pass $i failed"; tail -5 gpurun_out/pmc_${t}_$i.log; exit 1; }
  done
  for i in 1 2 3; do
    f=$(find gpurun_out/pmc_${t}_$i -name '*counter_collection.csv' | head -1)
    echo "== $t pass $i"; python tools/pmc_summary.py $f ${PAT[$t]}
  done > gpurun_out/r02_pmc_$t.txt
  t3=$(find gpurun_out/pmc_${t}_3 -name '*kernel_trace.csv' | head -1)
  python tools/ktrace_avg.py $t3 ${PAT[$t]} >> gpurun_out/r02_pmc_$t.txt
  cat gpurun_out/r02_pmc_$t.txt
done
