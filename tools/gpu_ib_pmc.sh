#!/bin/bash
# PMC of in-batch variants (VARS="a b"; "cur" = the in-tree library): MFMA busy cycles, LDS bank
# conflicts, VALU instructions and GRBM_GUI_ACTIVE (effective clock) in one pass per variant
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in ${VARS}; do
  if [ $v = cur ]; then unset RECSYS_HIP_LIB; else export RECSYS_HIP_LIB=tools/_exp_inbatch_$v.so; fi
  echo "== $v"
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE \
      --output-format csv -d gpurun_out/pmc_ib_$v -o x -- python3 tools/microbench_inbatch_prec.py 65536 6 > gpurun_out/pmc_ib_$v.log 2>&1 || { tail -5 gpurun_out/pmc_ib_$v.log; exit 1; }
  f=$(find gpurun_out/pmc_ib_$v -name '*counter_collection.csv' | head -1); python tools/pmc_summary.py $f inbatch_row
  t=$(find gpurun_out/pmc_ib_$v -name '*kernel_trace.csv' | head -1); python tools/ktrace_avg.py $t inbatch_row
done
