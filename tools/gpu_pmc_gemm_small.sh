#!/bin/bash
# PMC counters (one per pass) of the c3 tower split GEMMs (microbench_gemm_prec.py, SHAPES=c3)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { echo "+ $*"; "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
CTRS=${CTRS:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES"}
for c in $CTRS; do
  SHAPES=c3 run timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d gpurun_out/pmc_gs_$c -o x -- \
      python3 tools/microbench_gemm_prec.py 6
done
for c in $CTRS; do
  f=$(find gpurun_out/pmc_gs_$c -name '*counter_collection.csv' | head -1); echo "== $c"; python tools/pmc_summary.py $f gemm_x3
done
t=$(find gpurun_out/pmc_gs_GRBM_GUI_ACTIVE -name '*kernel_trace.csv' | head -1); python tools/ktrace_avg.py $t gemm_x3
