#!/bin/bash
# PMC counters (one per pass) for the split-precision in-batch pair, precision 6, B = 65536
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { echo "+ $*"; "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
CTRS=${CTRS:-"SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU"}
for c in $CTRS; do
  run timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d gpurun_out/pmc_sp_$c -o x -- \
      python3 tools/microbench_inbatch_prec.py 65536 ${PRECS:-6}
done
for c in $CTRS; do
  f=$(find gpurun_out/pmc_sp_$c -name '*counter_collection.csv' | head -1); echo "== $c"; python tools/pmc_summary.py $f x3
  t=$(find gpurun_out/pmc_sp_$c -name '*kernel_trace.csv' | head -1); python tools/ktrace_avg.py $t x3
done
