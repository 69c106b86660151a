#!/bin/bash
# MFMA utilisation of the split-operand GEMMs of the DCN-v2 cross stack (precision 6):
# SQ_VALU_MFMA_BUSY_CYCLES and GRBM_GUI_ACTIVE, one counter per pass, at the c5 per-GPU batch
# (16384) and at B = 65536 (the north-star batch)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { echo "+ $*"; "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
for bb in 16384 65536; do
  for c in SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE; do
    SHAPES=c5 C5_BATCH=$bb run timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --output-format csv \
        -d gpurun_out/pmc_x3_${bb}_$c -o x -- python3 tools/microbench_gemm_prec.py 6
  done
done
for bb in 16384 65536; do
  for c in SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE; do
    f=$(find gpurun_out/pmc_x3_${bb}_$c -name '*counter_collection.csv' | head -1); echo "== B=$bb $c"; python tools/pmc_summary.py $f gemm_x3
  done
  t=$(find gpurun_out/pmc_x3_${bb}_GRBM_GUI_ACTIVE -name '*kernel_trace.csv' | head -1); python tools/ktrace_avg.py $t gemm_x3
done
