#!/bin/bash
# MFMA utilisation evidence: SQ_VALU_MFMA_BUSY_CYCLES and GRBM_GUI_ACTIVE, one counter per pass,
# for the DCN-v2 cross stack (B = 65536) and the score-storing in-batch pair (B = 65536)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { echo "+ $*"; "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
for c in SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE; do
  run timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d gpurun_out/pmc_mf_dcn2_$c -o x -- \
      python3 tools/microbench_dcn2.py 65536 3344 4
  run timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d gpurun_out/pmc_mf_ib_$c -o x -- \
      python3 tools/microbench_inbatch.py 65536 128 stored
done
for t in dcn2 ib; do for c in SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE; do
  f=$(find gpurun_out/pmc_mf_${t}_$c -name '*counter_collection.csv' | head -1); echo "== $t $c"; python tools/pmc_summary.py $f rs::
done; done
