#!/bin/bash
# One PMC pass of SQ wave-state / LDS counters over the tower layers' kernels
# (tools/microbench_towers.py, eager), summed per kernel -> gpurun_out/TAG_pmc_wgrad.txt.
# Usage: tools/gpu_pmc_wgrad.sh TAG [kernel-name filter]
cd "$(dirname "$0")/.."
TAG=${1:-run}; FILT=${2:-ws_kernel}
mkdir -p gpurun_out
export TMPDIR=/tmp EAGER=1
d=gpurun_out/pmc_wg_$TAG
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $d -o x -- \
    python3 tools/microbench_towers.py 65536 > $d.log 2>&1 || { echo "pmc pass failed"; tail -5 $d.log; exit 1; }
f=$(find $d -name '*counter_collection.csv' | head -1)
python3 tools/pmc_summary.py $f $FILT > gpurun_out/${TAG}_pmc_wgrad.txt
rm -rf $d $d.log
cat gpurun_out/${TAG}_pmc_wgrad.txt
