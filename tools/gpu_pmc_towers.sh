#!/bin/bash
# PMC of the C3 tower Dense-layer GEMMs (tools/microbench_towers.py: skinny forward / dX, split-K
# dW): SQ issue / wait counters in one pass, FETCH_SIZE and WRITE_SIZE in their own passes
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
i=0
for pass in "$P1" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $pass --output-format csv -d gpurun_out/pmc_tw_$i -o x -- \
      python3 tools/microbench_towers.py > gpurun_out/pmc_tw_$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
for i in 1 2 3; do
  f=$(find gpurun_out/pmc_tw_$i -name '*counter_collection.csv' | head -1)
  python3 tools/pmc_summary.py $f > gpurun_out/pmc_tw_$i.txt
done
t=$(find gpurun_out/pmc_tw_1 -name '*kernel_trace.csv' | head -1); python3 tools/ktrace_avg.py $t > gpurun_out/pmc_tw_trace.txt
rm -rf gpurun_out/pmc_tw_1 gpurun_out/pmc_tw_2 gpurun_out/pmc_tw_3
cat gpurun_out/pmc_tw_1.txt | head -80
