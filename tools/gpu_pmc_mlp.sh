#!/bin/bash
# PMC of the one-launch Dense stack kernels (tools/microbench_mlp.py): SQ issue / wait counters and
# the instruction mix in two passes, kernel trace averages
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/microbench_mlp.py > gpurun_out/mb_mlp.log 2>&1 || exit $?
cat gpurun_out/mb_mlp.log
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_WAVES"
i=0
for pass in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $pass --output-format csv -d gpurun_out/pmc_mlp_$i -o x -- \
      python3 tools/microbench_mlp.py > gpurun_out/pmc_mlp_$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
for i in 1 2; do
  f=$(find gpurun_out/pmc_mlp_$i -name '*counter_collection.csv' | head -1)
  python3 tools/pmc_summary.py $f > gpurun_out/pmc_mlp_$i.txt
done
t=$(find gpurun_out/pmc_mlp_1 -name '*kernel_trace.csv' | head -1); python3 tools/ktrace_avg.py $t > gpurun_out/pmc_mlp_trace.txt
rm -rf gpurun_out/pmc_mlp_1 gpurun_out/pmc_mlp_2
grep -i mlp gpurun_out/pmc_mlp_trace.txt | cut -c1-160
grep -i -A12 mlp gpurun_out/pmc_mlp_1.txt | head -60
grep -i -A12 mlp gpurun_out/pmc_mlp_2.txt | head -60
