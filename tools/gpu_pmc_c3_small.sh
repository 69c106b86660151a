#!/bin/bash
# PMC of C3's mid-sized step kernels (finalizes, sparse passes, DCN cross, heads, gather): SQ issue /
# wait counters in one pass, FETCH_SIZE and WRITE_SIZE in their own passes (eager steps)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
RE="finalize|sparse|dcn_cross|heads_|gather_tables|slab_reduce"
i=0
for pass in "$P1" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $pass --kernel-include-regex "$RE" --output-format csv \
      -d gpurun_out/pmc_c3s_$i -o x -- python3 bench.py --extras off --no-cpu-baseline --no-f32-compare --eager \
      --steps 3 --warmup 1 -o gpurun_out/pmc_c3s_$i.json > gpurun_out/pmc_c3s_$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc_c3s_$i.log; exit 1; }
done
for i in 1 2 3; do
  f=$(find gpurun_out/pmc_c3s_$i -name '*counter_collection.csv' | head -1)
  python3 tools/pmc_summary.py $f > gpurun_out/pmc_c3s_$i.txt
done
t=$(find gpurun_out/pmc_c3s_1 -name '*kernel_trace.csv' | head -1); python3 tools/ktrace_avg.py $t > gpurun_out/pmc_c3s_trace.txt
rm -rf gpurun_out/pmc_c3s_1 gpurun_out/pmc_c3s_2 gpurun_out/pmc_c3s_3
cat gpurun_out/pmc_c3s_trace.txt | cut -c1-140
cat gpurun_out/pmc_c3s_1.txt gpurun_out/pmc_c3s_2.txt gpurun_out/pmc_c3s_3.txt | cut -c1-140
