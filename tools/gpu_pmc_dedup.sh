#!/bin/bash
# PMC on the deduplicated in-batch pair at the C3 shape (tools/microbench_inbatch_dedup.py):
# per-launch HBM traffic between marker kernels (FETCH_SIZE / WRITE_SIZE passes), then the
# wave-cycle split + instruction mix and MFMA busy + clock passes. One counter set per pass.
cd "$(dirname "$0")/.."
TAG=${1:-run}   # output prefix, e.g. r05
mkdir -p gpurun_out
export TMPDIR=/tmp
pass() {  # dir counters...
  local d=$1; shift
  local tag=$(echo "$*" | tr ' ' '_')
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d "$d/$tag" -o x -- \
      python3 tools/microbench_inbatch_dedup.py 4 > "$d.$tag.log" 2>&1 || { echo "pass $* failed"; tail -5 "$d.$tag.log"; exit 1; }
}
d=gpurun_out/pmc_ibdedup4
pass $d FETCH_SIZE
pass $d WRITE_SIZE
pass $d SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT
pass $d SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVES
python3 tools/traffic_summary.py gpurun_out/${TAG}_pmc_ibdedup_traffic.json ib_dedup=$d:4
for sub in $(ls $d); do
  f=$(find $d/$sub -name '*counter_collection.csv' | head -1)
  echo "== $sub"; python3 tools/pmc_summary.py $f inbatch_
done > gpurun_out/${TAG}_pmc_ibdedup.txt
f=$(find $d -name '*kernel_trace.csv' | head -1)
python3 tools/ktrace_avg.py $f inbatch_ >> gpurun_out/${TAG}_pmc_ibdedup.txt
cat gpurun_out/${TAG}_pmc_ibdedup.txt | cut -c1-150
rm -rf gpurun_out/pmc_ibdedup4 gpurun_out/pmc_ibdedup4.*.log
