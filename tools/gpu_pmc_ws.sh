#!/bin/bash
# PMC of the C3 tower layers (tools/microbench_towers.py, eager): per-dispatch FETCH_SIZE and
# WRITE_SIZE (KB) and the MFMA busy / clock pass, per GEMM kernel -> gpurun_out/TAG_pmc_ws.txt.
# Usage: tools/gpu_pmc_ws.sh TAG [lib.so] [kernel-name filter]
cd "$(dirname "$0")/.."
TAG=${1:-run}
LIB=${2:-recommendation-system-maang-nvidia-_amd/librecsys_hip.so}
FILT=${3:-gemm_}   # kernel-name filter
mkdir -p gpurun_out
export TMPDIR=/tmp EAGER=1 RECSYS_HIP_LIB=$LIB
d=gpurun_out/pmc_ws_$TAG
for ctr in FETCH_SIZE WRITE_SIZE "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES"; do
  tag=$(echo "$ctr" | tr ' ' '_')
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $ctr --output-format csv -d "$d/$tag" -o x -- \
      python3 tools/microbench_towers.py 65536 > "$d.$tag.log" 2>&1 || { echo "pass $ctr failed"; tail -5 "$d.$tag.log"; exit 1; }
done
for sub in $(ls $d); do
  f=$(find $d/$sub -name '*counter_collection.csv' | head -1)
  echo "== $sub"; python3 tools/pmc_summary.py $f $FILT
done > gpurun_out/${TAG}_pmc_ws.txt
f=$(find $d -name '*kernel_trace.csv' | head -1)
python3 tools/ktrace_avg.py $f $FILT >> gpurun_out/${TAG}_pmc_ws.txt
rm -rf $d $d.*.log
