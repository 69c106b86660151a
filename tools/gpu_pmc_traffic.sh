#!/bin/bash
# PMC passes (one counter set per pass, kernel trace only): per-launch HBM traffic of the
# c4 top-k call, the c5 cross stack at B = 16384 and 65536, and the C3 gather (traffic + L2 hit
# rate, Zipf and uniform ids). Writes gpurun_out/${TAG}_pmc_traffic.json.
cd "$(dirname "$0")/.."
TAG=${1:-run}   # output prefix, e.g. r05
mkdir -p gpurun_out
export TMPDIR=/tmp
pass() {  # workload N dir counters...
  local w=$1 n=$2 d=$3; shift 3
  local tag=$(echo "$*" | tr ' ' '_')
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d "$d/$tag" -o x -- \
      python3 tools/traffic_probe.py "$w" "$n" > "$d.$tag.log" 2>&1 || { echo "pass $w $* failed"; exit 1; }
}
for spec in "c4:4" "c5:16384:3" "c5:65536:2" "gather:zipf:20" "gather:uniform:20"; do
  n=${spec##*:}; w=${spec%:*}
  d=gpurun_out/pmc_$(echo $w | tr ':' '_')
  pass "$w" "$n" "$d" FETCH_SIZE
  pass "$w" "$n" "$d" WRITE_SIZE
  case $w in gather*) pass "$w" "$n" "$d" TCC_HIT_sum TCC_MISS_sum ;; esac
  echo "$w done"
done
python3 tools/traffic_summary.py gpurun_out/${TAG}_pmc_traffic.json \
  c4=gpurun_out/pmc_c4:4 c5_b16384=gpurun_out/pmc_c5_16384:3 c5_b65536=gpurun_out/pmc_c5_65536:2 \
  gather_zipf=gpurun_out/pmc_gather_zipf:20 gather_uniform=gpurun_out/pmc_gather_uniform:20
