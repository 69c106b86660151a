#!/bin/bash
# round 3 (session 2): bound-first top-k item loads -- non-temporal (default) vs plain, alternating
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
for v in "RS_TOPK_NT_LOADS=1" "RS_TOPK_PLAIN_DEFAULT=1"; do
  env $v GAUSS=1 PREC=6 timeout -k 10 200 python -u tools/microbench_topk.py 12500000 100 1024 \
      > gpurun_out/r03_nt_${v}_$i.log 2>&1 || exit $?
  echo "$v: $(grep 'Q= 1024' gpurun_out/r03_nt_${v}_$i.log)"
done
done
d=gpurun_out/pmc_c4nt
for c in FETCH_SIZE; do
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $d/$c -o x -- \
      python3 tools/traffic_probe.py c4 4 > $d.$c.log 2>&1 || { echo "pmc $c failed"; exit 1; }
done
python3 - <<'PY'
import glob, csv
f = glob.glob("gpurun_out/pmc_c4nt/FETCH_SIZE/**/*counter_collection.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if r["Counter_Name"] == "FETCH_SIZE" and "topk_thr" in r["Kernel_Name"]]
print("plain loads: topk_thr FETCH_SIZE KB per call (5 calls incl. warm-up):", sum(float(r["Counter_Value"]) for r in rows) / 5)
PY
