#!/bin/bash
# HBM-side traffic of the benched dominant kernels (round 2): one counter per pass (FETCH_SIZE,
# WRITE_SIZE), kernel-trace only; traffic = 2 x FETCH_SIZE (gfx950 halving of 16-B streaming reads,
# MI355X_MICROARCH.md HBM section) + WRITE_SIZE. C3 in-batch stored pair (B = 65536, precision 6)
# and the C5 cross stack kernels (B = 16384). Writes gpurun_out/r02_pmc_traffic.json.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $c --output-format csv -d gpurun_out/pmct_ib_$c -o x -- \
      python3 tools/microbench_inbatch_prec.py 65536 6 > gpurun_out/pmct_ib_$c.log 2>&1 || { echo "ib $c failed"; exit 1; }
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $c --output-format csv -d gpurun_out/pmct_xg_$c -o x -- \
      python3 tools/microbench_dcn2_planes.py 16384 > gpurun_out/pmct_xg_$c.log 2>&1 || { echo "xg $c failed"; exit 1; }
done
python3 - <<'PY'
import csv, glob, json
from collections import defaultdict
def per_kernel(tag, ctr):
    f = glob.glob(f"gpurun_out/pmct_{tag}_{ctr}/**/*counter_collection.csv", recursive=True)[0]
    acc = defaultdict(list)
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == ctr:
            acc[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}
out = {"method": "tools/gpu_pmc_traffic_r02.sh: rocprofv3 --kernel-trace --pmc <one counter> per pass; traffic bytes "
                 "= 2 x FETCH_SIZE (KB, gfx950 halving) + WRITE_SIZE (KB), x 1024; means per dispatch"}
for tag in ("ib", "xg"):
    fe, wr = per_kernel(tag, "FETCH_SIZE"), per_kernel(tag, "WRITE_SIZE")
    out[tag] = {k: {"FETCH_SIZE_KB": fe[k], "WRITE_SIZE_KB": wr.get(k, 0.0),
                    "traffic_bytes": int((2 * fe[k] + wr.get(k, 0.0)) * 1024)} for k in fe}
json.dump(out, open("gpurun_out/r02_pmc_traffic.json", "w"), indent=1)
for tag in ("ib", "xg"):
    for k, v in out[tag].items():
        if "inbatch" in k or "xgemm" in k or "ximg" in k:
            print(tag, k[:60], round(v["traffic_bytes"] / 1e9, 3), "GB")
PY
