#!/bin/bash
# Round 6: the id plan's bucket sort (ps_hist / ps_scatter / ps_bucket): the plan tests first
# (numpy-checked, incl. one-bucket cases), then the whole GPU suite, then one graph step's kernels.
cd "$(dirname "$0")/.."
out=gpurun_out/${1:-r06ac}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_gpu_inbatch_dedup.py > $out/tests_plan.log 2>&1
rc=$?; tail -n 1 $out/tests_plan.log; [ $rc -eq 0 ] || exit $rc
[ -n "$FULL" ] && { bash tools/gpu_suite.sh ${1:-r06ac}/s || exit $?; }
bash tools/gpu_r06_w.sh ${1:-r06ac}/w || exit $?
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r06ac/w/trace/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
st = [i for i, r in enumerate(rows) if "ib_id_key_kernel" in r["Kernel_Name"]]
spans = [(int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3 for a, b in zip(st, st[1:])]
k = min(range(len(spans)), key=lambda i: spans[i])
a = st[k]
t0 = int(rows[a]["Start_Timestamp"])
for r in rows[a:a + 12]:
    print(f"{(int(r['Start_Timestamp']) - t0) / 1e3:8.1f} {(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3:7.1f} us  {r['Kernel_Name'][:80]}")
print("step span", spans[k])
PY
