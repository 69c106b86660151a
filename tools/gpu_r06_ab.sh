#!/bin/bash
# Round 6: the id plan's run heads computed inside the scan's input iterator (no flag kernel): the
# plan / dedup / DP-sparse / C3-at-size tests, then one graph step's kernel sequence.
cd "$(dirname "$0")/.."
out=gpurun_out/${1:-r06ab}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_inbatch_dedup.py tests/test_gpu_dp_sparse.py tests/test_gpu_c3_dedup_at_size.py \
    > $out/tests.log 2>&1
rc=$?; tail -n 1 $out/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_r06_w.sh ${1:-r06ab}/w || exit $?
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r06ab/w/trace/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
st = [i for i, r in enumerate(rows) if "ib_id_key_kernel" in r["Kernel_Name"]]
spans = [(int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3 for a, b in zip(st, st[1:])]
k = min(range(len(spans)), key=lambda i: spans[i])
a = st[k]
t0 = int(rows[a]["Start_Timestamp"])
for r in rows[a:a + 20]:
    print(f"{(int(r['Start_Timestamp']) - t0) / 1e3:8.1f} {(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3:7.1f} us  {r['Kernel_Name'][:80]}")
print("step span", spans[k])
PY
