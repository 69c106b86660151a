"""One C3 step's kernels in launch order from a rocprofv3 kernel trace (csv): the launches between
the last two starts of the step's first kernel (ib_id_key_kernel), with durations and the gaps
between them. Usage: python tools/step_sequence.py <rocprof output dir> [marker]"""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
marker = sys.argv[2] if len(sys.argv) > 2 else "ib_id_key_kernel"
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
a, b = starts[-3], starts[-2]
t0 = int(rows[a]["Start_Timestamp"])
prev_end = None
busy = 0.0
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
    busy += (e - s) / 1e3
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} us  gap {gap:6.1f}  {r['Kernel_Name'][:100]}")
    prev_end = e
span = (int(rows[b]["Start_Timestamp"]) - t0) / 1e3
print(f"step span {span:.1f} us, kernels busy {busy:.1f} us, {b - a} launches")
