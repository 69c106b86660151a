"""Idle time of the GPU between kernels in a rocprofv3 kernel trace (csv): per step (split at the
largest gaps' kernel names is not needed: the total over the last N steps' window), the busy time,
the idle time and the largest gaps with the kernels on either side.
Usage: python tools/trace_gaps.py kernel_trace.csv [first_kernel_substring]"""
import csv
import sys

rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
# the timed window: from the first row kernel of the steps after warm-up to the end of the last one
mark = sys.argv[2] if len(sys.argv) > 2 else "inbatch_row_m16"
idx = [i for i, r in enumerate(rows) if mark in r[2]]
if len(idx) < 3:
    print("not enough steps"); sys.exit(0)
a, b = idx[len(idx) // 4], idx[-1]
win = rows[a:b]
busy = 0
end = win[0][0]
gaps = []
for s, e, n in win:
    if s > end:
        gaps.append((s - end, n))
    busy += max(0, e - max(s, end))
    end = max(end, e)
span = end - win[0][0]
steps = len([i for i in idx if a <= i < b])
print(f"window {span / 1e6:.3f} ms over {steps} steps: {span / steps / 1e3:.1f} us/step, busy {busy / steps / 1e3:.1f}, "
      f"idle {(span - busy) / steps / 1e3:.1f} us/step")
gaps.sort(reverse=True)
prev = {}
for i in range(1, len(win)):
    prev[win[i][2]] = win[i - 1][2]
for g, n in gaps[:25]:
    print(f"  gap {g / 1e3:8.1f} us before {n[:90]}")
