"""Mean dispatch duration per kernel from a rocprofv3 kernel_trace.csv.
Usage: python tools/ktrace_avg.py <kernel_trace.csv> [kernel-substring]"""
import csv
import sys
from collections import defaultdict

pat = sys.argv[2] if len(sys.argv) > 2 else ""
acc = defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if pat in r["Kernel_Name"]:
        acc[r["Kernel_Name"][:90]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, v in acc.items():
    print(f"  dur n={len(v)} mean={sum(v) / len(v) / 1e6:.3f} ms  {k}")
