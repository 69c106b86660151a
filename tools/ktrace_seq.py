"""The last N topk launches of a rocprofv3 kernel trace in order (per-range scan / select times).
Usage: python tools/ktrace_seq.py <rocprof output dir>"""
import csv, sys, glob
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
seq = [(r["Kernel_Name"][:40], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3) for r in rows if "topk" in r["Kernel_Name"]]
# last call's 16 launches (8 ranges x scan+select)
tail = seq[-16:]
for n, d in tail: print(f"{d:9.1f} us  {n}")
print("sum", sum(d for _, d in tail))
