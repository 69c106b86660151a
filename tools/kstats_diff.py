"""Per-kernel time difference (us per step) between two rocprofv3 kernel_stats.csv files.
Usage: python tools/kstats_diff.py A.csv B.csv steps [n]"""
import csv
import sys

def load(path):
    return {r["Name"][:90]: float(r["TotalDurationNs"]) for r in csv.DictReader(open(path))}

a, b = load(sys.argv[1]), load(sys.argv[2])
steps = float(sys.argv[3])
n = int(sys.argv[4]) if len(sys.argv) > 4 else 25
rows = [(k, a.get(k, 0.0) / steps / 1e3, b.get(k, 0.0) / steps / 1e3) for k in set(a) | set(b)]
rows.sort(key=lambda r: -abs(r[2] - r[1]))
for k, x, y in rows[:n]:
    print(f"{x:9.1f} {y:9.1f} {y - x:+9.1f} us/step  {k}")
print(f"total {sum(r[1] for r in rows):9.1f} {sum(r[2] for r in rows):9.1f}")
