"""Kernel statistics from a rocprofv3 rocpd database (run_results.db, the default output format of
rocprofv3 7.x): per kernel name total / count / average duration, sorted by total; also writes the
rows as CSV. Usage: python tools/rocpd_stats.py <run_results.db> <out.csv> [top-n]"""
import csv
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
name_col = "name" if "name" in cols else ("kernel_name" if "kernel_name" in cols else None)
if name_col is None:
    raise SystemExit(f"kernels view columns: {cols}")
rows = db.execute(f"select {name_col}, count(*), sum(end - start), avg(end - start) from kernels "
                  f"group by {name_col} order by sum(end - start) desc").fetchall()
tot = sum(r[2] for r in rows)
with open(sys.argv[2], "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
    for n, c, t, a in rows:
        w.writerow([n, c, t, a, 100.0 * t / tot])
for n, c, t, a in rows[: int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    print(f"{t / 1e6:9.2f} ms {100.0 * t / tot:6.2f}% calls={c:>5} avg={a / 1e3:10.1f}us  {n[:100]}")
print(f"total {tot / 1e6:.2f} ms")
