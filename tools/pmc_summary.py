"""Mean per-dispatch PMC counters per kernel from rocprofv3 --pmc CSV output.
Usage: python tools/pmc_summary.py <counter_collection.csv> [kernel-substring]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
pat = sys.argv[2] if len(sys.argv) > 2 else ""
acc = defaultdict(list)
for r in rows:
    name = r.get("Kernel_Name") or r.get("Kernel-Name") or ""
    if pat and pat not in name:
        continue
    acc[(name[:90], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (name, ctr), vals in sorted(acc.items()):
    print(f"{ctr:12s} n={len(vals):3d} mean={sum(vals) / len(vals):14.1f}  {name}")
