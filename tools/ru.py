"""Summarise hipcc -Rpass-analysis=kernel-resource-usage remarks: kernel, VGPRs, AGPRs, scratch, occupancy.
Usage: hipcc ... -Rpass-analysis=kernel-resource-usage 2>&1 | python tools/ru.py [name-filter]"""
import re
import sys

flt = sys.argv[1] if len(sys.argv) > 1 else ""
cur = None
rows = []
for line in sys.stdin:
    m = re.search(r"remark: Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)", line)
    if m and cur is not None:
        cur[m.group(1).split()[0]] = int(m.group(2))
for r in rows:
    if flt in r["name"]:
        print(f"V{r.get('VGPRs', 0):4d} A{r.get('AGPRs', 0):4d} scratch{r.get('ScratchSize', 0):6d} occ{r.get('Occupancy', 0)} "
              f"lds{r.get('LDS', 0):7d} {r['name'][:110]}")
