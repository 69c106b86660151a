"""Per-launch HBM traffic from rocprofv3 --pmc CSVs of tools/traffic_probe.py: the counters of the
dispatches between the two iteration_increment_kernel markers, summed and divided by the
probe's launch count. traffic = 2 x FETCH_SIZE (gfx950 reports half the bytes of 16-B streaming
reads, MI355X_MICROARCH.md HBM section) + WRITE_SIZE, both in KB -> bytes.
Usage: python tools/traffic_summary.py <out.json> <name>=<dir>:<N> ...   (dir holds one subdirectory per pass)"""
import csv
import glob
import json
import sys
from collections import defaultdict


def between_markers(d, ctr):
    rows = []
    for f in sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)):
        rows = [r for r in csv.DictReader(open(f)) if r["Counter_Name"] == ctr]
        if rows:
            break
    if not rows:
        return None
    rows.sort(key=lambda r: int(r.get("Dispatch_Id") or r.get("Dispatch-Id") or 0))
    marks = [i for i, r in enumerate(rows) if "iteration_increment_kernel" in r["Kernel_Name"]]
    assert len(marks) >= 2, f"{d}/{ctr}: markers not found"
    sel = rows[marks[-2] + 1: marks[-1]]
    per = defaultdict(float)
    for r in sel:
        per[r["Kernel_Name"].split("(")[0].replace("void ", "")[:80]] += float(r["Counter_Value"])
    return sum(per.values()), dict(per)


out = {"method": "tools/traffic_probe.py under rocprofv3 --kernel-trace --pmc <one counter per pass>; the dispatches "
                 "between two marker kernels; traffic bytes per launch = (2 x FETCH_SIZE + WRITE_SIZE) KB x 1024 / N"}
for arg in sys.argv[2:]:
    name, rest = arg.split("=")
    d, n = rest.rsplit(":", 1)
    n = int(n)
    fe = between_markers(d, "FETCH_SIZE")
    wr = between_markers(d, "WRITE_SIZE")
    rec = {"launches": n}
    if fe and wr:
        rec.update(FETCH_SIZE_KB_per_launch=fe[0] / n, WRITE_SIZE_KB_per_launch=wr[0] / n,
                   traffic_bytes=int((2 * fe[0] + wr[0]) * 1024 / n),
                   kernels_fetch_KB={k: v / n for k, v in fe[1].items()},
                   kernels_write_KB={k: v / n for k, v in wr[1].items()})
    hit = between_markers(d, "TCC_HIT_sum")
    miss = between_markers(d, "TCC_MISS_sum")
    if hit and miss:
        rec["l2_hit_rate"] = hit[0] / max(hit[0] + miss[0], 1.0)
    out[name] = rec
    print(name, {k: v for k, v in rec.items() if not k.startswith("kernels")}, flush=True)
json.dump(out, open(sys.argv[1], "w"), indent=1)
