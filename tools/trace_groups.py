#!/usr/bin/env python3
"""Split a rocprofv3 kernel trace at idle gaps (> 5 ms) and print, per group, the median
duration of each kernel name (the groups are the cases of tools/small_m_probe.py, in order)."""
import csv
import statistics
import sys

rows = []
for f in sys.argv[1:]:
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
groups, cur, last = [], [], None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if last is not None and s - last > 5_000_000:
        groups.append(cur)
        cur = []
    cur.append((r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0], (e - s) / 1000.0))
    last = e
groups.append(cur)
for i, g in enumerate(groups):
    names = {}
    for n, d in g:
        names.setdefault(n, []).append(d)
    print("group %d: " % i + ", ".join("%s x%d median %.1f us" % (n[:40], len(d), statistics.median(d))
                                        for n, d in names.items()))
