#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 --pmc passes (one or more dirs): the CSV
output, or the rocpd SQLite database (run_results.db, the ROCm 7 default)."""
import collections
import csv
import glob
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(d + "/**/*.db", recursive=True):
        import sqlite3

        per = collections.defaultdict(lambda: collections.defaultdict(float))
        db = sqlite3.connect(f)
        for k, disp, c, v in db.execute("select kernel_name, dispatch_id, counter_name, value from counters_collection"):
            per[(k, disp)][c] += float(v)
        for (k, _), cs in per.items():
            for c, v in cs.items():
                agg[k][c].append(v)
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(f)):
            per[(r["Kernel_Name"], r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
        for (k, _), cs in per.items():
            for c, v in cs.items():
                agg[k][c].append(v)
for k, cs in agg.items():
    name = k.replace("(anonymous namespace)::", "").split("(")[0]
    print("##", name)
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    for c in sorted(m):
        print("  %-28s %16.0f" % (c, m[c]))
    if "SQ_WAVE_CYCLES" in m and m["SQ_WAVE_CYCLES"]:
        w = m["SQ_WAVE_CYCLES"]
        print("  -> wait_any %.0f%%  wait_inst %.0f%%  active %.0f%%" % (
            100 * m.get("SQ_WAIT_ANY", 0) / w, 100 * m.get("SQ_WAIT_INST_ANY", 0) / w,
            100 * m.get("SQ_ACTIVE_INST_ANY", 0) / w))
    if "SQ_BUSY_CYCLES" in m and "SQ_VALU_MFMA_BUSY_CYCLES" in m and m["SQ_BUSY_CYCLES"]:
        # MFMA busy cycles are per SIMD summed over the chip; busy cycles per SE (x? ) -> report raw ratio
        print("  -> mfma_busy / busy = %.3f" % (m["SQ_VALU_MFMA_BUSY_CYCLES"] / m["SQ_BUSY_CYCLES"]))
    if "FETCH_SIZE" in m or "WRITE_SIZE" in m:
        # FETCH_SIZE / WRITE_SIZE are in KiB (L2 <-> memory traffic)
        print("  -> L2<->HBM fetch %.1f MB  write %.1f MB" % (m.get("FETCH_SIZE", 0) * 1024 / 1e6,
                                                          m.get("WRITE_SIZE", 0) * 1024 / 1e6))
    if m.get("TCC_HIT_sum", 0) + m.get("TCC_MISS_sum", 0):
        print("  -> L2 hit rate %.1f%%" % (100 * m["TCC_HIT_sum"] / (m["TCC_HIT_sum"] + m["TCC_MISS_sum"])))
