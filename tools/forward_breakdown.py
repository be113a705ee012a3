"""Per-kernel breakdown of ONE forward pass from a rocprofv3 kernel trace:
the dispatches between the last two `head_pool_kernel` launches (the last
forward of the run), grouped by kernel and in launch order.

  python tools/forward_breakdown.py trace.csv [--order]
"""

import argparse
import collections
import csv
import re


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "", 1)
    n = re.sub(r"\(.*", "", n)
    return re.sub(r"<.*", "<...>", n) if n.startswith("at::") else n[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--order", action="store_true", help="print every dispatch in order")
    ap.add_argument("--marker", default="head_pool_kernel")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.csv)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    if len(idx) < 2:
        raise SystemExit("need two %s dispatches" % a.marker)
    fwd = rows[idx[-2] + 1: idx[-1] + 1]
    t0, t1 = int(fwd[0]["Start_Timestamp"]), int(fwd[-1]["End_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in fwd)
    agg = collections.defaultdict(lambda: [0, 0])
    for r in fwd:
        k = short(r["Kernel_Name"])
        agg[k][0] += 1
        agg[k][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    print("one forward: %d dispatches, span %.1f us, kernel busy %.1f us (gaps %.1f us)" % (
        len(fwd), (t1 - t0) / 1e3, busy / 1e3, (t1 - t0 - busy) / 1e3))
    print("| kernel | calls | us | % |\n|---|---:|---:|---:|")
    for k, (n, ns) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print("| `%s` | %d | %.1f | %.1f |" % (k, n, ns / 1e3, 100.0 * ns / busy))
    if a.order:
        for r in fwd:
            print("%8.1f %-40s grid %s wg %s" % ((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3,
                                                short(r["Kernel_Name"]), r.get("Grid_Size", "?"),
                                                r.get("Workgroup_Size", "?")))


if __name__ == "__main__":
    main()
