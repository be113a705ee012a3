"""Kernel stats from a rocprofv3 ``*_kernel_trace.csv`` restricted to the
steady state: everything after the last dispatch of a warm-up marker kernel
(default: MIOpen's naive conv, which only runs while MIOpen tunes at load).

  python tools/window_stats.py trace.csv [--after naive_conv] [--top 20]
"""

import argparse
import collections
import csv
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--after", default="naive_conv")
    ap.add_argument("--top", type=int, default=20)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    cut = max((i for i, r in enumerate(rows) if a.after and a.after in r["Kernel_Name"]), default=-1)
    rows = rows[cut + 1:]
    agg = collections.defaultdict(lambda: [0, 0])
    for r in rows:
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "", 1)
        n = re.sub(r"\(.*", "", n)
        if n.startswith("at::"):
            n = re.sub(r"<.*", "<...>", n)
        n = n[:90]
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        agg[n][0] += 1
        agg[n][1] += d
    tot = sum(v[1] for v in agg.values())
    span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) if rows else 0
    print("| kernel | calls | total ms | avg us | % |")
    print("|---|---:|---:|---:|---:|")
    for n, (c, d) in sorted(agg.items(), key=lambda kv: -kv[1][1])[: a.top]:
        print("| `%s` | %d | %.1f | %.1f | %.2f |" % (n, c, d / 1e6, d / c / 1e3, 100.0 * d / tot))
    print("\nsteady-state window: %d dispatches, %.1f ms kernel time, %.1f ms wall span (busy %.0f%%)"
          % (len(rows), tot / 1e6, span / 1e6, 100.0 * tot / max(span, 1)))


if __name__ == "__main__":
    main()
