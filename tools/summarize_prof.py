"""Summarise a rocprofv3 ``*_kernel_stats.csv`` into a short markdown table.

  python tools/summarize_prof.py gpurun_out/prof/server_kernel_stats.csv [--top 15]
"""

import argparse
import csv
import re


def short(name, n=90):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "", 1)
    name = re.sub(r"\(.*", "", name)
    if not name.startswith("at::"):  # keep our template args (tile variants), elide torch's
        name = name if len(name) <= n else name[: n - 3] + "..."
    else:
        name = re.sub(r"<.*", "<...>", name)
    return name if len(name) <= n else name[: n - 3] + "..."


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--top", type=int, default=15)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    tot = sum(int(r["TotalDurationNs"]) for r in rows)
    print("| kernel | calls | total ms | avg us | % |")
    print("|---|---:|---:|---:|---:|")
    for r in rows[: a.top]:
        print("| `%s` | %s | %.1f | %.1f | %s |" % (
            short(r["Name"]), r["Calls"], int(r["TotalDurationNs"]) / 1e6,
            float(r["AverageNs"]) / 1e3, r["Percentage"]))
    print("\nTotal GPU kernel time: %.1f ms over %d kernel names" % (tot / 1e6, len(rows)))


if __name__ == "__main__":
    main()
