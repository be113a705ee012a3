#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel-trace database (rocpd SQLite, the ROCm 7
default output) as markdown: per-kernel totals over the whole run and the
breakdown of the last ``--window`` dispatches (e.g. one forward pass).

    python tools/rocpd_summary.py gpurun_out/prof/run_results.db --window 123 > profiles/x.md
"""

import argparse
import re
import sqlite3
from collections import OrderedDict


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"\s+\[clone [^\]]*\]", "", name)
    return name if len(name) < 110 else name[:107] + "..."


def table(rows, total):
    out = ["| kernel | calls | total us | avg us | % |", "|---|---:|---:|---:|---:|"]
    for name, (n, ns) in sorted(rows.items(), key=lambda kv: -kv[1][1]):
        out.append("| `%s` | %d | %.1f | %.2f | %.1f |" % (short(name), n, ns / 1e3, ns / 1e3 / n, 100.0 * ns / total))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--window", type=int, default=0, help="also break down the last N dispatches")
    ap.add_argument("--skip-last", type=int, default=0, help="ignore the final N dispatches (teardown)")
    ap.add_argument("--title", default="")
    args = ap.parse_args()
    c = sqlite3.connect(args.db)
    ks = list(c.execute("select name, start, end from kernels order by start"))
    if args.skip_last:
        ks = ks[:-args.skip_last]
    lines = ["# " + (args.title or "kernel trace: %s" % args.db), ""]
    agg = OrderedDict()
    for name, s, e in ks:
        n, ns = agg.get(name, (0, 0))
        agg[name] = (n + 1, ns + (e - s))
    total = sum(v[1] for v in agg.values())
    lines.append("whole run: %d dispatches, kernel time %.1f us" % (len(ks), total / 1e3))
    lines.append("")
    lines += table(agg, total)
    if args.window and len(ks) >= args.window:
        w = ks[-args.window:]
        span = w[-1][2] - w[0][1]
        busy = sum(e - s for _, s, e in w)
        lines += ["", "## last %d dispatches" % args.window, "",
                  "span %.1f us, kernel busy %.1f us (gaps %.1f us)" % (span / 1e3, busy / 1e3, (span - busy) / 1e3), ""]
        agg2 = OrderedDict()
        for name, s, e in w:
            n, ns = agg2.get(name, (0, 0))
            agg2[name] = (n + 1, ns + (e - s))
        lines += table(agg2, busy)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
