#!/usr/bin/env python3
"""One fp32 DenseNet forward from a rocprofv3 kernel trace (rocpd SQLite):
the dispatches between the last two head-pool launches, grouped into stem /
dense blocks / transitions / head, as a markdown table.

    python tools/fwd_blocks.py gpurun_out/prof_fwd64/*.db --title "bs64 forward"
"""
import argparse
import re
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--title", default="")
    a = ap.parse_args()
    ks = list(sqlite3.connect(a.db).execute("select name, start, end from kernels order by start"))
    idx = [i for i, k in enumerate(ks) if "head_pool" in k[0]]
    if len(idx) < 2:
        raise SystemExit("need two forwards in the trace")
    fwd = ks[idx[-2] + 1: idx[-1] + 1]
    parts, cur, blk = [], None, 1
    for name, s, e in fwd:
        n = re.sub(r"\(anonymous namespace\)::", "", name)
        if "stem" in n:
            key = "stem"
        elif "x3_conv1x1_kernel<true" in n:
            key = "transition %d" % blk
            blk += 1
        elif "head_pool" in n:
            key = "head"
        elif n.startswith("Cijk") or "gemm" in n.lower():
            key = "classifier"
        else:
            key = "block %d" % blk
        if cur is None or cur[0] != key:
            cur = [key, 0, 0.0, set()]
            parts.append(cur)
        cur[1] += 1
        cur[2] += (e - s) / 1e3
        cur[3].add(re.sub(r"\(.*", "", n.replace("void ", ""))[:48])
    span = (fwd[-1][2] - fwd[0][1]) / 1e3
    busy = sum(e - s for _, s, e in fwd) / 1e3
    print("# " + (a.title or "one forward"))
    print()
    print("%d dispatches, span %.1f us, kernel busy %.1f us." % (len(fwd), span, busy))
    print()
    print("| part | dispatches | us | % | kernels |")
    print("|---|---:|---:|---:|---|")
    for key, n, us, names in parts:
        print("| %s | %d | %.1f | %.1f | %s |" % (key, n, us, 100 * us / busy, ", ".join("`%s`" % x for x in sorted(names))))


if __name__ == "__main__":
    main()
