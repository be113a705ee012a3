"""Summarise tools/gemm_probe.py logs: PF/s per (tokens, gemm) for each log."""
import collections
import json
import sys

for path in sys.argv[1:]:
    d = collections.defaultdict(list)
    for line in open(path):
        if line.startswith("{"):
            r = json.loads(line)
            d[(r["tokens"], r["gemm"])].append((r["variant"], r["k15_PFps"], r["hipblaslt_PFps"]))
    for k, x in d.items():
        print(path.split("/")[-1], k, " ".join("v%s %.3f/%.3f" % t for t in x))
