#!/usr/bin/env python3
"""bf16 GEMM layout probe for the bert_large projections on hipBLASLt: the
same product y = x W^T + b with the weight stored [N][K] (nn.Linear, what
F.linear passes) vs pre-transposed [K][N], and addmm vs matmul + bias.

    python tools/gemm_layout_probe.py --m 24576
"""
import argparse
import time

import torch


def bench(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return 1e6 * (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=24576)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = "cuda"
    for name, k, n in [("qkv", 1024, 3072), ("out", 1024, 1024), ("ffn1", 1024, 4096), ("ffn2", 4096, 1024)]:
        x = torch.randn(a.m, k, device=dev, dtype=torch.bfloat16)
        w = torch.randn(n, k, device=dev, dtype=torch.bfloat16) * 0.02
        b = torch.randn(n, device=dev, dtype=torch.bfloat16)
        wt = w.t().contiguous()
        flop = 2.0 * a.m * k * n
        r = {}
        r["linear [N][K]"] = bench(lambda: torch.nn.functional.linear(x, w, b), a.iters)
        r["addmm [K][N]"] = bench(lambda: torch.addmm(b, x, wt), a.iters)
        r["mm [K][N]"] = bench(lambda: torch.mm(x, wt), a.iters)
        r["mm [N][K]^T"] = bench(lambda: torch.mm(x, w.t()), a.iters)
        if name == "ffn1":
            r["addmm_act gelu [N][K]^T"] = bench(lambda: torch._addmm_activation(b, x, w.t(), use_gelu=True), a.iters)
            r["addmm_act gelu [K][N]"] = bench(lambda: torch._addmm_activation(b, x, wt, use_gelu=True), a.iters)
        print("%s M=%d K=%d N=%d: %s" % (name, a.m, k, n, ", ".join("%s %.1f us (%.0f TF/s)" % (kk, v, flop / v / 1e6)
                                                                     for kk, v in r.items())), flush=True)


if __name__ == "__main__":
    main()
