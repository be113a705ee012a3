"""SDPA timing for the bert_large attention shape under different key-padding
mask encodings (which fused kernel torch-ROCm picks depends on it).

  python tools/attn_probe.py --batch 64
"""

import argparse
import time

import torch
import torch.nn.functional as F


def timed(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--seq", type=int, default=384)
    a = ap.parse_args()
    b, s, h, d = a.batch, a.seq, 16, 64
    q, k, v = (torch.randn(b, h, s, d, device="cuda", dtype=torch.bfloat16) for _ in range(3))
    keep = torch.ones(b, s, device="cuda", dtype=torch.bool)
    keep[:, s - 20:] = False
    add = ((~keep)[:, None, None, :].to(torch.bfloat16) * -10000.0)
    cases = {
        "none": lambda: F.scaled_dot_product_attention(q, k, v),
        "additive_b11s": lambda: F.scaled_dot_product_attention(q, k, v, attn_mask=add),
        "bool_b11s": lambda: F.scaled_dot_product_attention(q, k, v, attn_mask=keep[:, None, None, :]),
        "additive_bhss": lambda: F.scaled_dot_product_attention(q, k, v, attn_mask=add.expand(b, h, s, s).contiguous()),
    }
    flops = 4 * b * h * s * s * d
    for name, fn in cases.items():
        us = timed(fn)
        print({"case": name, "us": round(us, 1), "tflops": round(flops / us / 1e6, 1)}, flush=True)


if __name__ == "__main__":
    main()
