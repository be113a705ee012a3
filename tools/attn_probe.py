"""Attention timing for the bert_large shape: torch SDPA under different
key-padding mask encodings (which fused kernel torch-ROCm picks depends on
it; the SDPA cases exclude the transpose copy the model needs after them) vs
K12 (csrc/kernels/bert.hip), which reads the fused QKV layout and writes
[tokens, hidden] directly.

  python tools/attn_probe.py --batch 64
"""

import argparse
import time

import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


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
    ap.add_argument("--k12-only", action="store_true")
    ap.add_argument("--seq", type=int, default=384)
    ap.add_argument("--pad", type=int, default=20, help="padded (masked) keys at the end of every sequence")
    a = ap.parse_args()
    b, s, h, d = a.batch, a.seq, 16, 64
    q, k, v = (torch.randn(b, h, s, d, device="cuda", dtype=torch.bfloat16) for _ in range(3))
    keep = torch.ones(b, s, device="cuda", dtype=torch.bool)
    if a.pad:
        keep[:, s - a.pad:] = False
    add = ((~keep)[:, None, None, :].to(torch.bfloat16) * -10000.0)
    cases = {
        "none": lambda: F.scaled_dot_product_attention(q, k, v),
        "additive_b11s": lambda: F.scaled_dot_product_attention(q, k, v, attn_mask=add),
        "bool_b11s": lambda: F.scaled_dot_product_attention(q, k, v, attn_mask=keep[:, None, None, :]),
        "additive_bhss": lambda: F.scaled_dot_product_attention(q, k, v, attn_mask=add.expand(b, h, s, s).contiguous()),
    }
    from triton_client_amd.ops import hip

    qkv = torch.randn(b * s, 3 * h * d, device="cuda", dtype=torch.bfloat16)
    out = torch.empty(b * s, h * d, device="cuda", dtype=torch.bfloat16)
    mask = keep.to(torch.int32)
    st = torch.cuda.current_stream().cuda_stream
    if a.k12_only:
        cases = {}
    cases["K12 none"] = lambda: hip.attention(qkv.data_ptr(), None, out.data_ptr(), b, s, h, 0.125, stream=st)
    cases["K12 masked"] = lambda: hip.attention(qkv.data_ptr(), mask.data_ptr(), out.data_ptr(), b, s, h, 0.125,
                                                stream=st)
    flops = 4 * b * h * s * s * d
    for name, fn in cases.items():
        us = timed(fn)
        print({"case": name, "us": round(us, 1), "tflops": round(flops / us / 1e6, 1)}, flush=True)


if __name__ == "__main__":
    main()
