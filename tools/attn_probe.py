"""Attention timing for the bert_large shape: torch SDPA under different
key-padding mask encodings (which fused kernel torch-ROCm picks depends on
it; the SDPA cases exclude the transpose copy the model needs after them) vs
K12 (csrc/kernels/bert.hip), which reads the fused QKV layout and writes
[tokens, hidden] directly.

  python tools/attn_probe.py --batch 64
  python tools/attn_probe.py --batch 64 --f32   # K12x (fp32-parity) vs torch fp32 SDPA
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
    ap.add_argument("--f32", action="store_true", help="the fp32-parity kernel (K12x) and fp32 SDPA")
    a = ap.parse_args()
    if a.f32:
        return f32_cases(a)
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


def f32_cases(a):
    from triton_client_amd.ops import hip

    b, s, h, d = a.batch, a.seq, 16, 64
    qkv = torch.randn(b * s, 3 * h * d, device="cuda")
    keep = torch.ones(b, s, device="cuda", dtype=torch.bool)
    if a.pad:
        keep[:, s - a.pad:] = False
    mask = keep.to(torch.int32)
    out = torch.empty(b * s, h * d, device="cuda")
    out3 = torch.empty(b * s, 3 * h * d, device="cuda", dtype=torch.bfloat16)
    st = torch.cuda.current_stream().cuda_stream
    q, k, v = qkv.view(b, s, 3, h, d).permute(2, 0, 3, 1, 4)
    add = ((~keep)[:, None, None, :].float() * -10000.0)
    cases = {
        "K12x masked": lambda: hip.attention_f32(qkv.data_ptr(), mask.data_ptr(), out.data_ptr(), b, s, h, 0.125,
                                                 stream=st),
        "K12x masked x3 out": lambda: hip.attention_f32(qkv.data_ptr(), mask.data_ptr(), out3.data_ptr(), b, s, h,
                                                        0.125, stream=st, x3=True),
        "sdpa fp32 additive": lambda: F.scaled_dot_product_attention(q, k, v, attn_mask=add),
    }
    flops = 4 * b * h * s * s * d
    for name, fn in cases.items():
        us = timed(fn)
        print({"case": name, "us": round(us, 1), "tflops": round(flops / us / 1e6, 1)}, flush=True)


if __name__ == "__main__":
    main()
