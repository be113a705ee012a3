#!/usr/bin/env python3
"""Dense-layer pair (K8x 1x1 -> K9x 3x3) over a bs128 56x56 (or 28x28) feature
map, run whole or in image chunks so the 1x1's z (hi|lo, 512 B per pixel) is
re-read by the 3x3 while it is still in the 256 MB Infinity Cache (MALL).

    python tools/x3_pair_bench.py --hw 56 --k 64 --chunks 128,64,32,16
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hw", type=int, default=56)
    ap.add_argument("--k", type=int, default=64)
    ap.add_argument("--ldx", type=int, default=256)
    ap.add_argument("--imgs", type=int, default=128)
    ap.add_argument("--chunks", default="128,64,32,16")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    import torch

    from triton_client_amd.ops import hip

    dev = "cuda"
    st = torch.cuda.current_stream().cuda_stream
    HW = a.hw * a.hw
    M = a.imgs * HW
    K = a.k

    def split(t):
        h = t.to(torch.bfloat16)
        return h.contiguous(), (t - h.float()).to(torch.bfloat16).contiguous()

    x = torch.randn(M, a.ldx, device=dev)
    s = torch.rand(K, device=dev) + 0.5
    t = torch.randn(K, device=dev) * 0.1
    w1h, w1l = split(torch.randn(128, K, device=dev) / K ** 0.5)
    b1 = torch.randn(128, device=dev)
    w3h, w3l = split(torch.randn(32, 9 * 128, device=dev) * 0.03)
    zh = torch.empty(M, 128, device=dev, dtype=torch.bfloat16)
    zl = torch.empty_like(zh)
    ws = torch.empty(64 << 20, device=dev, dtype=torch.uint8)
    for c in [int(v) for v in a.chunks.split(",")]:
        def run():
            for i0 in range(0, a.imgs, c):
                n = min(c, a.imgs - i0)
                r0 = i0 * HW
                m = n * HW
                wsb = hip.x3_conv1x1_ws_bytes(m, K)
                hip.x3_conv1x1(x.data_ptr() + r0 * a.ldx * 4, a.ldx, m, K, s.data_ptr(), t.data_ptr(), w1h.data_ptr(),
                               w1l.data_ptr(), out_bias=b1.data_ptr(), z_hi=zh.data_ptr() + r0 * 256,
                               z_lo=zl.data_ptr() + r0 * 256, ws=ws.data_ptr(), ws_bytes=min(wsb, ws.numel()),
                               stream=st)
                hip.x3_conv3x3(zh.data_ptr() + r0 * 256, zl.data_ptr() + r0 * 256, n, a.hw, a.hw, w3h.data_ptr(),
                               w3l.data_ptr(), x.data_ptr() + (r0 * a.ldx + K) * 4, a.ldx, stream=st)
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            run()
        torch.cuda.synchronize()
        us = 1e6 * (time.perf_counter() - t0) / a.iters
        print("hw=%d k=%d chunk=%d: %.1f us per %d images" % (a.hw, K, c, us, a.imgs), flush=True)


if __name__ == "__main__":
    main()
